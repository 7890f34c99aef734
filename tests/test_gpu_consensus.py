"""GPU: eQTL / personal-genome 200-shift scoring (expecto_amd.consensus) against the reference
geuvadis_sed_for_top_eqtls.py / geuvadis_predict_consensus.py outputs
(tests/golden/make_golden_consensus.py; same seeded inputs regenerated here)."""
import os
import sys

import numpy as np
import pytest

from conftest import GOLDEN, assert_close

pytestmark = pytest.mark.gpu
sys.path.insert(0, GOLDEN)


@pytest.fixture(scope="module")
def inputs(tmp_path_factory):
    import make_golden_consensus as mg
    d = tmp_path_factory.mktemp("cons")
    p = mg.write_inputs(str(d))
    assert open(p["model"], "rb").read() == open(os.path.join(GOLDEN, "consensus_model.save"), "rb").read()
    return d, p, mg.GENES


def _score_close(got, want, what):
    np.testing.assert_allclose(np.asarray(got, np.float64), np.asarray(want, np.float64), rtol=1e-5, atol=2e-3,
                               err_msg=what)


def test_sed_for_top_eqtls_matches_reference(inputs):
    from expecto_amd import consensus, h5
    d, p, genes = inputs
    gold = np.load(os.path.join(GOLDEN, "consensus.npz"))
    out = d / "sed_out"
    consensus.sed_main([p["model"], p["consensus"], p["genes_csv"], p["eqtls_csv"], "--synthetic-weights", "0",
                        "-o", str(out), "--seq-batch", "1"])
    for gene, *_ in genes:
        r = h5.read(str(out / gene / f"{gene}.h5"))
        assert r["ref_preds"].shape == () and r["ref_preds"].dtype == np.float32
        _score_close(r["ref_preds"], gold[f"sed_ref_{gene}"], f"{gene} ref")
        _score_close(r["alt_preds"], gold[f"sed_alt_{gene}"], f"{gene} alt")
        _score_close(r["alt_preds"] - r["ref_preds"], gold[f"sed_alt_{gene}"] - gold[f"sed_ref_{gene}"],
                     f"{gene} alt-ref")
    # the SNV 24 kb from the TSS lies outside every window: alt == ref exactly, like the reference
    r = h5.read(str(out / "geneb" / "geneb.h5"))
    assert r["ref_preds"] == r["alt_preds"]


def test_predict_consensus_matches_reference(inputs, capsys):
    from expecto_amd import consensus, h5
    d, p, genes = inputs
    gold = np.load(os.path.join(GOLDEN, "consensus.npz"))
    out = d / "cons_out"
    args = [p["model"], p["consensus"], p["genes_csv"], "--synthetic-weights", "0", "-o", str(out)]
    consensus.consensus_main(args)
    assert capsys.readouterr().out == open(os.path.join(GOLDEN, "consensus_stdout.txt")).read()
    for gene, *_ in genes:
        r = h5.read(str(out / gene / f"{gene}.h5"))
        c = h5.read(str(out / gene / f"{gene}_chromatin.h5"))
        ids = [x.decode() for x in r["record_ids"]]
        gids = [x.decode() for x in gold[f"cons_ids_{gene}"]]
        assert sorted(ids) == sorted(gids) and [x.decode() for x in c["record_ids"]] == ids
        order = [ids.index(g) for g in gids]            # glob order may differ between file systems
        _score_close(r["expecto_preds"][order], gold[f"cons_preds_{gene}"], f"{gene} expecto_preds")
        cp = c["chromatin_preds"][order]
        assert cp.dtype == np.float64 and cp.shape == tuple(gold[f"cons_chrom_shape_{gene}"])
        assert_close(cp[:, ::25, ::7], gold[f"cons_chrom_rows_{gene}"], what=f"{gene} chromatin preds")
        np.testing.assert_allclose(cp.sum(axis=(1, 2)), gold[f"cons_chrom_sum_{gene}"], rtol=1e-6)
    # second run: existing outputs are skipped
    consensus.consensus_main(args)
    assert capsys.readouterr().out.splitlines()[1:] == [f"Skipping gene {g} since h5 is already present."
                                                        for g, *_ in genes]
    # --exp_only: expression scores from the stored chromatin predictions
    first = {g: h5.read(str(out / g / f"{g}.h5"))["expecto_preds"] for g, *_ in genes}
    consensus.consensus_main(args + ["--exp_only", "--overwrite"])
    for g, *_ in genes:
        _score_close(h5.read(str(out / g / f"{g}.h5"))["expecto_preds"], first[g], f"{g} exp_only")
