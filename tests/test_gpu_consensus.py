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


def _score_bound(m, x, pbar, weights, rows=None):
    """Bound on |score(ours) - score(reference)| for the gblinear score psum = f32(bias + base),
    psum = f32(psum + f32(f32(x_j) w_j)) over the 20030 features (xgboost 0.7 GBLinear::Pred),
    when our features x come from window predictions pbar [S, 2002] each within the parity bar
    1e-4|p| + 1e-5 of the reference's: feature (k, f) of the legacy layout may differ by
    dx = sum_s W[k,s] (1e-4 |pbar[s,f]| + 1e-5) (only over the windows `rows` that can differ;
    all by default), moving the exact sum by sum_j |w_j| dx_j; each side's float32 evaluation
    then deviates from its exact sum by at most (n+1) u max_j |psum_j| (one rounding of the
    product and one of the sum per feature, u = 2^-24)."""
    W = weights if rows is None else weights[:, rows]
    p = pbar if rows is None else pbar[rows]
    dx = W @ (1e-4 * np.abs(p) + 1e-5)                                 # [10, 2002]
    dx = np.concatenate([np.zeros((10, 1)), dx], 1).reshape(-1)        # legacy zero column per block
    w = m.weights[:, 0].astype(np.float64)
    psum = float(m.bias[0]) + float(m.base_score) + np.cumsum(w * x)
    return float(np.abs(w) @ dx + 2 * (x.size + 1) * 2.0 ** -24 * np.abs(psum).max())


def test_sed_for_top_eqtls_matches_reference(inputs):
    """The 200-shift SNV path (forward_segment_pairs) against geuvadis_sed_for_top_eqtls.py:
    per-window chromatin predictions of both alleles (the SNV's windows and every 8th window,
    captured from the reference Beluga forwards) at the parity bar, the 20030 features at the
    same bar, our scoring bit for bit equal to the restated GBLinear::Pred on our features, and
    the scores (and alt - ref) within the bound _score_bound derives from the parity bar and
    the float32 accumulation of the score sum."""
    from expecto_amd import consensus, h5
    from expecto_amd.features import tss_pos_weights
    from expecto_amd.xgblinear import GBLinear
    d, p, genes = inputs
    gold = np.load(os.path.join(GOLDEN, "consensus.npz"))
    out = d / "sed_out"
    cap = {}
    consensus.sed_main([p["model"], p["consensus"], p["genes_csv"], p["eqtls_csv"], "--synthetic-weights", "0",
                        "-o", str(out), "--seq-batch", "1"], capture=cap)
    y = {a: np.concatenate(cap[f"y_{a}"], axis=1) for a in ("ref", "alt")}     # [2, n, 200, 2002]
    x = {a: np.concatenate(cap[f"x_{a}"], axis=0) for a in ("ref", "alt")}     # [n, 20030]
    from oracle.gblinear_np import predict as gblinear_ref
    m = GBLinear.load(p["model"])
    weights = tss_pos_weights()
    for gi, (gene, *_) in enumerate(genes):
        win = {a: y[a][:, gi].reshape(400, 2002) for a in y}                     # rows: 200 fwd then 200 rc
        rows = gold[f"sed_win_rows_{gene}"]
        for a in ("ref", "alt"):
            assert_close(win[a][rows, ::5], gold[f"sed_win_{a}_{gene}"], what=f"{gene} {a} window predictions")
            np.testing.assert_allclose(win[a].astype(np.float64).sum(1), gold[f"sed_win_{a}sum_{gene}"], rtol=2e-6,
                                       atol=0, err_msg=f"{gene} {a} row sums")
            assert_close(x[a][gi, ::4], gold[f"sed_feat_{a}_{gene}"], what=f"{gene} {a} features")
        gd = gold[f"sed_win_alt_{gene}"].astype(np.float64) - gold[f"sed_win_ref_{gene}"]
        assert_close(win["alt"][rows, ::5].astype(np.float64) - win["ref"][rows, ::5], gd,
                     what=f"{gene} alt-ref window predictions")
        # windows without the SNV are bitwise the ref ones, as in the reference
        same = ~(gold[f"sed_win_alt_{gene}"] != gold[f"sed_win_ref_{gene}"]).any(1)
        assert (win["alt"][rows[same]] == win["ref"][rows[same]]).all()
        r = h5.read(str(out / gene / f"{gene}.h5"))
        assert r["ref_preds"].shape == () and r["ref_preds"].dtype == np.float32
        pbar = {a: (win[a][:200].astype(np.float64) + win[a][200:]) / 2 for a in win}
        b = {a: _score_bound(m, x[a][gi], pbar[a], weights) for a in ("ref", "alt")}
        for a in ("ref", "alt"):
            got, want = float(r[f"{a}_preds"]), float(gold[f"sed_{a}_{gene}"])
            # the scoring itself is exact: our score of our features == the restated GBLinear::Pred
            assert np.float32(got) == gblinear_ref(x[a][gi][None], m.weights[:, 0], m.bias[0], m.base_score)[0]
            assert abs(got - want) <= b[a], (gene, a, got, want, b[a])
        # alt - ref: only the windows holding the SNV can move the features apart
        snv = np.nonzero((win["alt"][:200] != win["ref"][:200]).any(1) | (win["alt"][200:] != win["ref"][200:]).any(1))[0]
        bd = _score_bound(m, x["alt"][gi], pbar["alt"], weights, snv) + _score_bound(m, x["ref"][gi], pbar["ref"],
                                                                                      weights, snv)
        got = float(r["alt_preds"]) - float(r["ref_preds"])
        want = float(gold[f"sed_alt_{gene}"]) - float(gold[f"sed_ref_{gene}"])
        assert abs(got - want) <= bd, (gene, "alt-ref", got, want, bd)
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
