"""GPU: the predict.py drop-in (expecto_amd.predict) and the gblinear scoring kernel against
the reference predict.py outputs (tests/golden/make_golden_predict.py) and the CPU oracle."""
import os

import numpy as np
import pandas as pd
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu
PRED = os.path.join(GOLDEN, "predict_sed")


@pytest.mark.parametrize("run", ["all", "notf"])
def test_gblinear_kernel_is_bitwise_equal_to_oracle(run):
    import torch
    from expecto_amd.xgblinear import GBLinear
    from oracle import gblinear_np
    feats = np.load(os.path.join(GOLDEN, "predict_features.npz"))
    m = GBLinear.load(os.path.join(PRED, run, "model.save"))
    df = pd.read_csv(os.path.join(PRED, "deepsea_beluga_2002_features.tsv"), sep="\t", index_col=0)
    keep = np.ones(len(df), bool)
    if run == "notf":
        keep &= (df["Assay type"] != "TF").to_numpy() & ~df["Assay"].str.startswith("Pol").to_numpy()
    cols = gblinear_np.keep_columns(keep)
    rng = np.random.default_rng(0)
    x = np.concatenate([feats["ref"], feats["alt"], rng.normal(0, 1, (150, 20020))])   # 164 rows: 3 blocks
    want = gblinear_np.predict(x[:, cols], m.weights[:, 0], m.bias[0], m.base_score)
    got = m.predict(torch.from_numpy(x).cuda(), torch.from_numpy(cols.astype(np.int32)).cuda()).cpu().numpy()
    assert np.array_equal(got, want)


def _write_h5(d):
    from expecto_amd import h5
    chrom = np.load(os.path.join(GOLDEN, "chromatin.npz"))
    feats = np.load(os.path.join(GOLDEN, "predict_features.npz"))
    os.makedirs(d / "out", exist_ok=True)
    for s in (0, -200, 200):
        h5.write(str(d / "out" / f"snps.shift_{s}.diff.h5"), {k: chrom[f"{k}_{s}"] for k in ("diff", "ref", "alt")})
    (d / "coor.vcf").write_text("##fileformat=VCFv4.3\n" + "".join(str(r) + "\n" for r in feats["coor_rows"]))
    (d / "genes.tsv").write_text("".join(str(r) + "\n" for r in feats["gene_rows"]))


@pytest.mark.parametrize("run,extra", [("all", ["--batchSize", "3"]), ("notf", ["--no_tf_features", "--no_pol2"])])
def test_predict_cli_matches_reference(tmp_path, capsys, run, extra):
    from expecto_amd import predict
    _write_h5(tmp_path)
    out = tmp_path / "pout"
    predict.main(["--model_save_file", os.path.join(PRED, run, "model.save"),
                  "--belugaFeatures", os.path.join(PRED, "deepsea_beluga_2002_features.tsv"),
                  "--coorFile_chromatin", str(tmp_path / "coor.vcf"), "--geneFile", str(tmp_path / "genes.tsv"),
                  "--snpEffectFilePattern", str(tmp_path / "out" / "snps.shift_SHIFT.diff.h5"),
                  "--maxshift", "200", "-o", str(out), *extra])
    assert capsys.readouterr().out == open(os.path.join(PRED, run, "stdout.txt")).read()
    for name in ("sed.tsv", "sed_sorted_by_magnitude.tsv", "sed_sorted_by_proportion.tsv"):
        got = pd.read_csv(out / name, sep="\t", float_precision="round_trip")
        want = pd.read_csv(os.path.join(PRED, run, name), sep="\t", float_precision="round_trip")
        assert list(got.columns) == list(want.columns), name
        if name != "sed.tsv":   # same rows; sorted by the key (ties may order either way)
            key = got.columns[-1]
            assert np.all(np.diff(got[key].to_numpy()) <= 0)
            got = got.sort_values("index").reset_index(drop=True)
            want = want.sort_values("index").reset_index(drop=True)
        num = ["REF", "ALT", "SED"] + [c for c in got.columns if c.startswith("SED_")]
        other = [c for c in got.columns if c not in num]
        assert got[other].astype(str).equals(want[other].astype(str)), name
        for c in num:
            np.testing.assert_allclose(got[c].to_numpy(), want[c].to_numpy(), rtol=1e-5, atol=1e-6, err_msg=c)
