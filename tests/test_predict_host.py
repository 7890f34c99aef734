"""CPU: expression-scoring host logic (predict.py drop-in) against the reference's outputs.

The golden TSVs come from running the reference predict.py (tests/golden/make_golden_predict.py)
on the reference chromatin.py outputs, with xgboost's gblinear restated in the stub."""
import os

import numpy as np
import pandas as pd
import pytest

from conftest import GOLDEN

PRED = os.path.join(GOLDEN, "predict_sed")
FEATURES_TSV = os.path.join(PRED, "deepsea_beluga_2002_features.tsv")


def test_legacy_model_reader_and_writer_roundtrip(tmp_path):
    from expecto_amd.xgblinear import GBLinear
    path = os.path.join(PRED, "all", "model.save")
    m = GBLinear.load(path)
    assert m.num_feature == 20020 and m.groups == 1
    assert m.base_score == 2.0 and np.float32(m.bias[0]) == np.float32(0.37)
    assert m.objective == "reg:linear"
    out = tmp_path / "m.save"
    m.save_legacy(str(out))
    assert open(out, "rb").read() == open(path, "rb").read()


def test_json_and_dump_readers_agree(tmp_path):
    import json
    from expecto_amd.xgblinear import GBLinear
    m = GBLinear.load(os.path.join(PRED, "notf", "model.save"))
    w = np.concatenate([m.weights[:, 0], m.bias])
    js = {"learner": {"gradient_booster": {"name": "gblinear", "model": {"weights": [float(x) for x in w]}},
                      "learner_model_param": {"base_score": "2E0", "num_feature": str(m.num_feature), "num_class": "0"},
                      "objective": {"name": "reg:squarederror"}}}
    (tmp_path / "m.json").write_text(json.dumps(js))
    mj = GBLinear.load(str(tmp_path / "m.json"))
    assert np.array_equal(mj.weights, m.weights) and np.array_equal(mj.bias, m.bias) and mj.base_score == 2.0
    dump = "bias:\n%r\nweight:\n" % float(m.bias[0]) + "".join("%r\n" % float(x) for x in m.weights[:, 0])
    (tmp_path / "m.dump").write_text(dump)
    with pytest.raises(ValueError):
        GBLinear.load(str(tmp_path / "m.dump"))
    md = GBLinear.load(str(tmp_path / "m.dump"), base_score=2.0)
    assert np.array_equal(md.weights, m.weights) and md.base_score == 2.0
    (tmp_path / "bad.save").write_bytes(b"binf" + b"\0" * 40)
    with pytest.raises(ValueError):
        GBLinear.load(str(tmp_path / "bad.save"))


def test_oracle_gblinear_reproduces_reference_predictions():
    """Oracle scoring of the feature matrices the reference predict.py built == its REF/ALT."""
    from expecto_amd.xgblinear import GBLinear
    from oracle import gblinear_np
    feats = np.load(os.path.join(GOLDEN, "predict_features.npz"))
    m = GBLinear.load(os.path.join(PRED, "all", "model.save"))
    sed = pd.read_csv(os.path.join(PRED, "all", "sed.tsv"), sep="\t", float_precision="round_trip")
    for k, col in (("ref", "REF"), ("alt", "ALT")):
        got = gblinear_np.predict(feats[k], m.weights[:, 0], m.bias[0], m.base_score)
        assert np.array_equal(got.astype(np.float64), sed[col].to_numpy()), k


def test_keep_mask_and_repeats_match_reference():
    from expecto_amd import predict
    df = pd.read_csv(FEATURES_TSV, sep="\t", index_col=0)
    m = predict.get_keep_mask(df, True, False, False, False, True)
    assert m.sum() == 1312
    assert predict.get_keep_mask(df, False, False, False, False, False).sum() == 2002
    genes = pd.DataFrame([[1, 5, 6, "A", "G", 0], [1, 5, 6, "A", "G", 1], [2, 7, 8, "C", "T", 2],
                          [1, 5, 6, "A", "G", 3]])
    assert predict.get_num_repeats(genes) == [2, 1, 1]
    assert predict.get_num_repeats(genes.iloc[:0]) == [0]


def test_consensus_fasta_and_natsort(tmp_path):
    from expecto_amd import consensus
    p = tmp_path / "x.fa"
    p.write_text(">chr1:-5-393210 extra words\nacgt\nNNAC\n>second\nGG\n")
    recs = list(consensus.parse_fasta(str(p)))
    assert recs == [("chr1:-5-393210", "acgtNNAC"), ("second", "GG")]
    s = consensus.normalize_consensus(*recs[0])
    assert len(s) == consensus.ENFORMER_SEQ_LENGTH and s.endswith("ACGTNNAC") and s[0] == "N"
    with pytest.raises(AssertionError):
        consensus.normalize_consensus("chr1:1-10", "ACGT")
    assert consensus.natsorted(["g10", "g2", "a", "g1"]) == ["a", "g1", "g2", "g10"]


def test_h5_scalar_and_string_datasets(tmp_path):
    from expecto_amd import h5
    f = str(tmp_path / "t.h5")
    h5.write(f, {"ref_preds": np.float32(1.25), "record_ids": np.array(["chr1:1-9|HG1", "x"], "S"),
                 "m": np.arange(6.0).reshape(2, 3)})
    r = h5.read(f)
    assert r["ref_preds"].shape == () and r["ref_preds"] == np.float32(1.25)
    assert list(r["record_ids"]) == [b"chr1:1-9|HG1", b"x"]
    assert np.array_equal(r["m"], np.arange(6.0).reshape(2, 3))


@pytest.mark.parametrize("rf", [False, True])
def test_closest_genes_match_reference(tmp_path, rf):
    """make_closest_genes_file.py drop-in (host logic) == the reference's files byte for byte."""
    import sys
    sys.path.insert(0, GOLDEN)
    import make_golden_extra as mg
    from expecto_amd import closest
    p = mg.write_inputs(str(tmp_path))
    out = tmp_path / "cg"
    closest.main([p["vcf"], "--geneanno_file", p["anno"], "-o", str(out)] + (["--all_in_receptive_field"] if rf else []))
    tag = "_rf" if rf else ""
    for name in ("closest_genes", "snps_hg19"):
        ext = "tsv" if name == "closest_genes" else "vcf"
        got = open(out / f"{name}.{ext}").read()
        assert got == open(os.path.join(GOLDEN, "extra", f"{name}{tag}.{ext}")).read(), name


def test_merge_geuvadis_consensus_matches_reference(tmp_path):
    """merge_geuvadis_predict_consensus.py (host only) on per-gene files holding the reference
    for_top_eqtls outputs (tests/golden/geuvadis_extra.npz): the merged record ids, genes and
    preds equal the reference merge's bit for bit; a sample mismatch between genes or a wrong
    gene count fails as the script's asserts do."""
    import os
    import numpy as np
    import pytest
    from conftest import GOLDEN
    from expecto_amd import consensus, h5
    gold = np.load(os.path.join(GOLDEN, "geuvadis_extra.npz"))
    genes = ['hla-b', 'hla-c', 'rpl28', 'cpamd8', 'tmem121b', 'scn11a']
    for gi, g in enumerate(genes):
        os.makedirs(tmp_path / "out" / g)
        h5.write(str(tmp_path / "out" / g / f"{g}.h5"), {"preds": gold[f"top_preds_{gi}"],
                                                         "record_ids": gold[f"top_ids_{gi}"],
                                                         "seqs": np.array([b"ACGT"], "S")})
    consensus.merge_main(["--batch_dir", str(tmp_path / "out"), "--n_genes", "6", "-o", str(tmp_path / "m")])
    r = h5.read(str(tmp_path / "m" / "expecto_preds.h5"))
    for k in ("record_ids", "genes", "preds"):
        assert r[k].dtype == gold[f"merge_{k}"].dtype and np.array_equal(r[k], gold[f"merge_{k}"]), k
    with pytest.raises(AssertionError):
        consensus.merge_main(["--batch_dir", str(tmp_path / "out"), "--n_genes", "5", "-o", str(tmp_path / "m2")])
    h5.write(str(tmp_path / "out" / "hla-b" / "hla-b.h5"), {"preds": gold["top_preds_0"],
                                                            "record_ids": np.array([b"chr6:1-2|NA1|+|x"], "S")})
    with pytest.raises(AssertionError):
        consensus.merge_main(["--batch_dir", str(tmp_path / "out"), "--n_genes", "6", "-o", str(tmp_path / "m3")])
