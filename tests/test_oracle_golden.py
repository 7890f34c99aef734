"""CPU: the oracle restatement pinned against the reference's golden vectors."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, assert_close


@pytest.fixture(scope="module")
def sd():
    from oracle import weights
    return weights.seeded_state_dict(0)


def test_seeded_weights_match_reference_checksum(sd):
    from oracle import weights
    gold = json.load(open(os.path.join(GOLDEN, "weights_checksum.json")))["checksum"]
    mine = weights.checksum(sd)
    assert sorted(mine) == sorted(gold)
    for k in gold:
        np.testing.assert_allclose(mine[k], gold[k], rtol=1e-12, err_msg=k)


def test_product_module_init_equals_oracle_weights(sd):
    """The drop-in Beluga reproduces the reference init under the same seed (state-dict keys too)."""
    import math
    import torch
    from expecto_amd import beluga
    m = beluga.seeded(0, gain=math.sqrt(6.0))
    msd = m.state_dict()
    assert list(msd) == list(sd)
    for k in sd:
        assert torch.equal(msd[k], sd[k]), k


def _forward_inputs():
    from oracle.encode_np import encode_seqs
    z = np.load(os.path.join(GOLDEN, "forward.npz"))
    seqs = [s.decode() for s in z["seqs"]]
    return encode_seqs(seqs).astype(np.float32), z["y"]


def test_oracle_torch_cpu_forward_matches_reference(sd):
    import torch
    from oracle.beluga_np import forward_torch_cpu
    x, y = _forward_inputs()
    got = forward_torch_cpu(sd, torch.from_numpy(x)).numpy()
    assert_close(got, y, rtol=1e-6, atol=1e-7, what="torch-CPU restatement")


def test_oracle_numpy_forward_matches_reference(sd):
    from oracle.beluga_np import forward_numpy
    x, y = _forward_inputs()
    got = forward_numpy({k: v.numpy() for k, v in sd.items()}, x[[0, 2, 3]])
    assert_close(got, y[[0, 2, 3]], what="numpy restatement")


def test_macs_per_window():
    from oracle.beluga_np import macs_per_window
    assert macs_per_window() == 3_901_588_246


def test_encoders_match_reference_golden():
    from oracle.encode_np import encode_seqs
    from expecto_amd.encode import encodeSeqs
    z = np.load(os.path.join(GOLDEN, "encode.npz"))
    seqs = [s.decode() for s in z["seqs"]]
    want = np.unpackbits(z["onehot"], axis=-1)[..., :2000].astype(bool)
    assert np.array_equal(encode_seqs(seqs), want)
    assert np.array_equal(encodeSeqs(seqs), want)


@pytest.mark.parametrize("bad", ["R", "*", "x", "1"])
def test_encoders_raise_keyerror_like_reference(bad):
    from oracle.encode_np import encode_seqs
    from expecto_amd.encode import encodeSeqs
    s = "A" * 999 + bad + "C" * 1000
    with pytest.raises(KeyError):
        encode_seqs([s])
    with pytest.raises(KeyError):
        encodeSeqs([s])


def test_encoder_short_and_long_crops():
    """Python-slice semantics of the crop for short / odd-length inputs (chromatin.py:164)."""
    from oracle.encode_np import encode_seqs
    from expecto_amd.encode import encodeSeqs
    rng = np.random.default_rng(0)
    for n in (1990, 1999, 2000, 2001, 2002, 2100, 2101, 2177):
        s = "".join(rng.choice(list("ACGTacgtN"), n))
        assert np.array_equal(encodeSeqs([s]), encode_seqs([s])), n


def test_tss_weights_and_reduce_oracle():
    from oracle.reduce_np import tss_pos_weights, tss_reduce
    from expecto_amd.features import tss_pos_weights as prod_w
    w = tss_pos_weights()
    assert w.shape == (10, 200) and w.dtype == np.float64
    assert np.array_equal(w, prod_w())
    rng = np.random.default_rng(1)
    f = rng.random((200, 2002), dtype=np.float32)
    r = rng.random((200, 2002), dtype=np.float32)
    out = tss_reduce(f, r)
    pred = (np.float32(0.5) * (f + r)).astype(np.float64)
    np.testing.assert_allclose(out, (w @ pred).flatten(), rtol=1e-12)


@pytest.mark.slow
def test_oracle_tss_features_match_reference(sd):
    """Full TSS tiling (2 genes x 400 windows) through the torch-CPU oracle vs the reference."""
    import torch
    from expecto_amd import synthetic
    from expecto_amd.genome import Fasta
    from oracle.beluga_np import forward_torch_cpu
    from oracle.encode_np import tss_window
    from oracle.reduce_np import TSS_SHIFTS, tss_reduce
    fa = Fasta.from_dict(synthetic.genome_bytes(n_contigs=3, contig_len=60000, seed=7))
    gold = np.load(os.path.join(GOLDEN, "tss.npz"))
    torch.set_num_threads(8)
    from expecto_amd.encode import seqs_to_codes, codes_to_onehot
    for gi, (chrom, tss, strand) in enumerate((("chr1", 30000, 1), ("chr2", 29123, -1))):
        seqs = [tss_window(fa, chrom, tss, strand, int(s)) for s in TSS_SHIFTS]
        x = codes_to_onehot(seqs_to_codes(seqs), with_rc=False).astype(np.float32)
        xt = torch.from_numpy(x).unsqueeze(2)
        fwd = forward_torch_cpu(sd, xt).numpy()
        rc = forward_torch_cpu(sd, torch.from_numpy(np.ascontiguousarray(x[:, ::-1, ::-1])).unsqueeze(2)).numpy()
        assert_close(tss_reduce(fwd, rc), gold["features"][gi], what=f"gene {gi}")
        if gi == 1:
            pr = np.float32(0.5) * (fwd + rc)
            assert_close(pr[::8], gold["rep_rows"], what="replicate rows")


def test_oracle_variant_reduce_matches_predict_py():
    from oracle.reduce_np import fwd_rc_average, variant_reduce, variant_weights
    gold = np.load(os.path.join(GOLDEN, "chromatin.npz"))
    feats = np.load(os.path.join(GOLDEN, "predict_features.npz"))
    rows = [r.split("\t") for r in feats["gene_rows"]]
    coor = [r.split("\t") for r in feats["coor_rows"]]
    vidx = [next(i for i, c in enumerate(coor) if c[0].replace("chr", "") == r[0] and c[1] == r[2]) for r in rows]
    shifts = [0, -200, 200]
    dist = -np.array([int(r[-1]) for r in rows])
    strand = np.array([r[-3] == "+" for r in rows])
    w = variant_weights(dist, strand, shifts)
    for name in ("diff", "ref", "alt"):
        eff = [fwd_rc_average(gold[f"{name}_{s}"])[vidx] for s in shifts]
        np.testing.assert_allclose(variant_reduce(eff, w), feats[name], rtol=1e-12, atol=0, err_msg=name)


def test_oracle_chromatin_windows_match_reference_outputs(sd):
    """fetchSeqs + encodeSeqs restated, through the torch-CPU oracle, reproduce the reference
    chromatin.py run (all shifts, SNVs, indels) -- pins the window geometry."""
    import torch
    from expecto_amd import synthetic
    from expecto_amd.genome import Fasta
    from oracle.beluga_np import forward_torch_cpu
    from oracle.encode_np import encode_seqs, fetch_seqs
    fa = Fasta.from_dict(synthetic.genome_bytes(n_contigs=3, contig_len=60000, seed=7))
    rows = [l.split("\t") for l in open(os.path.join(GOLDEN, "chromatin_vcf.txt")).read().splitlines()]
    rows = [r for r in rows if not r[0].startswith("chrUn")]
    gold = np.load(os.path.join(GOLDEN, "chromatin.npz"))
    torch.set_num_threads(8)
    for s in (0, -200, 200):
        refs, alts = [], []
        for r in rows:
            chrom = "chr" + r[0].replace("chr", "")
            a, b, _, _ = fetch_seqs(fa, chrom, int(r[1]), r[3], r[4], shift=s)
            refs.append(a)
            alts.append(b)
        xr = torch.from_numpy(encode_seqs(refs).astype(np.float32)).unsqueeze(2)
        xa = torch.from_numpy(encode_seqs(alts).astype(np.float32)).unsqueeze(2)
        yr = forward_torch_cpu(sd, xr).numpy()
        ya = forward_torch_cpu(sd, xa).numpy()
        assert_close(yr, gold[f"ref_{s}"], rtol=1e-6, atol=1e-7, what=f"ref {s}")
        assert_close(ya, gold[f"alt_{s}"], rtol=1e-6, atol=1e-7, what=f"alt {s}")
        assert_close(ya - yr, gold[f"diff_{s}"], rtol=1e-5, atol=1e-7, what=f"diff {s}")
