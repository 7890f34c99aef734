"""Handle tuning knobs: the ones documented as "same bits either way" give the
default handle's outputs bit for bit on the 200-window segment-pair path; FC2 without split-K
(sigmoid fused into the GEMM epilogue) stays within the parity bar and keeps the segment path
bitwise equal to the per-window path."""
import math

import numpy as np
import pytest
import torch

from conftest import assert_close

pytestmark = pytest.mark.gpu

GENOME_ARGS = dict(n_contigs=3, contig_len=200_000, seed=17)


def _setup(n=12, shifts=None):
    from expecto_amd import synthetic
    from expecto_amd.genome import DeviceGenome, Fasta
    from expecto_amd.pipeline import VariantSet
    g = synthetic.genome_bytes(**GENOME_ARGS)
    fa = Fasta.from_dict(g)
    snv = synthetic.snvs(g, n, seed=5, margin=25_000)
    vs = VariantSet([s[0] for s in snv], np.array([s[1] for s in snv]), [s[2] for s in snv], [s[3] for s in snv])
    return fa, DeviceGenome(fa), vs, shifts or list(range(-20000, 20000, 200))


def _run(monkeypatch, env, fa, dg, vs, shifts, max_batch=2048, use_segments=True, use_pairs=True):
    from expecto_amd import beluga
    from expecto_amd.pipeline import VariantPipeline
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    eng = beluga.seeded(0, gain=math.sqrt(6.0), max_batch=max_batch).cuda().engine()
    for k in env:
        monkeypatch.delenv(k)
    pipe = VariantPipeline(eng, fa, dg, use_segments=use_segments, use_pairs=use_pairs)
    y = pipe.predict(vs, shifts).clone()
    torch.cuda.synchronize()
    return y


@pytest.mark.parametrize("env", [{"EXPECTO_SEG_CHUNK_WINDOWS": "1000"}, {"EXPECTO_OVERLAP": "0"},
                                 {"EXPECTO_CONV_TILE": "256"}, {"EXPECTO_POOL_ONE_PASS": "0"},
                                 {"EXPECTO_FUSE_CONV1": "0"},
                                 {"EXPECTO_FC_WIDE": "0"}, {"EXPECTO_FC_WIDE": "0", "EXPECTO_FC1_ORDER": "2"},
                                 {"EXPECTO_FC_WIDE": "0", "EXPECTO_FC1_ORDER": "0", "EXPECTO_FC1_M_ORDER_MB": "0"},
                                 {"EXPECTO_FC_WIDE": "0", "EXPECTO_FC1_M_GROUP": "3"}])
def test_same_bits_knobs(monkeypatch, env):
    fa, dg, vs, shifts = _setup()
    want = _run(monkeypatch, {}, fa, dg, vs, shifts)
    got = _run(monkeypatch, env, fa, dg, vs, shifts)
    assert torch.equal(got, want), f"{env}: max|diff| {float((got - want).abs().max())}"


def test_fc2_without_split_k(monkeypatch):
    fa, dg, vs, _ = _setup(n=9)
    shifts = [-800, -400, 0, 400, 800]
    base = _run(monkeypatch, {}, fa, dg, vs, shifts)
    seg = _run(monkeypatch, {"EXPECTO_FC2_SPLITS": "1"}, fa, dg, vs, shifts)
    per_window = _run(monkeypatch, {"EXPECTO_FC2_SPLITS": "1"}, fa, dg, vs, shifts, use_segments=False)
    assert torch.equal(seg, per_window)
    assert_close(seg.cpu().numpy(), base.cpu().numpy(), what="FC2 split 1 vs split 7")


@pytest.mark.parametrize("use_pairs", [True, False])
def test_fused_conv1_bitwise_on_window_paths(monkeypatch, use_pairs):
    """conv1 inside the conv2 launch (default) vs the separate conv1 launch: the per-window path
    (forward_codes, fwd + rc) and the pair path (forward_pairs: ref conv2 fused, the alt conv2
    patch computed from the alt codes) give the same bits."""
    fa, dg, vs, _ = _setup(n=40)
    shifts = [-400, 0, 400]
    fused = _run(monkeypatch, {}, fa, dg, vs, shifts, use_segments=False, use_pairs=use_pairs)
    sep = _run(monkeypatch, {"EXPECTO_FUSE_CONV1": "0"}, fa, dg, vs, shifts, use_segments=False,
               use_pairs=use_pairs)
    assert torch.equal(fused, sep), f"max|diff| {float((fused - sep).abs().max())}"
