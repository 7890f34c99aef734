"""Handle tuning knobs: the ones documented as "same bits either way" give the
default handle's outputs bit for bit on the 200-window segment-pair path; FC2 without split-K
(sigmoid fused into the GEMM epilogue) stays within the parity bar and keeps the segment path
bitwise equal to the per-window path."""
import math

import numpy as np
import pytest
import torch

from conftest import assert_close, sweep_in_roles

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


def _run(monkeypatch, env, fa, dg, vs, shifts, max_batch=2048, use_segments=True, use_pairs=True, roles=False):
    """roles: per-window runs with each window in the FC1 role the segment path gives it."""
    from expecto_amd import beluga
    from expecto_amd.pipeline import VariantPipeline
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    eng = beluga.seeded(0, gain=math.sqrt(6.0), max_batch=max_batch).cuda().engine()
    for k in env:
        monkeypatch.delenv(k)
    pipe = VariantPipeline(eng, fa, dg, use_segments=use_segments, use_pairs=use_pairs)
    y = sweep_in_roles(eng, lambda: pipe.predict(vs, shifts), shifts) if roles else pipe.predict(vs, shifts).clone()
    torch.cuda.synchronize()
    return y


@pytest.mark.parametrize("env", [{"EXPECTO_SEG_CHUNK_WINDOWS": "1000"}, {"EXPECTO_OVERLAP": "0"},
                                 {"EXPECTO_CONV_TILE": "256"}, {"EXPECTO_POOL_ONE_PASS": "0"},
                                 {"EXPECTO_FC_WIDE": "0"}, {"EXPECTO_FC_WIDE": "0", "EXPECTO_FC1_ORDER": "2"},
                                 {"EXPECTO_FC_WIDE": "0", "EXPECTO_FC1_ORDER": "0", "EXPECTO_FC1_M_ORDER_MB": "0"},
                                 {"EXPECTO_FC_WIDE": "0", "EXPECTO_FC1_M_GROUP": "3"},
                                 {"EXPECTO_FC1K_SLICE": "700"}, {"EXPECTO_FC1_NARROW": "1"},
                                 {"EXPECTO_CONV_NARROW": "1"}, {"EXPECTO_CONV_EA": "0"}, {"EXPECTO_POOL_FUSED": "0"}])
def test_same_bits_knobs(monkeypatch, env):
    fa, dg, vs, shifts = _setup()
    want = _run(monkeypatch, {}, fa, dg, vs, shifts)
    got = _run(monkeypatch, env, fa, dg, vs, shifts)
    assert torch.equal(got, want), f"{env}: max|diff| {float((got - want).abs().max())}"


def test_conv_early_reads_same_bits_with_fused_conv1(monkeypatch):
    """The conv consumers' early next-stage reads (EXPECTO_CONV_EA) on the MFMA conv2 with conv1 fused
    into its producers (EXPECTO_CONV2_TABLE=0, which itself changes conv2's sums): the same bits on
    and off."""
    fa, dg, vs, shifts = _setup()
    want = _run(monkeypatch, {"EXPECTO_CONV2_TABLE": "0"}, fa, dg, vs, shifts)
    got = _run(monkeypatch, {"EXPECTO_CONV2_TABLE": "0", "EXPECTO_CONV_EA": "0"}, fa, dg, vs, shifts)
    assert torch.equal(got, want), f"max|diff| {float((got - want).abs().max())}"


def test_tile_widths_small_batches(monkeypatch):
    """Per-window batches take narrower N tiles where they need fewer rounds of workgroups: the
    grouped FC1, the direct FC1 and FC2 112 instead of 336 columns (beluga.hip fc1_narrow; part-filled
    M tiles' empty waves skip their MFMAs), the direct FC1 and FC2 of <= 32 rows 32 x 48 tiles on a
    7-stage ring (fc_skinny, beluga_fc_h3s), conv3 / conv4 128 and conv5 / conv6 64 instead of 160
    (conv_narrow).  Batch 5 / 32 / 200 / 512 in FC1 roles 0, 3 and the direct FC1: the same bits as
    the wide tiles (EXPECTO_FC1_NARROW=0, EXPECTO_CONV_NARROW=0)."""
    from expecto_amd import beluga
    rng = np.random.default_rng(61)
    codes = torch.from_numpy(rng.integers(0, 5, (512, 2000)).astype(np.uint8)).cuda()
    engs = {}
    for v in ("0", "-1"):
        monkeypatch.setenv("EXPECTO_FC1_NARROW", v)
        monkeypatch.setenv("EXPECTO_CONV_NARROW", v)
        engs[v] = beluga.seeded(0, gain=math.sqrt(6.0), max_batch=512).cuda().engine()
        monkeypatch.delenv("EXPECTO_FC1_NARROW")
        monkeypatch.delenv("EXPECTO_CONV_NARROW")
    for role in (0, 3, 4):
        for b in (5, 32, 200, 512):
            ys = []
            for eng in engs.values():
                eng.set_fc1_role(role)
                ys.append(eng.forward_codes(codes[:b], 2).clone())
                eng.set_fc1_role(4)
            assert torch.equal(ys[0], ys[1]), (role, b, float((ys[0] - ys[1]).abs().max()))


def test_fc2_without_split_k(monkeypatch):
    fa, dg, vs, _ = _setup(n=9)
    shifts = [-800, -400, 0, 400, 800]
    base = _run(monkeypatch, {}, fa, dg, vs, shifts)
    seg = _run(monkeypatch, {"EXPECTO_FC2_SPLITS": "1"}, fa, dg, vs, shifts)
    per_window = _run(monkeypatch, {"EXPECTO_FC2_SPLITS": "1"}, fa, dg, vs, shifts, use_segments=False, roles=True)
    assert torch.equal(seg, per_window)
    assert_close(seg.cpu().numpy(), base.cpu().numpy(), what="FC2 split 1 vs split 7")


@pytest.mark.parametrize("use_segments,use_pairs", [(True, True), (False, True), (False, False)])
def test_fused_conv1_bitwise(monkeypatch, use_segments, use_pairs):
    """conv2 on the MFMAs (EXPECTO_CONV2_TABLE=0): conv1 inside the conv2 launch vs the separate
    conv1 launch give the same bits on the segment-pair path, the per-window path (forward_codes,
    fwd + rc) and the pair path (forward_pairs: ref conv2 fused, the alt conv2 patch computed from
    the alt codes)."""
    fa, dg, vs, _ = _setup(n=40)
    shifts = list(range(-20000, 20000, 200)) if use_segments else [-400, 0, 400]
    base = {"EXPECTO_CONV2_TABLE": "0"}
    fused = _run(monkeypatch, base, fa, dg, vs, shifts, use_segments=use_segments, use_pairs=use_pairs)
    sep = _run(monkeypatch, dict(base, EXPECTO_FUSE_CONV1="0"), fa, dg, vs, shifts, use_segments=use_segments,
               use_pairs=use_pairs)
    assert torch.equal(fused, sep), f"max|diff| {float((fused - sep).abs().max())}"


@pytest.mark.parametrize("use_segments,use_pairs", [(True, True), (False, True), (False, False)])
def test_conv2_table_paths_bitwise_and_parity(monkeypatch, use_segments, use_pairs):
    """conv1 + conv2 + pool1 from the k-mer table (default): the segment-pair, pair and per-window
    paths agree bit for bit with each other (every conv2 row is the same gather of its codes) and
    with conv2 on the MFMAs (EXPECTO_CONV2_TABLE=0) to the parity bar."""
    fa, dg, vs, _ = _setup(n=24)
    shifts = [-800, -400, 0, 400, 800]
    tab = _run(monkeypatch, {}, fa, dg, vs, shifts, use_segments=use_segments, use_pairs=use_pairs)
    ref = _run(monkeypatch, {}, fa, dg, vs, shifts, use_segments=False, use_pairs=False, roles=use_segments)
    assert torch.equal(tab, ref), f"max|diff| {float((tab - ref).abs().max())}"
    mfma = _run(monkeypatch, {"EXPECTO_CONV2_TABLE": "0"}, fa, dg, vs, shifts, use_segments=use_segments,
                use_pairs=use_pairs)
    assert_close(tab.cpu().numpy(), mfma.cpu().numpy(), what="conv2 k-mer table vs MFMA")


def test_conv2_table_accuracy_against_float64(monkeypatch):
    """Against a float64 forward, the k-mer tables' outputs (quad tables with the pair-table N
    fallback, and the pair tables alone) are at least as accurate as conv2 on the MFMAs (the
    tables are built in fp64 and rounded once; the MFMA path multiplies 22-bit operand splits),
    and inside the parity bound; N runs and scattered N bases (code 4) included."""
    import os
    from expecto_amd import beluga
    from expecto_amd.encode import codes_to_onehot
    from oracle.beluga_np import forward_torch_cpu
    rng = np.random.default_rng(21)
    codes_np = rng.integers(0, 4, (16, 2000)).astype(np.uint8)
    codes_np[3, 500:900] = 4
    codes_np[7, ::37] = 4
    codes = torch.from_numpy(codes_np).cuda()
    m = beluga.seeded(0, gain=math.sqrt(6.0), max_batch=64)
    sd64 = {k: v.detach().double() for k, v in m.state_dict().items()}
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    y64 = forward_torch_cpu(sd64, torch.from_numpy(codes_to_onehot(codes_np).astype(np.float64)).unsqueeze(2)).numpy()
    err = {}
    for name, env in (("quad", {}), ("pair", {"EXPECTO_KMER_QUAD": "0"}), ("mfma", {"EXPECTO_CONV2_TABLE": "0"})):
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        mm = beluga.seeded(0, gain=math.sqrt(6.0), max_batch=64).cuda()
        for k in env:
            monkeypatch.delenv(k)
        y = mm.forward_codes(codes, 2).cpu().numpy().astype(np.float64)
        assert mm.engine().f16_state()[0] == 0
        err[name] = float((np.abs(y - y64) / (1e-4 * np.abs(y64) + 1e-5)).max())
        del mm
    for name in ("quad", "pair"):   # quad tables, and the pair tables alone (the N fallback)
        assert err[name] < 0.5, err
        assert err[name] <= 1.25 * err["mfma"], err


def test_kmer_tables_are_shared_and_freed():
    """Handles with the same conv1 / conv2 weights share one set of k-mer tables (20.7 GB); the
    last handle to go frees them, so creating and dropping engines does not leak device memory."""
    import gc
    from expecto_amd import beluga
    table = (4 * 5 ** 9 + 2 * 4 ** 11) * 320 * 4
    gc.collect()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    free0 = torch.cuda.mem_get_info()[0]
    # a seed no other test uses, so no live handle elsewhere already holds these weights' tables
    a = beluga.seeded(4242, gain=math.sqrt(6.0), max_batch=64).cuda()
    ea = a.engine()
    free1 = torch.cuda.mem_get_info()[0]
    assert free0 - free1 >= table, (free0 - free1) / 1e9
    b = beluga.seeded(4242, gain=math.sqrt(6.0), max_batch=64).cuda()
    eb = b.engine()
    free2 = torch.cuda.mem_get_info()[0]
    assert free1 - free2 < table / 2, (free1 - free2) / 1e9          # b shares a's tables
    del ea, eb, a, b
    gc.collect()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    free3 = torch.cuda.mem_get_info()[0]
    assert free0 - free3 < 1 << 30, (free0 - free3) / 1e9            # all of it back
