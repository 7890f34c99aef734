"""FC1 as a block-Karatsuba convolution (f16x3; beluga.hip "FC1 as a block-Karatsuba convolution",
Beluga.py:43-44): accuracy against a float64 forward in every role, the direct FC1 to the parity
bar, the segment path's windows equal to per-window forwards in their role bit for bit (including
the alt windows of segment pairs and windows whose group is incomplete), and the pair path's masked
in-place alt FC1 equal to full alt forwards."""
import math
import os

import numpy as np
import pytest
import torch

from conftest import assert_close, run_in_roles

pytestmark = pytest.mark.gpu


def _model(monkeypatch=None, env=None, max_batch=128):
    from expecto_amd import beluga
    for k, v in (env or {}).items():
        monkeypatch.setenv(k, v)
    m = beluga.seeded(0, gain=math.sqrt(6.0), max_batch=max_batch).cuda()
    m.engine()                       # the handle reads the environment when it is created
    for k in (env or {}):
        monkeypatch.delenv(k)
    return m


def _ratio(got, want):
    return float((np.abs(got.astype(np.float64) - want) / (1e-4 * np.abs(want) + 1e-5)).max())


def test_every_role_is_accurate_against_float64(monkeypatch):
    """16 windows (N runs included) in each of the 4 roles and with the direct FC1
    (EXPECTO_FC1_KARATSUBA=0): all inside half the parity bound of a float64 forward."""
    from expecto_amd.encode import codes_to_onehot
    from oracle.beluga_np import forward_torch_cpu
    rng = np.random.default_rng(31)
    codes_np = rng.integers(0, 4, (16, 2000)).astype(np.uint8)
    codes_np[2, 700:1300] = 4
    codes_np[9, ::41] = 4
    codes = torch.from_numpy(codes_np).cuda()
    m = _model()
    sd64 = {k: v.detach().double().cpu() for k, v in m.state_dict().items()}
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    y64 = forward_torch_cpu(sd64, torch.from_numpy(codes_to_onehot(codes_np).astype(np.float64)).unsqueeze(2)).numpy()
    eng = m.engine()
    ys = run_in_roles(eng, lambda: m.forward_codes(codes, 2))
    assert eng.f16_state()[0] == 0
    r = {role: _ratio(y.cpu().numpy(), y64) for role, y in ys.items()}
    md = _model(monkeypatch, {"EXPECTO_FC1_KARATSUBA": "0"})
    r["direct"] = _ratio(md.forward_codes(codes, 2).cpu().numpy(), y64)
    print("fraction of the parity bound vs float64:", r)
    assert max(r.values()) < 0.5, r
    assert not torch.equal(ys[0], ys[1])                 # the roles are different sums (same bar)


def test_segment_windows_equal_per_window_forwards_in_their_role():
    """forward_segments over 200-bp offsets (full groups of 4, a trailing incomplete group, both
    strands) and over scattered 4-aligned offsets: every window equals forward_codes of its own
    2000 codes in its role (pipeline.fc1_role) bit for bit."""
    from expecto_amd.pipeline import fc1_role
    rng = np.random.default_rng(32)
    m = _model(max_batch=256)
    eng = m.engine()
    for offs in (np.arange(0, 4601, 200), np.array([0, 4, 400, 404, 800, 1200, 1604, 2000, 2396, 3000], np.int64)):
        L = int(offs.max()) + 2000
        L += (-L) % 4
        ns = 3
        seg = torch.from_numpy(rng.integers(0, 5, (ns, L)).astype(np.uint8)).cuda()
        v_i, j_i = np.meshgrid(np.arange(ns), np.arange(offs.size), indexing="ij")
        win_seg, win_off = v_i.ravel().astype(np.int32), offs[j_i.ravel()].astype(np.int32)
        y = eng.forward_segments(seg, L, win_seg, win_off, None, 2).view(2, ns, offs.size, 2002)
        wins = torch.stack([seg[v, o:o + 2000] for v, o in zip(win_seg, win_off)]).contiguous()
        by_role = run_in_roles(eng, lambda: eng.forward_codes(wins, 2).view(2, ns, offs.size, 2002))
        for sd in range(2):
            for j, o in enumerate(offs):
                want = by_role[fc1_role(int(o), L, sd == 1)][sd, :, j]
                assert torch.equal(y[sd, :, j], want), (offs.tolist(), sd, int(o))


def test_pair_path_masked_alt_fc1_equals_full_forward_in_every_role():
    """forward_pairs' alt FC1 recomputes only the (product, slab, tail) partials the SNV's 20
    changed conv6 rows reach and keeps the ref partials for the rest: equal to full alt forwards,
    SNVs anywhere in the window, in each role."""
    m = _model()
    eng = m.engine()
    rng = np.random.default_rng(33)
    pos = np.array([0, 150, 400, 799, 800, 1000, 1199, 1200, 1600, 1999], np.int32)
    n = pos.size
    ref = torch.from_numpy(rng.integers(0, 4, (n, 2000)).astype(np.uint8)).cuda()
    alt = ref.clone()
    alt[torch.arange(n), torch.from_numpy(pos).long()] = (alt[torch.arange(n), torch.from_numpy(pos).long()] + 1) % 4
    for role in range(4):
        eng.set_fc1_role(role)
        y = torch.empty((2, 2, n, 2002), device="cuda")
        yv = y.view(4 * n, 2002)
        eng.forward_pairs(ref, alt, pos, yv[0:], yv[n:], 2 * n, 2)
        assert torch.equal(y[:, 0].reshape(2 * n, 2002), eng.forward_codes(ref, 2)), role
        assert torch.equal(y[:, 1].reshape(2 * n, 2002), eng.forward_codes(alt, 2)), role
    eng.set_fc1_role(4)


def test_headline_segment_pairs_equal_per_window_in_role():
    """The headline's path (200-window SNV sweeps, segment pairs, rows="variant"): 3 variants,
    every ref and alt window against forward_codes in its role."""
    from expecto_amd import synthetic
    from expecto_amd.genome import DeviceGenome, Fasta
    from expecto_amd.pipeline import VariantPipeline, VariantSet, fc1_role
    g = synthetic.genome_bytes(n_contigs=2, contig_len=120_000, seed=3)
    fa = Fasta.from_dict(g)
    dg = DeviceGenome(fa)
    snv = synthetic.snvs(g, 3, seed=4, margin=25_000)
    vs = VariantSet([s[0] for s in snv], np.array([s[1] for s in snv]), [s[2] for s in snv], [s[3] for s in snv])
    shifts = list(range(-20000, 20000, 200))
    m = _model(max_batch=1024)
    eng = m.engine()
    y = VariantPipeline(eng, fa, dg).predict(vs, shifts)             # [2, 2, S, 3, 2002]
    pw = VariantPipeline(eng, fa, dg, use_segments=False, use_pairs=False)
    by_role = run_in_roles(eng, lambda: pw.predict(vs, shifts))
    L = 2000 + shifts[-1] - shifts[0]
    for sd in range(2):
        for j, sh in enumerate(shifts):
            r = fc1_role(sh - shifts[0], L, sd == 1)
            assert torch.equal(y[sd, :, j], by_role[r][sd, :, j]), (sd, sh, r)
