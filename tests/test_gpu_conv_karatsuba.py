"""conv3 / conv4 as pair Karatsuba GEMMs (f16x3, opt-in EXPECTO_CONV_KARATSUBA=1; gemm_kernel.h
beluga_conv_h3k, Beluga.py:29-32):
accuracy against a float64 forward in both conv roles and with EXPECTO_CONV_KARATSUBA=0, the direct
role equal to the Karatsuba-off handle bit for bit, and the segment and segment-pair paths (their
even-row alt patches included) equal to per-window forwards in the pair role when every window
starts on an even pool1 row of both strands."""
import math

import numpy as np
import pytest
import torch

from conftest import run_in_roles

pytestmark = pytest.mark.gpu


def _model(monkeypatch, env=None, max_batch=128):
    """A seeded model whose handle runs the pair Karatsuba conv3 / conv4 (opt-in) unless env says
    otherwise; the handle reads the environment when it is created."""
    from expecto_amd import beluga
    env = {"EXPECTO_CONV_KARATSUBA": "1", **(env or {})}
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    m = beluga.seeded(0, gain=math.sqrt(6.0), max_batch=max_batch).cuda()
    m.engine()
    for k in env:
        monkeypatch.delenv(k)
    return m


def _ratio(got, want):
    return float((np.abs(got.astype(np.float64) - want) / (1e-4 * np.abs(want) + 1e-5)).max())


def test_both_roles_accurate_and_direct_role_equals_karatsuba_off(monkeypatch):
    """16 windows (N runs included): the pair role, the direct role and a Karatsuba-off handle all
    inside half the parity bound of a float64 forward; the direct role is the off handle's bits."""
    import os
    from expecto_amd.encode import codes_to_onehot
    from oracle.beluga_np import forward_torch_cpu
    rng = np.random.default_rng(41)
    codes_np = rng.integers(0, 4, (16, 2000)).astype(np.uint8)
    codes_np[3, 500:1100] = 4
    codes_np[11, ::37] = 4
    codes = torch.from_numpy(codes_np).cuda()
    m = _model(monkeypatch)
    sd64 = {k: v.detach().double().cpu() for k, v in m.state_dict().items()}
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    y64 = forward_torch_cpu(sd64, torch.from_numpy(codes_to_onehot(codes_np).astype(np.float64)).unsqueeze(2)).numpy()
    eng = m.engine()
    y_pair = m.forward_codes(codes, 2).clone()
    eng.set_conv_role(1)
    y_direct = m.forward_codes(codes, 2).clone()
    eng.set_conv_role(0)
    assert eng.f16_state()[0] == 0
    off = _model(monkeypatch, {"EXPECTO_CONV_KARATSUBA": "0"})
    y_off = off.forward_codes(codes, 2)
    r = {"pairs": _ratio(y_pair.cpu().numpy(), y64), "direct": _ratio(y_direct.cpu().numpy(), y64),
         "off": _ratio(y_off.cpu().numpy(), y64)}
    print("fraction of the parity bound vs float64:", r)
    assert max(r.values()) < 0.5, r
    assert torch.equal(y_direct, y_off)
    assert not torch.equal(y_pair, y_direct)


def test_segment_windows_on_even_rows_equal_per_window_pair_role(monkeypatch):
    """forward_segments over windows at 8-aligned offsets (even pool1 rows on both strands,
    scattered, so FC1 roles mix): every window equals forward_codes of its own codes in the pair
    conv role and its FC1 role, bit for bit."""
    from expecto_amd.pipeline import conv_role, fc1_role
    rng = np.random.default_rng(42)
    m = _model(monkeypatch, max_batch=256)
    eng = m.engine()
    offs = np.array([0, 8, 200, 408, 800, 1208, 1600, 2000, 2392, 3000], np.int64)
    L = int(offs.max()) + 2000
    L += (-L) % 8
    assert conv_role(offs, L) == 0
    ns = 3
    seg = torch.from_numpy(rng.integers(0, 5, (ns, L)).astype(np.uint8)).cuda()
    v_i, j_i = np.meshgrid(np.arange(ns), np.arange(offs.size), indexing="ij")
    win_seg, win_off = v_i.ravel().astype(np.int32), offs[j_i.ravel()].astype(np.int32)
    y = eng.forward_segments(seg, L, win_seg, win_off, None, 2).view(2, ns, offs.size, 2002)
    wins = torch.stack([seg[v, o:o + 2000] for v, o in zip(win_seg, win_off)]).contiguous()
    by_role = run_in_roles(eng, lambda: eng.forward_codes(wins, 2).view(2, ns, offs.size, 2002))
    for sd in range(2):
        for j, o in enumerate(offs):
            assert torch.equal(y[sd, :, j], by_role[fc1_role(int(o), L, sd == 1)][sd, :, j]), (sd, int(o))


@pytest.mark.parametrize("max_batch", [300, 40])
def test_segment_pairs_on_even_rows_alt_patches_bitwise(monkeypatch, max_batch):
    """forward_segment_pairs with every window on an even pool1 row (pair conv role): the alt runs'
    even-row conv3 / conv4 patches (SNVs at the segment edges, patch clamps at both ends, the middle)
    give exactly the full forwards of every ref and alt window, both strands."""
    from expecto_amd.pipeline import conv_role, fc1_role
    eng = _model(monkeypatch, max_batch=max_batch).engine()
    rng = np.random.default_rng(43)
    L = 2000 + 1600
    q = np.array([0, 3, 7, 30, 31, 500, 1234, 1799, 1800, 2001, 3000, L - 40, L - 9, L - 2, L - 1], np.int32)
    n = q.size
    ref = torch.from_numpy(rng.integers(0, 5, (n, L)).astype(np.uint8)).cuda()
    alt_code = torch.from_numpy(((ref.cpu().numpy()[np.arange(n), q] + 1 + rng.integers(0, 3, n)) % 4)
                                .astype(np.uint8)).cuda()
    alt = ref.clone()
    alt[torch.arange(n), torch.from_numpy(q).long()] = alt_code
    offs = np.array([0, 8, 200, 792, 800, 1000, 1592, 1600], np.int32)
    assert conv_role(offs, L) == 0
    S = offs.size
    v_i, j_i = np.meshgrid(np.arange(n), np.arange(S), indexing="ij")
    win_seg, win_off, win_row = v_i.ravel().astype(np.int32), offs[j_i.ravel()], (j_i * n + v_i).ravel().astype(np.int32)
    y = torch.full((2, 2, S * n, 2002), float("nan"), device="cuda")
    yf = y.view(4 * S * n, 2002)
    eng.forward_segment_pairs(ref, L, q, alt_code, win_seg, win_off, win_row, yf[0:], yf[S * n:], 2 * S * n)
    n_alt = int(sum(((o <= q) & (q < o + 2000)).sum() for o in offs))
    role = (lambda o, sd: 4) if 3 * n_alt > S * n else (lambda o, sd: fc1_role(int(o), L, sd == 1))
    for a, src in enumerate((ref, alt)):
        wins = torch.stack([src[:, o:o + 2000] for o in offs], 0).reshape(S * n, 2000).contiguous()
        by_role = run_in_roles(eng, lambda: eng.forward_codes(wins, 2).view(2, S, n, 2002))
        want = torch.stack([torch.stack([by_role[role(o, sd)][sd, j] for j, o in enumerate(offs)])
                            for sd in range(2)]).view(2, S * n, 2002)
        d = (y[:, a] - want).abs().amax(-1).view(2, S, n).cpu().numpy()
        assert (d == 0).all(), f"allele {a}: strand x offset x variant max|diff| {d}"
