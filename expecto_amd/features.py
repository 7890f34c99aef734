"""Spatial-feature reductions on the device (HBM-bound kernels of reduce.hip).

* ``tss_pos_weights`` + ``tss_reduce``: ``compute_expecto_features.py:88-124`` --
  ``F[g, k*2002+f] = sum_s W[k,s] * 0.5*(fwd[g,s,f] + rc[g,s,f])`` in float64.
* ``fwd_rc_average``: ``predict.py:186-190`` ``(x[:N] + x[N:]) / 2``.
* ``variant_features``: ``predict.py:87-136`` -- exp(-c*floor(|d|/200)) weights per shift,
  split by upstream/downstream, summed over shifts into ``[n, 10*2002]`` float64.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib

DECAY = (0.01, 0.02, 0.05, 0.1, 0.2)
TSS_SHIFTS = tuple(range(-20000, 20000, 200))     # compute_expecto_features.py:88


def tss_pos_weights(shifts=TSS_SHIFTS) -> np.ndarray:
    """10 x S float64 (compute_expecto_features.py:91-101)."""
    s = np.asarray(shifts)
    rows = [np.exp(-c * np.abs(s) / 200) * (s <= 0) for c in DECAY]
    rows += [np.exp(-c * np.abs(s) / 200) * (s >= 0) for c in DECAY]
    return np.vstack(rows)


def tss_reduce(fwd: torch.Tensor, rc: torch.Tensor, weights: torch.Tensor, out: torch.Tensor | None = None):
    """fwd, rc: [G, S, F] fp32 (device); weights [10, S] fp64 (device) -> [G, 10*F] fp64."""
    lib = _lib.load()
    G, S, F = fwd.shape
    if rc.shape != fwd.shape or weights.shape != (10, S):
        raise RuntimeError("tss_reduce: shape mismatch")
    fwd, rc, weights = fwd.contiguous(), rc.contiguous(), weights.contiguous()
    if out is None:
        out = torch.empty((G, 10 * F), dtype=torch.float64, device=fwd.device)
    _lib.check(lib.expecto_tss_reduce(_lib.dptr(fwd), _lib.dptr(rc), _lib.dptr(weights), G, S, F,
                                      _lib.dptr(out), _lib.stream_ptr()), "tss_reduce")
    return out


def fwd_rc_average(x: torch.Tensor, out: torch.Tensor | None = None):
    """[2N, F] fp32 -> [N, F]: (x[:N] + x[N:]) / 2 (predict.py:186)."""
    lib = _lib.load()
    x = x.contiguous()
    n = x.shape[0] // 2
    F = x.shape[1]
    if out is None:
        out = torch.empty((n, F), dtype=x.dtype, device=x.device)
    _lib.check(lib.expecto_fwd_rc_average(_lib.dptr(x), n, F, _lib.dptr(out), _lib.stream_ptr()), "fwd_rc_average")
    return out


def variant_features(effects: torch.Tensor, dist, strand_plus, shifts, out: torch.Tensor | None = None):
    """effects [S, n, F] fp32 (device, fwd/rc averaged, shift order), dist [n] (pos - TSS),
    strand_plus [n] bool -> [n, 10*F] fp64 (predict.py:87-124 layout: index k*F + f)."""
    return variant_reduce(effects, variant_tables(dist, strand_plus, shifts, effects.device), out)


def variant_tables(dist, strand_plus, shifts, device) -> tuple:
    """The per-batch inputs of ``variant_reduce`` on the device: dist [n] int64, strand [n] u8,
    shifts [S] int32 and the host exp table ``decay_table`` (numpy's exp, as the reference)."""
    d = torch.as_tensor(np.asarray(dist, np.int64), device=device)
    sp = torch.as_tensor(np.asarray(strand_plus, np.uint8), device=device)
    sh = torch.as_tensor(np.asarray(list(shifts), np.int32), device=device)
    lut = torch.from_numpy(decay_table(dist, strand_plus, shifts)).to(device)
    return d, sp, sh, lut


def variant_reduce(effects: torch.Tensor, tables: tuple, out: torch.Tensor | None = None):
    """``variant_features`` on tables already resident (``variant_tables``): one launch per
    65,535 variants (the grid's y limit)."""
    lib = _lib.load()
    S, n, F = effects.shape
    d, sp, sh, lut = tables
    if d.shape != (n,) or sp.shape != (n,) or sh.shape != (S,):
        raise RuntimeError("variant_reduce: table shapes do not match the effects")
    effects = effects.contiguous()
    if out is None:
        out = torch.empty((n, 10 * F), dtype=torch.float64, device=effects.device)
    for v0 in range(0, n, 65535):
        v1 = min(n, v0 + 65535)
        eff = effects[:, v0:v1].contiguous() if (v0 or v1 != n) else effects
        _lib.check(lib.expecto_variant_reduce_lut(_lib.dptr(eff), _lib.dptr(d[v0:v1]), _lib.dptr(sp[v0:v1]),
                                                  _lib.dptr(sh), S, v1 - v0, F, _lib.dptr(lut), lut.shape[1],
                                                  _lib.dptr(out[v0:v1]), _lib.stream_ptr()), "variant_reduce")
    return out


def decay_table(dist, strand_plus, shifts) -> np.ndarray:
    """[5, K] float64 exp(-c_k * fl) for fl = 0..K-1, K covering every floor(|d|/200) of the
    batch (d = dist*sgn + shift*sgn): numpy's exp of the arguments predict.py:88-107 passes it,
    so the device reduction reproduces the reference's weights exactly."""
    sgn = np.where(np.asarray(strand_plus, bool), 1, -1).astype(np.int64)
    d = np.asarray(dist, np.int64) * sgn
    sh = np.asarray(list(shifts), np.int64)
    reach = int(np.abs(d).max(initial=0)) + int(np.abs(sh).max(initial=0))
    fl = np.arange(int(np.floor(reach / 200.0)) + 1, dtype=np.float64)
    return np.ascontiguousarray(np.stack([np.exp(-c * fl) for c in (0.01, 0.02, 0.05, 0.1, 0.2)]))
