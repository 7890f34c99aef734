"""CPU restatement of the spatial-feature reductions -- TEST INFRASTRUCTURE (oracle) ONLY.

* ``tss_pos_weights`` / ``tss_reduce`` -- ``compute_expecto_features.py:88-101,123-124``:
  ``pred = 0.5*(fwd+rc)`` (f32), ``F[k,f] = sum_s W[k,s] * pred[s,f]`` in float64,
  flattened k-major to 10*2002 = 20020 features.
* ``fwd_rc_average`` -- ``predict.py:183-194``: average the fwd half and the rc half of
  a ``.diff.h5`` dataset ``(2N, 2002)`` -> ``(N, 2002)`` f32.
* ``variant_weights`` / ``variant_reduce`` -- ``predict.py:87-136``: per shift j,
  ``d = dist*sgn + shift_j*sgn``; ``W_j[:,k] = exp(-c_k*floor(|d|/200))`` masked by
  ``d<=0`` (k<5) or ``d>=0`` (k>=5); ``F[n, k*2002+f] = sum_j W_j[n,k]*eff_j[n,f]`` (f64).
"""
from __future__ import annotations

import numpy as np

DECAY = (0.01, 0.02, 0.05, 0.1, 0.2)
TSS_SHIFTS = np.arange(-20000, 20000, 200)          # compute_expecto_features.py:88


def tss_pos_weights(shifts=TSS_SHIFTS) -> np.ndarray:
    """10 x len(shifts) float64 (compute_expecto_features.py:91-101)."""
    s = np.asarray(shifts)
    rows = [np.exp(-c * np.abs(s) / 200) * (s <= 0) for c in DECAY]
    rows += [np.exp(-c * np.abs(s) / 200) * (s >= 0) for c in DECAY]
    return np.vstack(rows)


def tss_reduce(pred_fwd: np.ndarray, pred_rc: np.ndarray, weights=None) -> np.ndarray:
    """One gene: [200,2002] f32 fwd and rc predictions -> f64 [20020]."""
    if weights is None:
        weights = tss_pos_weights()
    pred = np.float32(0.5) * (np.asarray(pred_fwd, np.float32) + np.asarray(pred_rc, np.float32))
    return np.sum(weights[:, :, None] * pred[None, :, :], axis=1).flatten()


def fwd_rc_average(x: np.ndarray) -> np.ndarray:
    """predict.py:186: (x[:N] + x[N:]) / 2.0 with N = rows/2, kept in f32."""
    n = x.shape[0] // 2
    return ((x[0:n] + x[n:2 * n]) / np.float32(2.0)).astype(x.dtype)


def variant_weights(dist, strand_plus, shifts) -> list:
    """predict.py:87-109: one (n,10) f64 matrix per shift (in the given shift order)."""
    sgn = np.where(np.asarray(strand_plus, bool), 1, -1)
    snpdists = np.asarray(dist) * sgn
    out = []
    for sh in shifts:
        d = snpdists + sh * sgn
        fl = np.floor(np.abs(d) / 200.0)
        cols = [np.exp(-c * fl) * (d <= 0) for c in DECAY] + [np.exp(-c * fl) * (d >= 0) for c in DECAY]
        out.append(np.vstack(cols).T)
    return out


def variant_reduce(effects: list, weights: list, nfeatures: int = 2002) -> np.ndarray:
    """predict.py:123-124: sum_j tile(eff_j,10) * repeat(W_j, nfeatures, axis=1) -> f64."""
    acc = None
    for eff, w in zip(effects, weights):
        term = np.tile(np.asarray(eff), 10) * np.repeat(w, nfeatures, axis=1)
        acc = term if acc is None else acc + term
    return acc
