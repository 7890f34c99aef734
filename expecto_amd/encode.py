"""Sequence encoding: the ``encodeSeqs`` twin and the uint8 base-code path.

``encodeSeqs(seqs, inputsize)`` reproduces ``chromatin.py:138-172`` /
``expecto_utils.py:5-39`` exactly (bool ``[fwd rows; rc rows]``, centre crop with
``floor((len-L)/2)``, A,G,C,T -> channels 0..3 in either case, N/n/H/- -> zeros,
any other character -> ``KeyError``), vectorised with a 256-entry lookup table.

The GPU path never materialises one-hot floats on the host: ``seqs_to_codes`` turns the
cropped strings into uint8 codes (0=A 1=G 2=C 3=T 4=zero column) and the conv1 kernel
expands them (and their reverse complement) in LDS.
"""
from __future__ import annotations

import math

import numpy as np

CODE_ZERO = 4
_LUT = np.full(256, 255, np.uint8)
for _ch, _c in (("A", 0), ("G", 1), ("C", 2), ("T", 3)):
    _LUT[ord(_ch)] = _c
    _LUT[ord(_ch.lower())] = _c
for _ch in "NnH-":
    _LUT[ord(_ch)] = CODE_ZERO
_ONEHOT = np.zeros((256, 4), np.bool_)
_ONEHOT[np.arange(4), np.arange(4)] = True


def crop_bounds(length: int, inputsize: int = 2000):
    """Centre-crop slice of chromatin.py:164."""
    lo = int(math.floor((length - inputsize) / 2.0))
    hi = int(math.floor(length - (length - inputsize) / 2.0))
    return lo, hi


def _to_bytes(s) -> bytes:
    return s if isinstance(s, (bytes, bytearray)) else s.encode("latin-1")


def seq_codes(seq, inputsize: int = 2000) -> np.ndarray:
    """Codes of one sequence after the centre crop; raises KeyError like encodeSeqs."""
    b = _to_bytes(seq)
    lo, hi = crop_bounds(len(b), inputsize)
    raw = np.frombuffer(bytes(b[lo:hi]), np.uint8)  # Python slice semantics, as the reference
    codes = _LUT[raw]
    bad = np.nonzero(codes == 255)[0]
    if bad.size:
        raise KeyError(chr(raw[bad[0]]))
    return codes


def seqs_to_codes(seqs, inputsize: int = 2000) -> np.ndarray:
    """uint8 [n, inputsize]; short cropped sequences leave trailing zero columns (code 4),
    as encodeSeqs leaves the tail of its zero-initialised array."""
    out = np.full((len(seqs), inputsize), CODE_ZERO, np.uint8)
    for i, s in enumerate(seqs):
        c = seq_codes(s, inputsize)
        out[i, : c.size] = c
    return out


def codes_to_onehot(codes: np.ndarray, with_rc: bool = True) -> np.ndarray:
    """bool [n(,x2), 4, L] from codes (code 4 -> all-zero column)."""
    oh = _ONEHOT[codes].transpose(0, 2, 1)
    if with_rc:
        oh = np.concatenate([oh, oh[:, ::-1, ::-1]], axis=0)
    return np.ascontiguousarray(oh)


def encodeSeqs(seqs, inputsize: int = 2000) -> np.ndarray:
    """Drop-in for the reference encodeSeqs (chromatin.py:138-172): [fwd; rc] bool."""
    return codes_to_onehot(seqs_to_codes(seqs, inputsize), with_rc=True)


def encodeSeqs_fwd(seqs, inputsize: int = 2000) -> np.ndarray:
    """The TSS scripts' variant without the rc half (compute_expecto_features.py:184-218)."""
    return codes_to_onehot(seqs_to_codes(seqs, inputsize), with_rc=False)
