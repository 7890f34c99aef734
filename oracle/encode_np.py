"""CPU restatement of the sequence-preparation rows -- TEST INFRASTRUCTURE (oracle) ONLY.

* ``encode_seqs``    -- ``encodeSeqs`` (``chromatin.py:138-172``; identical
                        ``expecto_utils.py:5-39``): centre-crop with
                        ``floor((len-L)/2)``, one-hot A,G,C,T -> channels 0..3 (either
                        case), N/n/H/- -> all zero, anything else -> KeyError; output
                        ``[fwd rows ; rc rows]`` where rc = ``[:, ::-1, ::-1]``.
                        ``with_rc=False`` is the TSS scripts' variant
                        (``compute_expecto_features.py:184-218``, rc lines commented out).
* ``fetch_seqs``     -- ``fetchSeqs`` (``chromatin.py:175-209``) over any object with a
                        pyfasta-style ``sequence({'chr','start','stop'})`` (1-based,
                        inclusive).
* ``tss_window``     -- the TSS tiling (``compute_expecto_features.py:107-111``).
"""
from __future__ import annotations

import math

import numpy as np

_ONEHOT = {
    "A": (1, 0, 0, 0), "G": (0, 1, 0, 0), "C": (0, 0, 1, 0), "T": (0, 0, 0, 1),
    "N": (0, 0, 0, 0), "H": (0, 0, 0, 0),
    "a": (1, 0, 0, 0), "g": (0, 1, 0, 0), "c": (0, 0, 1, 0), "t": (0, 0, 0, 1),
    "n": (0, 0, 0, 0), "-": (0, 0, 0, 0),
}


def crop(line: str, inputsize: int = 2000) -> str:
    """Centre crop of chromatin.py:164."""
    lo = int(math.floor((len(line) - inputsize) / 2.0))
    hi = int(math.floor(len(line) - (len(line) - inputsize) / 2.0))
    return line[lo:hi]


def encode_seqs(seqs, inputsize: int = 2000, with_rc: bool = True) -> np.ndarray:
    """Pure-Python restatement of encodeSeqs (small cases only)."""
    out = np.zeros((len(seqs), 4, inputsize), np.bool_)
    for n, line in enumerate(seqs):
        for i, c in enumerate(crop(line, inputsize)):
            out[n, :, i] = _ONEHOT[c]            # KeyError on unknown characters
    if with_rc:
        out = np.concatenate([out, out[:, ::-1, ::-1]], axis=0)
    return out


def fetch_seqs(genome, chrom, pos, ref, alt, shift=0, inputsize=2000):
    """fetchSeqs (chromatin.py:175-209): window [pos+shift-1049, pos+shift+1050]."""
    windowsize = inputsize + 100
    mutpos = int(windowsize / 2 - 1 - shift)
    seq = genome.sequence({"chr": chrom, "start": pos + shift - int(windowsize / 2 - 1),
                           "stop": pos + shift + int(windowsize / 2)})
    ref_ok = seq[mutpos:(mutpos + len(ref))].upper() == ref.upper()
    alt_ok = seq[mutpos:(mutpos + len(ref))].upper() == alt.upper()
    return (seq[:mutpos] + ref + seq[(mutpos + len(ref)):],
            seq[:mutpos] + alt + seq[(mutpos + len(ref)):], ref_ok, alt_ok)


def shift_order(maxshift: int):
    """Shift order of chromatin.py:243 / predict.py:109,173."""
    return [0] + list(range(-200, -maxshift - 1, -200)) + list(range(200, maxshift + 1, 200))


def tss_window(genome, chrom, tss, strand, shift, windowsize=2000):
    """compute_expecto_features.py:108-110."""
    return genome.sequence({"chr": chrom,
                            "start": tss + (shift * strand) - int(windowsize / 2 - 1),
                            "stop": tss + (shift * strand) + int(windowsize / 2)})
