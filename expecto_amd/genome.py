"""Genome access: a pyfasta-compatible FASTA reader and a device-resident code genome.

``Fasta(path).sequence({'chr','start','stop'})`` returns the 1-based inclusive slice
as a ``str`` -- the only pyfasta call the reference makes (``chromatin.py:44,205``,
``compute_expecto_features.py:31,108``; pyfasta==0.5.2 is not installable offline).
Contig sequences are kept as bytes (case preserved, as pyfasta does).

``DeviceGenome`` concatenates every contig's uint8 base codes (0=A 1=G 2=C 3=T 4=zero)
into one HBM tensor (hg19 is ~3.1 GB, a few % of 288 GB), with ``GUARD`` zero codes
between contigs.  Windows running up to GUARD bases past a contig end read zero columns
(pyfasta's behaviour there is not pinned by any fixture: SURVEY.md 7, "Window-edge
semantics"); ``check_spans`` rejects any window reaching further, so the window
kernels never read a neighbouring contig.
"""
from __future__ import annotations

import os

import numpy as np

from .encode import CODE_ZERO, _LUT

GUARD = 32768     # > the +-21 kb reach of a TSS segment (compute_expecto_features.py:88)


class Fasta:
    def __init__(self, path: str):
        self.path = path
        self._seqs: dict[str, bytes] = {}
        name, buf = None, []
        with open(path, "rb") as f:
            for line in f:
                line = line.rstrip(b"\r\n")
                if line.startswith(b">"):
                    if name is not None:
                        self._seqs[name] = b"".join(buf)
                    name, buf = line[1:].split()[0].decode(), []
                elif line:
                    buf.append(line)
        if name is not None:
            self._seqs[name] = b"".join(buf)

    @classmethod
    def from_dict(cls, seqs: dict) -> "Fasta":
        obj = cls.__new__(cls)
        obj.path = None
        obj._seqs = {k: (v if isinstance(v, bytes) else v.encode()) for k, v in seqs.items()}
        return obj

    def keys(self):
        return self._seqs.keys()

    def __contains__(self, name):
        return name in self._seqs

    def __len__(self):
        return len(self._seqs)

    def raw(self, chrom: str) -> bytes:
        return self._seqs[chrom]

    def sequence(self, f: dict, one_based: bool = True) -> str:
        start = f["start"] - 1 if one_based else f["start"]
        stop = f["stop"]
        if start < 0:
            raise ValueError(f"window {f} starts before the contig (edge semantics unpinned)")
        return self._seqs[f["chr"]][start:stop].decode("latin-1")


class CodeGenome:
    """Host-side concatenated codes + per-contig offsets (built once, reused per shift)."""

    def __init__(self, fasta: Fasta):
        names = list(fasta.keys())
        total = GUARD + sum(len(fasta.raw(n)) + GUARD for n in names)
        codes = np.full(total, CODE_ZERO, np.uint8)
        self.offsets: dict[str, int] = {}
        self.lengths: dict[str, int] = {}
        pos = GUARD
        bad_off, bad_chr = [], []
        for n in names:
            raw = np.frombuffer(fasta.raw(n), np.uint8)
            c = _LUT[raw]
            bad = np.nonzero(c == 255)[0]
            if bad.size:  # characters encodeSeqs rejects: windows touching them raise KeyError
                bad_off.append(bad + pos)
                bad_chr.append(raw[bad])
                c[bad] = CODE_ZERO
            codes[pos:pos + raw.size] = c
            self.offsets[n] = pos
            self.lengths[n] = raw.size
            pos += raw.size + GUARD
        self.codes = codes
        self.invalid_offsets = np.concatenate(bad_off).astype(np.int64) if bad_off else np.zeros(0, np.int64)
        self.invalid_chars = np.concatenate(bad_chr) if bad_chr else np.zeros(0, np.uint8)

    def offset(self, chrom: str, pos1: int) -> int:
        """Flat offset of the 1-based position ``pos1`` of ``chrom``."""
        return self.offsets[chrom] + pos1 - 1

    def check_spans(self, chroms, lo, hi) -> None:
        """Raise ValueError if a window span [lo[i], hi[i]] (flat offsets) of contig chroms[i]
        reaches more than GUARD bases outside that contig (it would read the next one)."""
        lo = np.asarray(lo, np.int64).reshape(-1)
        hi = np.asarray(hi, np.int64).reshape(-1)
        if lo.size == 0:
            return
        start = np.array([self.offsets[c] for c in chroms], np.int64)
        end = start + np.array([self.lengths[c] for c in chroms], np.int64)
        bad = np.nonzero((lo < start - GUARD) | (hi >= end + GUARD))[0]
        if bad.size:
            i = int(bad[0])
            raise ValueError(f"window of {chroms[i]} reaches more than {GUARD} bp past the contig "
                             f"(offsets {int(lo[i] - start[i])}..{int(hi[i] - start[i])} of {int(end[i] - start[i])})")


class DeviceGenome:
    """CodeGenome resident in HBM as a torch uint8 tensor."""

    def __init__(self, fasta: Fasta, device="cuda"):
        import torch

        self.host = CodeGenome(fasta)
        self.codes = torch.from_numpy(self.host.codes).to(device)
        self.offsets = self.host.offsets
        self.lengths = self.host.lengths

    def offset(self, chrom: str, pos1: int) -> int:
        return self.host.offset(chrom, pos1)

    def check_spans(self, chroms, lo, hi) -> None:
        self.host.check_spans(chroms, lo, hi)


def open_genome(path: str) -> Fasta:
    if not os.path.exists(path):
        raise FileNotFoundError(path)
    return Fasta(path)
