"""Variant shift-sweep pipeline on the device (the hot loop of chromatin.py:243-286).

For a batch of variants and a list of shifts:

1. window codes for every (allele, shift, variant) are generated ON THE DEVICE from the
   HBM-resident genome (``expecto_variant_windows``; SNVs), or on the host for indels
   and MNPs (``fetchSeqs`` splice + centre crop, chromatin.py:202-209,164), then
2. ONE ``forward_codes(..., BOTH)`` call runs the Beluga forward over all of them
   (fwd rows then rc rows, the encodeSeqs order of chromatin.py:170-171),
3. ``diff = alt - ref`` (chromatin.py:281) on the device.

Output tensor ``y[strand][allele][shift][variant][2002]``; per shift the reference's
h5 datasets are ``ref = y[:,0,j]``, ``alt = y[:,1,j]`` (each [2N,2002], fwd rows first).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

from . import _lib
from .encode import _LUT, seq_codes

CHRS = ['chr1', 'chr2', 'chr3', 'chr4', 'chr5', 'chr6', 'chr7', 'chr8', 'chr9',
        'chr10', 'chr11', 'chr12', 'chr13', 'chr14', 'chr15', 'chr16', 'chr17',
        'chr18', 'chr19', 'chr20', 'chr21', 'chr22', 'chrX', 'chrY']   # chromatin.py:108-110


def shift_order(maxshift: int):
    """chromatin.py:243 (and predict.py:109,173)."""
    return [0] + list(range(-200, -maxshift - 1, -200)) + list(range(200, maxshift + 1, 200))


def _allele_code(a: str) -> int:
    c = int(_LUT[ord(a)]) if len(a) == 1 and ord(a) < 256 else 255
    if c == 255:
        raise KeyError(a)          # encodeSeqs' dict lookup fails the same way
    return c


@dataclass
class VariantSet:
    chrom: list
    pos: np.ndarray          # 1-based
    ref: list
    alt: list

    def __len__(self):
        return len(self.chrom)


def fetch_window(fasta, chrom, pos, ref, allele, shift, inputsize=2000) -> str:
    """fetchSeqs for one allele (chromatin.py:202-209)."""
    windowsize = inputsize + 100
    mutpos = int(windowsize / 2 - 1 - shift)
    seq = fasta.sequence({"chr": chrom, "start": pos + shift - int(windowsize / 2 - 1),
                          "stop": pos + shift + int(windowsize / 2)})
    return seq[:mutpos] + allele + seq[(mutpos + len(ref)):]


def match_counts(fasta, vs: VariantSet):
    """(ref_matched, alt_matched) booleans of chromatin.py:207-208 (window-independent)."""
    rm, am = [], []
    for c, p, r, a in zip(vs.chrom, vs.pos, vs.ref, vs.alt):
        g = fasta.raw(c)[int(p) - 1:int(p) - 1 + len(r)].decode("latin-1").upper()
        rm.append(g == r.upper())
        am.append(g == a.upper())
    return np.array(rm, bool), np.array(am, bool)


class VariantPipeline:
    """Holds the device genome + model engine; computes shift sweeps for variant batches."""

    def __init__(self, engine, fasta, dgenome, inputsize: int = 2000):
        if inputsize != 2000:
            raise ValueError("Beluga's FC1 fixes the input size at 2000 (Beluga.py:43)")
        self.engine = engine
        self.fasta = fasta
        self.dg = dgenome
        self.device = dgenome.codes.device
        self.lib = _lib.load()

    def prepare(self, vs: VariantSet, shifts) -> dict:
        """Host checks + the device-resident variant table (offsets, allele codes, shifts)."""
        n = len(vs)
        snv = np.array([len(r) == 1 and len(a) == 1 for r, a in zip(vs.ref, vs.alt)], bool)
        off = np.array([self.dg.offset(c, int(p)) for c, p in zip(vs.chrom, vs.pos)], np.int64)
        self._check_window_chars(off[snv], shifts)
        rc = np.array([_allele_code(r) if s else 4 for r, s in zip(vs.ref, snv)], np.uint8)
        ac = np.array([_allele_code(a) if s else 4 for a, s in zip(vs.alt, snv)], np.uint8)
        prep = {"n": n, "S": len(shifts), "shifts": list(shifts),
                "off": torch.from_numpy(off).to(self.device), "rc": torch.from_numpy(rc).to(self.device),
                "ac": torch.from_numpy(ac).to(self.device),
                "sh": torch.tensor(list(shifts), dtype=torch.int32, device=self.device), "host": None}
        if n and not snv.all():
            # indels / MNPs: length-changing splice + floor crop on the host (chromatin.py:164,209)
            idx = np.nonzero(~snv)[0]
            host = np.empty((2, len(shifts), idx.size, 2000), np.uint8)
            for k, v in enumerate(idx):
                for j, sh in enumerate(shifts):
                    for a, allele in enumerate((vs.ref[v], vs.alt[v])):
                        w = fetch_window(self.fasta, vs.chrom[v], int(vs.pos[v]), vs.ref[v], allele, sh)
                        c = seq_codes(w)
                        host[a, j, k, :] = 4
                        host[a, j, k, :c.size] = c
            prep["host"] = (torch.from_numpy(idx).to(self.device), torch.from_numpy(host).to(self.device))
        return prep

    def window_codes(self, prep: dict, out: torch.Tensor | None = None) -> torch.Tensor:
        """uint8 [2 alleles, S, n, 2000] on the device (no host work)."""
        n, S = prep["n"], prep["S"]
        codes = out if out is not None else torch.empty((2, S, n, 2000), dtype=torch.uint8, device=self.device)
        if n == 0:
            return codes
        st = _lib.stream_ptr()
        for v0 in range(0, n, 65535):
            v1 = min(n, v0 + 65535)
            # the kernel writes [2][S][nv][2000]; split batches go through a scratch slab
            blk = codes if (v0 == 0 and v1 == n) else torch.empty((2, S, v1 - v0, 2000), dtype=torch.uint8,
                                                                   device=self.device)
            _lib.check(self.lib.expecto_variant_windows(
                _lib.dptr(self.dg.codes), self.dg.codes.numel(), _lib.dptr(prep["off"][v0:v1]),
                _lib.dptr(prep["rc"][v0:v1]), _lib.dptr(prep["ac"][v0:v1]), v1 - v0, _lib.dptr(prep["sh"]), S,
                _lib.dptr(blk), st), "variant_windows")
            if blk is not codes:
                codes[:, :, v0:v1] = blk
        if prep["host"] is not None:
            idx, host = prep["host"]
            codes[:, :, idx] = host
        return codes

    def _check_window_chars(self, off, shifts):
        """encodeSeqs raises KeyError on characters outside A/C/G/T/N/H/- (chromatin.py:166)."""
        bad = self.dg.host.invalid_offsets
        if bad.size == 0 or off.size == 0:
            return
        lo = off + min(shifts) - 999
        hi = off + max(shifts) + 1000
        i = np.searchsorted(bad, lo)
        hit = (i < bad.size) & (bad[np.minimum(i, bad.size - 1)] <= hi)
        if hit.any():
            b = bad[i[np.nonzero(hit)[0][0]]]
            raise KeyError(chr(self.dg.host.invalid_chars[np.searchsorted(bad, b)]))

    def predict(self, vs, shifts=None, out: torch.Tensor | None = None, codes: torch.Tensor | None = None):
        """y [2 strands, 2 alleles, S, n, 2002] fp32 on the device.  `vs` is a VariantSet
        (prepared here) or the dict returned by prepare()."""
        prep = vs if isinstance(vs, dict) else self.prepare(vs, shifts)
        n, S = prep["n"], prep["S"]
        codes = self.window_codes(prep, codes)
        flat = codes.view(2 * S * n, 2000)
        if out is None:
            out = torch.empty((2, 2, S, n, 2002), dtype=torch.float32, device=self.device)
        self.engine.forward_codes(flat, _lib.STRAND_BOTH, out=out.view(4 * S * n, 2002))
        return out

    def diff(self, y: torch.Tensor) -> torch.Tensor:
        """diff[strand][shift][v] = alt - ref (chromatin.py:281), [2, S, n, 2002]."""
        d = torch.empty((2,) + tuple(y.shape[2:]), dtype=y.dtype, device=y.device)
        st = _lib.stream_ptr()
        for s in range(2):
            cnt = y[s, 0].numel()
            _lib.check(self.lib.expecto_diff(_lib.dptr(y[s, 1]), _lib.dptr(y[s, 0]), cnt, _lib.dptr(d[s]), st),
                       "diff")
        return d


def per_shift_datasets(y: torch.Tensor, d: torch.Tensor, j: int):
    """Host arrays (diff, ref, alt) for shift index j in the reference's [2N,2002] layout."""
    n = y.shape[3]
    ref = y[:, 0, j].reshape(2 * n, 2002)
    alt = y[:, 1, j].reshape(2 * n, 2002)
    return d[:, j].reshape(2 * n, 2002).cpu().numpy(), ref.cpu().numpy(), alt.cpu().numpy()
