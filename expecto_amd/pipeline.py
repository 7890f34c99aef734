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


def fc1_role(offset: int, seg_len: int, rc: bool = False) -> int:
    """Block-Karatsuba FC1 role of the window at bp `offset` of a segment of `seg_len` bp on the
    segment path (include/expecto_hip.h expecto_beluga_set_fc1_role): its 25-conv6-row (400 bp)
    step within its pool2-phase block, mod 4; on the rc strand the window's offset in the
    reverse-complemented segment."""
    o = seg_len - 2000 - offset if rc else offset
    return ((o >> 4) // 25) % 4


def sweep_roles(shifts, pairs: bool = True) -> np.ndarray:
    """[2 strands, S] FC1 roles of a variant sweep's windows on the segment path (segment layout of
    VariantPipeline.prepare: window j at offset shifts[j] - min(shifts)).  Segment pairs in which
    more than a third of the windows hold the SNV (shift in (-1001, 999]) run the direct FC1: role 4
    for every window (include/expecto_hip.h expecto_beluga_set_fc1_role)."""
    lo, hi = min(shifts), max(shifts)
    L = 2000 + hi - lo
    if pairs and 3 * sum(1 for s in shifts if -1001 < s <= 999) > len(shifts):
        return np.full((2, len(shifts)), 4, np.int64)
    return np.array([[fc1_role(s - lo, L, rc) for s in shifts] for rc in (False, True)], np.int64)


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

    def slice(self, a: int, b: int) -> "VariantSet":
        return VariantSet(self.chrom[a:b], self.pos[a:b], self.ref[a:b], self.alt[a:b])


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
        g = bytes(fasta.raw(c)[int(p) - 1:int(p) - 1 + len(r)]).decode("latin-1").upper()
        rm.append(g == r.upper())
        am.append(g == a.upper())
    return np.array(rm, bool), np.array(am, bool)


def gather_segments(lib, dg, start: torch.Tensor, seg_len: int, splice_pos=None, splice_code=None,
                    out: torch.Tensor | None = None) -> torch.Tensor:
    """uint8 [n, seg_len] genome slices (+ optional single-base splice) on the device."""
    n = start.numel()
    codes = out if out is not None else torch.empty((n, seg_len), dtype=torch.uint8, device=start.device)
    st = _lib.stream_ptr()
    for i0 in range(0, n, 65535):
        i1 = min(n, i0 + 65535)
        _lib.check(lib.expecto_gather_segments(
            _lib.dptr(dg.codes), dg.codes.numel(), _lib.dptr(start[i0:i1]), i1 - i0, seg_len,
            None if splice_pos is None else _lib.dptr(splice_pos[i0:i1]),
            None if splice_code is None else _lib.dptr(splice_code[i0:i1]), _lib.dptr(codes[i0:i1]), st),
            "gather_segments")
    return codes


def to_device(a, device) -> torch.Tensor:
    """Host array -> device tensor without a host sync: staged through pinned memory (torch's
    caching host allocator keeps it alive until the copy ran), so preparing batch k+1 does not
    wait for batch k's kernels (a pageable .to(device) synchronises the stream)."""
    t = torch.from_numpy(np.ascontiguousarray(a))
    return t.pin_memory().to(device, non_blocking=True)


class VariantPipeline:
    """Holds the device genome + model engine; computes shift sweeps for variant batches.

    SNVs go through the segment path: per variant ONE ref sequence covering every shift's
    window (length 2000 + max_shift - min_shift), so the conv trunk is computed once per
    sequence instead of once per shift, and the alt allele recomputes only the rows the SNV
    changes at each layer (use_pairs); single-shift runs use the per-window pair path.
    Outputs are bit-identical to the per-window forward of every window.
    Indels/MNPs, whose windows are length-changing splices, use the per-window path with
    host-built codes; shift lists that are not 4-aligned use per-window device windows."""

    def __init__(self, engine, fasta, dgenome, inputsize: int = 2000, use_segments: bool = True,
                 use_pairs: bool = True):
        if inputsize != 2000:
            raise ValueError("Beluga's FC1 fixes the input size at 2000 (Beluga.py:43)")
        self.engine = engine
        self.fasta = fasta
        self.dg = dgenome
        self.device = dgenome.codes.device
        self.lib = _lib.load()
        self.use_segments = use_segments
        self.use_pairs = use_pairs

    def prepare(self, vs: VariantSet, shifts, rows: str = "shift") -> dict:
        """Host checks + the device-resident variant tables (done once, outside the hot loop).

        rows="shift" (chromatin.py's per-shift files): ``y[strand][allele][shift][variant]``;
        rows="variant" (the 200-shift eQTL scoring, geuvadis_sed_for_top_eqtls.py:61-98):
        ``y[strand][allele][variant][shift]``, so each variant's [S, 2002] block is contiguous
        for the shift reductions.  "variant" needs SNVs on 4-aligned shifts (segment path)."""
        if rows not in ("shift", "variant"):
            raise ValueError("rows must be 'shift' or 'variant'")
        n, S = len(vs), len(shifts)
        shifts = list(shifts)
        snv = np.array([len(r) == 1 and len(a) == 1 for r, a in zip(vs.ref, vs.alt)], bool).reshape(-1)
        off = np.array([self.dg.offset(c, int(p)) for c, p in zip(vs.chrom, vs.pos)], np.int64).reshape(-1)
        snv_idx, ind_idx = np.nonzero(snv)[0], np.nonzero(~snv)[0]
        self._check_window_chars(off[snv_idx], shifts)
        if n:
            self.dg.check_spans(vs.chrom, off + min(shifts) - 999, off + max(shifts) + 1000)
        rc = np.array([_allele_code(vs.ref[v]) for v in snv_idx], np.uint8).reshape(-1)
        ac = np.array([_allele_code(vs.alt[v]) for v in snv_idx], np.uint8).reshape(-1)
        ns = snv_idx.size
        dev = self.device
        prep = {"n": n, "S": S, "shifts": shifts, "rows": rows, "snv_idx": to_device(snv_idx, dev),
                "ind_idx": to_device(ind_idx, dev), "n_snv": ns, "n_ind": ind_idx.size,
                "seg": None, "win": None, "ind_codes": None}
        lo_s, hi_s = min(shifts), max(shifts)
        if ns and S > 1 and self.use_segments and all((x - lo_s) % 4 == 0 for x in shifts):
            L = 2000 + hi_s - lo_s
            if self.use_pairs:
                # ref segment v; window (v, j) at offset shifts[j] - lo_s -> row j*ns + v of each
                # allele block; the alt segment is the ref one with the alt base at 999 - lo_s
                v_i, j_i = np.meshgrid(np.arange(ns), np.arange(S), indexing="ij")
                prep["seg"] = {
                    "L": L, "pairs": True,
                    "start": to_device(off[snv_idx] + lo_s - 999, dev),
                    "splice_pos": torch.full((ns,), 999 - lo_s, dtype=torch.int32, device=dev),
                    "splice_code": to_device(rc, dev),
                    "alt_code": to_device(ac, dev),
                    "var_pos": np.full(ns, 999 - lo_s, np.int32),
                    "win_seg": v_i.ravel().astype(np.int32),
                    "win_off": (np.asarray(shifts)[j_i.ravel()] - lo_s).astype(np.int32),
                    "win_row": ((j_i * ns + v_i) if rows == "shift" else (v_i * S + j_i)).ravel().astype(np.int32),
                }
            else:
                # segment a*ns + v; window (a, v, j) at offset shifts[j] - lo_s -> row (a*S + j)*ns + v
                a_i, v_i, j_i = np.meshgrid(np.arange(2), np.arange(ns), np.arange(S), indexing="ij")
                prep["seg"] = {
                    "L": L, "pairs": False,
                    "start": to_device(np.concatenate([off[snv_idx], off[snv_idx]]) + lo_s - 999, dev),
                    "splice_pos": torch.full((2 * ns,), 999 - lo_s, dtype=torch.int32, device=dev),
                    "splice_code": to_device(np.concatenate([rc, ac]), dev),
                    "win_seg": (a_i * ns + v_i).ravel().astype(np.int32),
                    "win_off": (np.asarray(shifts)[j_i.ravel()] - lo_s).astype(np.int32),
                    "win_row": (((a_i * S + j_i) * ns + v_i) if rows == "shift" else
                                ((a_i * ns + v_i) * S + j_i)).ravel().astype(np.int32),
                }
        elif ns:
            prep["win"] = {"off": to_device(off[snv_idx], dev), "rc": to_device(rc, dev),
                           "ac": to_device(ac, dev),
                           "sh": to_device(np.asarray(shifts, np.int32), dev)}
        if rows == "variant" and (prep["seg"] is None or ind_idx.size):
            raise ValueError('rows="variant" needs SNVs on 4-aligned shifts (the segment path)')
        if ind_idx.size:
            prep["ind_codes"] = self._indel_window_codes(vs, ind_idx, shifts)
        return prep

    def _indel_window_codes(self, vs: VariantSet, ind_idx: np.ndarray, shifts) -> torch.Tensor:
        """uint8 [2 alleles, S, n_ind, 2000] windows of indels / MNPs: the length-changing splice
        of fetchSeqs and the floor centre crop of encodeSeqs (chromatin.py:164,202-209).  Items
        whose 2100-base fetch window lies inside the contig with the splice inside it and a
        spliced length >= 2000 are built on the device (expecto_indel_windows, one kernel for the
        batch); the rest -- the reference's Python-slicing corner cases (negative slice starts,
        windows cut by the contig end) -- through the host twin fetch_window + seq_codes."""
        S, ni = len(shifts), ind_idx.size
        A, J, K = (x.ravel() for x in np.meshgrid(np.arange(2), np.arange(S), np.arange(ni), indexing="ij"))
        v = ind_idx[K]
        sh = np.asarray(shifts, np.int64)[J]
        pos = np.asarray(vs.pos, np.int64).reshape(-1)[v]
        chroms = [vs.chrom[x] for x in v]
        lens = np.array([[len(vs.ref[x]), len(vs.alt[x])] for x in ind_idx], np.int64).reshape(ni, 2)
        lref, lalt = lens[K, 0], lens[K, A]
        mut = 1049 - sh                                  # mutpos of fetchSeqs (windowsize 2100)
        ls = 2100 - lref + lalt                          # spliced length
        crop = (ls - 2000) // 2                          # floor((len - 2000) / 2), chromatin.py:164
        cs = pos + sh - 1050                             # window start inside the contig (0-based)
        clen = np.array([self.dg.lengths[c] for c in chroms], np.int64)
        acodes = [[_LUT[np.frombuffer(vs.ref[x].encode("latin-1"), np.uint8)],
                   _LUT[np.frombuffer(vs.alt[x].encode("latin-1"), np.uint8)]] for x in ind_idx]
        valid = np.array([[(c != 255).all() for c in pair] for pair in acodes], bool).reshape(ni, 2)
        dev_ok = (cs >= 0) & (cs + 2100 <= clen) & (mut >= 0) & (mut + lref <= 2100) & (ls >= 2000) & valid[K, A]
        s0 = np.array([self.dg.offsets[c] for c in chroms], np.int64) + cs
        # encodeSeqs' KeyError on characters outside A/C/G/T/N/H/- in the visible genome bases
        bad = self.dg.host.invalid_offsets
        if bad.size and dev_ok.any():
            d = np.nonzero(dev_ok)[0]
            lo1, hi1 = s0[d] + crop[d], s0[d] + np.minimum(mut[d], crop[d] + 2000)
            lo2 = s0[d] + np.maximum(mut[d] + lalt[d], crop[d]) - lalt[d] + lref[d]
            hi2 = s0[d] + crop[d] + 2000 - lalt[d] + lref[d]
            for lo, hi in ((lo1, hi1), (lo2, hi2)):
                i = np.searchsorted(bad, lo)
                hit = (i < bad.size) & (bad[np.minimum(i, bad.size - 1)] < hi) & (lo < hi)
                if hit.any():
                    b = bad[i[np.nonzero(hit)[0][0]]]
                    raise KeyError(chr(self.dg.host.invalid_chars[np.searchsorted(bad, b)]))
        flat = [c for pair in acodes for c in pair]      # allele (k, a) -> flat index 2k + a
        aoff = np.concatenate([[0], np.cumsum([c.size for c in flat])]).astype(np.int64)
        table = np.concatenate(flat + [np.zeros(1, np.uint8)]).astype(np.uint8)
        n_items = 2 * S * ni
        out = torch.empty((n_items, 2000), dtype=torch.uint8, device=self.device)
        d = np.nonzero(dev_ok)[0]
        if d.size:
            dev = self.device
            tab = to_device(table, dev)
            cols = [to_device(np.ascontiguousarray(x), dev) for x in
                    (s0[d], mut[d].astype(np.int32), lref[d].astype(np.int32), lalt[d].astype(np.int32),
                     crop[d].astype(np.int32), aoff[2 * K[d] + A[d]].astype(np.int32))]
            blk = torch.empty((d.size, 2000), dtype=torch.uint8, device=dev)
            st = _lib.stream_ptr()
            for i0 in range(0, d.size, 65535):
                i1 = min(d.size, i0 + 65535)
                _lib.check(self.lib.expecto_indel_windows(
                    _lib.dptr(self.dg.codes), self.dg.codes.numel(), *(_lib.dptr(c[i0:i1]) for c in cols),
                    _lib.dptr(tab), i1 - i0, _lib.dptr(blk[i0:i1]), st), "indel_windows")
            out[to_device(d, dev)] = blk
        h = np.nonzero(~dev_ok)[0]
        if h.size:
            host = np.full((h.size, 2000), 4, np.uint8)
            for r, t in enumerate(h):
                x = int(v[t])
                allele = vs.alt[x] if A[t] else vs.ref[x]
                c = seq_codes(fetch_window(self.fasta, vs.chrom[x], int(vs.pos[x]), vs.ref[x], allele, int(sh[t])))
                host[r, :c.size] = c
            out[to_device(h, self.device)] = to_device(host, self.device)
        return out.view(2, S, ni, 2000)

    def _snv_window_codes(self, prep: dict) -> torch.Tensor:
        """uint8 [2 alleles, S, n_snv, 2000] per-window codes on the device."""
        ns, S, w = prep["n_snv"], prep["S"], prep["win"]
        codes = torch.empty((2, S, ns, 2000), dtype=torch.uint8, device=self.device)
        st = _lib.stream_ptr()
        for v0 in range(0, ns, 65535):
            v1 = min(ns, v0 + 65535)
            blk = codes if (v0 == 0 and v1 == ns) else torch.empty((2, S, v1 - v0, 2000), dtype=torch.uint8,
                                                                    device=self.device)
            _lib.check(self.lib.expecto_variant_windows(
                _lib.dptr(self.dg.codes), self.dg.codes.numel(), _lib.dptr(w["off"][v0:v1]), _lib.dptr(w["rc"][v0:v1]),
                _lib.dptr(w["ac"][v0:v1]), v1 - v0, _lib.dptr(w["sh"]), S, _lib.dptr(blk), st), "variant_windows")
            if blk is not codes:
                codes[:, :, v0:v1] = blk
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

    def predict(self, vs, shifts=None, out: torch.Tensor | None = None):
        """y [2 strands, 2 alleles, S, n, 2002] fp32 on the device.  `vs` is a VariantSet
        (prepared here) or the dict returned by prepare()."""
        prep = vs if isinstance(vs, dict) else self.prepare(vs, shifts)
        n, S, ns, ni = prep["n"], prep["S"], prep["n_snv"], prep["n_ind"]
        if out is None:
            shape = (2, 2, S, n, 2002) if prep.get("rows", "shift") == "shift" else (2, 2, n, S, 2002)
            out = torch.empty(shape, dtype=torch.float32, device=self.device)
        if ns:
            y = out if ni == 0 else torch.empty((2, 2, S, ns, 2002), dtype=torch.float32, device=self.device)
            seg = prep["seg"]
            if seg is not None:
                scodes = gather_segments(self.lib, self.dg, seg["start"], seg["L"], seg["splice_pos"],
                                         seg["splice_code"])
                if seg["pairs"]:
                    yf = y.view(4 * S * ns, 2002)
                    self.engine.forward_segment_pairs(scodes, seg["L"], seg["var_pos"], seg["alt_code"],
                                                      seg["win_seg"], seg["win_off"], seg["win_row"], yf[0:],
                                                      yf[S * ns:], 2 * S * ns, _lib.STRAND_BOTH)
                else:
                    self.engine.forward_segments(scodes, seg["L"], seg["win_seg"], seg["win_off"], seg["win_row"],
                                                 _lib.STRAND_BOTH, out=y.view(4 * S * ns, 2002))
            elif self.use_pairs:
                # alt-cone reuse per shift: the alt window recomputes only the SNV's cone
                codes = self._snv_window_codes(prep)
                yf = y.view(2 * 2 * S * ns, 2002)
                if "pair_pos" not in prep:
                    prep["pair_pos"] = [torch.full((ns,), 999 - sh, dtype=torch.int32, device=self.device)
                                        for sh in prep["shifts"]]
                for j in range(S):
                    self.engine.forward_pairs(codes[0, j], codes[1, j], prep["pair_pos"][j], yf[j * ns:],
                                              yf[(S + j) * ns:], 2 * S * ns, _lib.STRAND_BOTH)
            else:
                codes = self._snv_window_codes(prep)
                self.engine.forward_codes(codes.view(2 * S * ns, 2000), _lib.STRAND_BOTH,
                                          out=y.view(4 * S * ns, 2002))
            if ni:
                out.index_copy_(3, prep["snv_idx"], y)
        if ni:
            yi = torch.empty((2, 2, S, ni, 2002), dtype=torch.float32, device=self.device)
            self.engine.forward_codes(prep["ind_codes"].view(2 * S * ni, 2000), _lib.STRAND_BOTH,
                                      out=yi.view(4 * S * ni, 2002))
            out.index_copy_(3, prep["ind_idx"], yi)
        return out

    def recompute_overflowed(self, vs: VariantSet, shifts, out: torch.Tensor, rows: str = "shift",
                             parts: int = 8) -> int:
        """Release-point recovery of a batch whose deferred f16x3 overflow flag fired (the engine
        in deferred mode, ``overflow_take``): instead of recomputing the whole batch in bf16x6,
        rerun it in f16x3 as `parts` variant slices with one flag each -- an output row depends
        only on its own window, so the rerun reproduces the batch's bits and only locates the
        overflow -- then recompute just the flagged slices in bf16x6 into `out`.  Cost 1 + 2f
        batch-times for a flagged fraction f, against 2 for the whole batch.  If no slice flags
        again, the whole batch is recomputed in bf16x6 (counted once).  Returns the number of
        bf16x6 recomputations, as the engine's fallback counter counts them: one per flagged
        slice, or 1 when the whole batch was recomputed; ``self.last_recomputed_slices`` holds the
        number of slices whose rows were recomputed (all `parts` slices in the second case)."""
        eng = self.engine
        n = len(vs)
        if n == 0:
            return 0
        bounds = np.unique(np.linspace(0, n, min(parts, n) + 1).round().astype(int))
        k = len(bounds) - 1
        flags = torch.zeros(k, dtype=torch.int32).pin_memory()
        preps = []
        for i in range(k):
            prep = self.prepare(vs.slice(int(bounds[i]), int(bounds[i + 1])), shifts, rows)
            preps.append(prep)
            self.predict(prep)
            eng.overflow_take(flags[i:i + 1])
        torch.cuda.current_stream().synchronize()
        dim = 3 if rows == "shift" else 2
        redone = 0
        for i in range(k):
            if not int(flags[i]):
                continue
            with eng.precision_override("bf16x6"):
                y = self.predict(preps[i])
            out.narrow(dim, int(bounds[i]), int(bounds[i + 1] - bounds[i])).copy_(y)
            eng.count_fallback()
            redone += 1
        if redone == 0:
            # the batch flagged but no slice rerun did: the rerun did not reproduce the batch's
            # launches (a launch-size dependence of some kernel), so the overflowed rows are not
            # located -- recompute the whole batch in bf16x6 rather than release them
            with eng.precision_override("bf16x6"):
                self.predict(self.prepare(vs, shifts, rows), out=out)
            eng.count_fallback()
            self.last_recomputed_slices = k
            return 1
        self.last_recomputed_slices = redone
        return redone

    def sed_features(self, y: torch.Tensor, weights: torch.Tensor, out: torch.Tensor | None = None,
                     legacy: bool = True) -> torch.Tensor:
        """Per-allele eQTL features of a rows="variant" prediction y[2, 2, n, S, 2002]:
        float64 fwd/rc mean, then the 10 x S exp-decay shift reduction
        (geuvadis_sed_for_top_eqtls.py:83-121); out [2 alleles, n, 20030] (legacy layout, a zero
        column ahead of each decay block) or [2, n, 20020]."""
        _, _, n, S, F = y.shape
        width = 10 * (F + (1 if legacy else 0))
        if out is None:
            out = torch.empty((2, n, width), dtype=torch.float64, device=y.device)
        if not (y.is_contiguous() and out.is_contiguous() and tuple(out.shape) == (2, n, width)):
            raise RuntimeError("sed_features: y must be contiguous [2,2,n,S,2002], out [2,n,width]")
        st = _lib.stream_ptr()
        flags = 1 | (2 if legacy else 0)          # EXPECTO_REDUCE_F64AVG | EXPECTO_REDUCE_LEGACY20030
        for a in range(2):
            for v0 in range(0, n, 65535):
                v1 = min(n, v0 + 65535)
                _lib.check(self.lib.expecto_shift_reduce(_lib.dptr(y[0, a, v0:v1]), _lib.dptr(y[1, a, v0:v1]),
                                                         _lib.dptr(weights), v1 - v0, S, F, flags,
                                                         _lib.dptr(out[a, v0:v1]), st), "shift_reduce")
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
