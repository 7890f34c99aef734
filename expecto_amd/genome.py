"""Genome access: a pyfasta-compatible FASTA reader over a memory-mapped code cache, and the
device-resident code genome.

``Fasta(path).sequence({'chr','start','stop'})`` returns the 1-based inclusive slice as a
``str`` -- the only pyfasta call the reference makes (``chromatin.py:44,205``,
``compute_expecto_features.py:31,108``, ``replicate_expecto_features.py:28``;
pyfasta==0.5.2, ``requirements.txt:20``, is not installable offline).  Case is preserved, as
pyfasta does.

**Code cache** (round 4; the role pyfasta's ``.flat`` + ``.gdx`` play for the reference: it
flattens the FASTA once and memory-maps it on every later open).  The first open of a FASTA
writes (about 2x the genome's size; one line on stderr says where), next to it, or under
``$EXPECTO_CACHE_DIR`` when that is set or the FASTA's directory is read-only:

* ``<fa>.expecto.flat``  -- the contigs' sequence bytes, newlines removed (case kept);
* ``<fa>.expecto.codes`` -- the device layout: one uint8 code per base (0=A 1=G 2=C 3=T
  4=zero column) with ``GUARD`` zero codes before, between and after the contigs;
* ``<fa>.expecto.gdx.npz`` -- the index: contig names, lengths, offsets in both files, the
  code offsets and bytes of characters encodeSeqs rejects (so windows touching them still raise
  ``KeyError``), and the source's size and mtime.

Every later open (every run, every rank) maps these files: ``Fasta.sequence`` slices the
``.flat`` map, ``CodeGenome.codes`` is the ``.codes`` map, and ``DeviceGenome`` streams it into
HBM through two pinned chunks.  Ranks of one node share the page cache instead of each parsing
and encoding the FASTA (an hg19-sized genome: ~34 s parse + ~15 s encode and ~9 GB of host
memory per process before round 4).  A cache whose source changed (size or mtime) or whose
format differs is rebuilt; the build holds an ``flock`` so concurrent ranks build it once.

``DeviceGenome`` windows running up to GUARD bases past a contig end read zero columns
(pyfasta's behaviour there is not pinned by any fixture: SURVEY.md 7, "Window-edge
semantics"); ``check_spans`` rejects any window reaching further, so the window
kernels never read a neighbouring contig.
"""
from __future__ import annotations

import hashlib
import json
import os
import time

import numpy as np

from .encode import CODE_ZERO, _LUT

GUARD = 32768     # > the +-21 kb reach of a TSS segment (compute_expecto_features.py:88)
CACHE_VERSION = 1
_CHUNK = 64 << 20  # bytes of FASTA per parse step (bounds the build's memory)
LAST_OPEN = {}     # how the last Fasta(path) got its cache: {"built": bool, "s": seconds} (bench reads it)


# ---------------------------------------------------------------------------- code cache
def _stat_key(path: str) -> dict:
    st = os.stat(path)
    return {"source": os.path.realpath(path), "size": st.st_size, "mtime_ns": st.st_mtime_ns,
            "version": CACHE_VERSION, "guard": GUARD}


def cache_prefix(path: str) -> str:
    """Where the cache files of FASTA ``path`` live: under ``$EXPECTO_CACHE_DIR`` keyed by the
    real path when it is set, else next to the FASTA when that directory is writable, else under
    ``~/.cache/expecto_amd``."""
    d = os.path.dirname(os.path.abspath(path))
    if not os.environ.get("EXPECTO_CACHE_DIR") and os.access(d, os.W_OK):
        return os.path.abspath(path) + ".expecto"
    root = os.environ.get("EXPECTO_CACHE_DIR") or os.path.join(os.path.expanduser("~"), ".cache", "expecto_amd")
    os.makedirs(root, exist_ok=True)
    h = hashlib.sha1(os.path.realpath(path).encode()).hexdigest()[:16]
    return os.path.join(root, f"{os.path.basename(path)}.{h}.expecto")


def _load_index(prefix: str):
    try:
        with np.load(prefix + ".gdx.npz", allow_pickle=False) as z:
            meta = json.loads(bytes(z["meta"]).decode())
            inv_off, inv_chr = z["invalid_offsets"].astype(np.int64), z["invalid_chars"].astype(np.uint8)
    except (OSError, ValueError, KeyError):
        return None
    return meta, inv_off, inv_chr


def _headers(buf: np.ndarray):
    """(name, sequence start, sequence end) per '>' header line of the mapped FASTA ``buf``, in
    file order (the same records as a line-by-line parse: a '>' counts only at a line start)."""
    n = buf.size
    gts = []
    for a in range(0, n, _CHUNK):
        b = min(n, a + _CHUNK)
        p = np.flatnonzero(buf[a:b] == ord(">")) + a
        if p.size:
            prev = buf[np.maximum(p - 1, 0)]
            p = p[(p == 0) | (prev == ord("\n"))]
        gts.append(p)
    gts = np.concatenate(gts) if gts else np.zeros(0, np.int64)
    recs = []
    for i, g in enumerate(gts):
        g, w = int(g), 4096
        while True:                       # end of the header line
            j = bytes(buf[g:g + w]).find(b"\n")
            if j >= 0 or g + w >= n:
                nl = g + j if j >= 0 else n
                break
            w *= 4
        name = bytes(buf[g + 1:nl]).rstrip(b"\r").split()[0].decode()
        end = int(gts[i + 1]) if i + 1 < gts.size else n
        recs.append((name, min(nl + 1, n), end))
    return recs


def build_cache(path: str, prefix: str | None = None) -> str:
    """Flatten + encode FASTA ``path`` into the cache files (``cache_prefix``); returns the
    prefix.  One streaming pass of ``_CHUNK``-sized pieces: newline / CR bytes dropped (as the
    line reader's rstrip), bytes appended to ``.flat``, their codes (``encode._LUT``; rejected
    characters stored as the zero code and recorded) to ``.codes`` with GUARD zero codes around
    each contig.  Files are written under temporary names and renamed, the index last."""
    prefix = prefix or cache_prefix(path)
    key = _stat_key(path)
    import secrets
    import socket
    # unique per builder even where flock does not reach across nodes (a shared / network file
    # system): host, pid and a random token, so two builders never write the same temp files
    tmp = f".tmp.{socket.gethostname()}.{os.getpid()}.{secrets.token_hex(4)}"
    names, lengths, flat_off, code_off = [], [], [], []
    bad_off, bad_chr = [], []
    guard = np.full(GUARD, CODE_ZERO, np.uint8)
    with open(path, "rb") as src:
        size = os.fstat(src.fileno()).st_size
        buf = np.memmap(src, np.uint8, "r") if size else np.zeros(0, np.uint8)
        recs = _headers(buf)
        seen = set()
        for name, _, _ in recs:
            if name in seen:
                raise ValueError(f"{path}: contig {name} appears twice")
            seen.add(name)
        # the pieces are independent (numpy releases the GIL in the masks, compress and LUT):
        # up to `ahead` of them in flight on a thread pool, written in file order
        tasks = [(r, a, min(b0, a + _CHUNK)) for r, (_, a0, b0) in enumerate(recs) for a in range(a0, b0, _CHUNK)]

        def piece(t):
            c = np.asarray(buf[t[1]:t[2]])
            keep = c[(c != ord("\n")) & (c != ord("\r"))]
            codes = _LUT[keep]
            bad = np.flatnonzero(codes == 255)
            if bad.size:   # characters encodeSeqs rejects: windows touching them raise KeyError
                codes[bad] = CODE_ZERO
            return keep, codes, bad

        from concurrent.futures import ThreadPoolExecutor
        workers = max(1, min(8, os.cpu_count() or 1))
        ahead = 2 * workers
        with open(prefix + ".flat" + tmp, "wb") as ff, open(prefix + ".codes" + tmp, "wb") as fc, \
                ThreadPoolExecutor(workers) as ex:
            fc.write(guard.tobytes())
            fpos, cpos, ln, cur = 0, GUARD, 0, -1
            futs = [ex.submit(piece, t) for t in tasks[:ahead]]
            for i, t in enumerate(tasks + [(len(recs), 0, 0)]):
                while cur < t[0]:                  # close the open record, open the next ones
                    if cur >= 0:
                        lengths.append(ln)
                        fpos += ln
                        cpos += ln + GUARD
                        fc.write(guard.tobytes())
                    cur += 1
                    if cur < len(recs):
                        names.append(recs[cur][0])
                        flat_off.append(fpos)
                        code_off.append(cpos)
                        ln = 0
                if i == len(tasks):
                    break
                keep, codes, bad = futs[i].result()
                futs[i] = None
                if i + ahead < len(tasks):
                    futs.append(ex.submit(piece, tasks[i + ahead]))
                if bad.size:
                    bad_off.append(bad.astype(np.int64) + cpos + ln)
                    bad_chr.append(keep[bad])
                ff.write(keep.tobytes())
                fc.write(codes.tobytes())
                ln += keep.size
        del buf
    meta = dict(key, names=names, lengths=lengths, flat_offsets=flat_off, code_offsets=code_off,
                code_total=cpos, flat_total=fpos)
    inv_off = np.concatenate(bad_off) if bad_off else np.zeros(0, np.int64)
    inv_chr = np.concatenate(bad_chr) if bad_chr else np.zeros(0, np.uint8)
    with open(prefix + ".gdx.npz" + tmp, "wb") as fi:
        np.savez(fi, meta=np.frombuffer(json.dumps(meta).encode(), np.uint8), invalid_offsets=inv_off,
                 invalid_chars=inv_chr)
    for ext in (".flat", ".codes", ".gdx.npz"):
        os.replace(prefix + ext + tmp, prefix + ext)
    import sys
    print(f"expecto_amd.genome: built the code cache of {path} at {prefix}.{{flat,codes,gdx.npz}} "
          f"({(fpos + cpos) / 1e9:.2f} GB; EXPECTO_CACHE_DIR moves it)", file=sys.stderr)
    return prefix


def open_cache(path: str):
    """(prefix, meta, invalid offsets, invalid chars) of an up-to-date cache of ``path``, building
    it first when missing or stale (under an exclusive flock, so concurrent ranks build once)."""
    import fcntl
    prefix = cache_prefix(path)
    key = _stat_key(path)
    t0 = time.perf_counter()

    def fresh():
        idx = _load_index(prefix)
        if idx is None or any(idx[0].get(k) != v for k, v in key.items()):
            return None
        if any(not os.path.exists(prefix + e) for e in (".flat", ".codes")):
            return None
        # both data files at the byte lengths the index recorded (a torn or foreign write is rebuilt)
        if (os.path.getsize(prefix + ".codes") != idx[0]["code_total"]
                or os.path.getsize(prefix + ".flat") != idx[0]["flat_total"]):
            return None
        return idx

    idx = fresh()
    built = False
    if idx is None:
        with open(prefix + ".lock", "a+") as lk:
            fcntl.flock(lk, fcntl.LOCK_EX)
            try:
                idx = fresh()             # another rank may have built it while we waited
                if idx is None:
                    build_cache(path, prefix)
                    built = True
                    idx = fresh()
            finally:
                fcntl.flock(lk, fcntl.LOCK_UN)
        if idx is None:
            raise RuntimeError(f"{path}: the genome cache at {prefix}.* could not be built")
    LAST_OPEN.clear()
    LAST_OPEN.update(built=built, s=time.perf_counter() - t0, prefix=prefix)
    return (prefix,) + idx


# ---------------------------------------------------------------------------- FASTA
class Fasta:
    """pyfasta.Fasta subset.  ``Fasta(path)`` maps the code cache of ``path`` (built on the first
    open); ``Fasta.from_dict`` holds in-memory contigs (tests, the synthetic benchmark genome)."""

    def __init__(self, path: str):
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        self.path = path
        prefix, meta, inv_off, inv_chr = open_cache(path)
        self.cache_prefix = prefix
        self._meta = meta
        self._flat = (np.memmap(prefix + ".flat", np.uint8, "r") if meta["flat_total"]
                      else np.zeros(0, np.uint8))
        self._seqs = {n: self._flat[o:o + ln] for n, o, ln in
                      zip(meta["names"], meta["flat_offsets"], meta["lengths"])}
        self._invalid = (inv_off, inv_chr)

    @classmethod
    def from_dict(cls, seqs: dict) -> "Fasta":
        obj = cls.__new__(cls)
        obj.path = None
        obj.cache_prefix = None
        obj._meta = None
        obj._seqs = {k: (v if isinstance(v, bytes) else v.encode()) for k, v in seqs.items()}
        return obj

    def keys(self):
        return self._seqs.keys()

    def __contains__(self, name):
        return name in self._seqs

    def __len__(self):
        return len(self._seqs)

    def raw(self, chrom: str):
        """The contig's sequence bytes: ``bytes`` (in-memory) or a read-only uint8 map (cached);
        both slice, and ``bytes(...)`` of a slice gives the bases."""
        return self._seqs[chrom]

    def sequence(self, f: dict, one_based: bool = True) -> str:
        start = f["start"] - 1 if one_based else f["start"]
        stop = f["stop"]
        if start < 0:
            raise ValueError(f"window {f} starts before the contig (edge semantics unpinned)")
        return bytes(self._seqs[f["chr"]][start:stop]).decode("latin-1")


class CodeGenome:
    """Host-side concatenated codes + per-contig offsets: the cache's ``.codes`` map for a
    cached Fasta (nothing re-encoded), else encoded in memory from the contigs."""

    def __init__(self, fasta: Fasta):
        self.codes_path = None
        if getattr(fasta, "_meta", None) is not None:
            m = fasta._meta
            self.codes_path = fasta.cache_prefix + ".codes"
            self.codes = np.memmap(self.codes_path, np.uint8, "r", shape=(m["code_total"],))
            self.offsets = dict(zip(m["names"], m["code_offsets"]))
            self.lengths = dict(zip(m["names"], m["lengths"]))
            self.invalid_offsets, self.invalid_chars = fasta._invalid
            return
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


def upload_codes(host: CodeGenome, device, chunk: int = 256 << 20):
    """The host codes as a uint8 device tensor.  A cached genome streams its ``.codes`` file
    through two pinned chunks (file read of chunk k+1 while chunk k's copy runs; no pageable
    copy, no full host copy); an in-memory one is copied directly."""
    import torch
    n = int(host.codes.size)
    out = torch.empty(n, dtype=torch.uint8, device=device)
    if host.codes_path is None or n <= chunk:
        src = host.codes if host.codes.flags.writeable else np.array(host.codes)   # a read-only map: copy (torch
        out.copy_(torch.from_numpy(np.ascontiguousarray(src)))                      # warns on non-writable arrays)
        return out
    bufs = [torch.empty(chunk, dtype=torch.uint8, pin_memory=True) for _ in range(2)]
    events = [None, None]
    with torch.cuda.device(out.device), open(host.codes_path, "rb", buffering=0) as f:
        for i, a in enumerate(range(0, n, chunk)):
            b = min(n, a + chunk)
            k = i % 2
            if events[k] is not None:
                events[k].synchronize()       # the copy that last used this pinned chunk is done
            mv = memoryview(bufs[k].numpy()[:b - a])
            got = 0
            while got < b - a:
                r = f.readinto(mv[got:])
                if not r:
                    raise IOError(f"{host.codes_path}: short read at {a + got}")
                got += r
            out[a:b].copy_(bufs[k][:b - a], non_blocking=True)
            events[k] = torch.cuda.Event()
            events[k].record()
        torch.cuda.current_stream().synchronize()
    return out


class DeviceGenome:
    """CodeGenome resident in HBM as a torch uint8 tensor."""

    def __init__(self, fasta: Fasta, device="cuda"):
        self.host = CodeGenome(fasta)
        self.codes = upload_codes(self.host, device)
        self.offsets = self.host.offsets
        self.lengths = self.host.lengths

    def offset(self, chrom: str, pos1: int) -> int:
        return self.host.offset(chrom, pos1)

    def check_spans(self, chroms, lo, hi) -> None:
        self.host.check_spans(chroms, lo, hi)


def open_genome(path: str) -> Fasta:
    return Fasta(path)
