"""Multi-rank .diff.h5 write path without GPUs.

`chromatin --output-mode rank` has every rank pwrite its own rows into the snps.shift_*.diff.h5
.part files rank 0 created (expecto_amd/chromatin.py; reference layout chromatin.py:281-286).
This probe runs exactly that write pattern with R processes and synthetic rows: rank 0 creates
the files (h5.RowWriter, fsynced), every rank attaches (RowWriter(create=False)) and writes, per
batch of B variants, for every shift, strand and dataset one block of B rows at the global row
index (fwd rows at lo + k*B, rc rows N later) -- the CLI's complete() loop.  Rows hold
f(global row, shift, dataset), so the files can be checked byte for byte afterwards.

  python tools/write_probe.py --ranks 8 --variants 100000 --dir /tmp/wp [--stagger]

--stagger: rank r starts its shift loop at shift r % S (ranks spread over the files instead of
all taking the same file's inode lock first).  Prints one JSON line: aggregate GB/s = all bytes
/ the slowest rank's write time (ranks start together at a barrier).
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from expecto_amd import h5  # noqa: E402
from expecto_amd.dist import shard_range  # noqa: E402

DATASETS = ("ref", "alt", "diff")
F = 2002


def row_block(rows: np.ndarray, out: np.ndarray) -> np.ndarray:
    """Rows of global indices `rows`: every element holds float32(row) except column 0, which
    the writer stamps with the (shift, dataset) tag j * 4 + d before each write (one column,
    so generating the rows costs little next to writing them)."""
    out[:] = rows.astype(np.float32)[:, None]
    return out


def _files(d: str, shifts):
    return {s: os.path.join(d, f"snps.shift_{s}.diff.h5.part") for s in shifts}


def _rank(rank, ranks, n, shifts, batch, d, stagger, barrier, q, threads=1):
    specs = {k: ((2 * n, F), np.float32) for k in DATASETS}
    writers = {s: h5.RowWriter(p, specs, create=False) for s, p in _files(d, shifts).items()}
    lo, hi = shard_range(n, rank, ranks)
    S = len(shifts)
    order = [(j + (rank % S if stagger else 0)) % S for j in range(S)]
    blk = np.empty((min(batch, max(1, hi - lo)), F), np.float32)
    barrier.wait()
    t0 = time.perf_counter()
    nbytes = 0
    blk2 = np.empty_like(blk)
    pool = None
    if threads > 1:   # the CLI's --write-threads: one shift's 6 blocks written concurrently
        from concurrent.futures import ThreadPoolExecutor
        pool = ThreadPoolExecutor(max_workers=threads)
        tagged = [np.empty_like(blk) for _ in range(2 * len(DATASETS))]
    for b0 in range(lo, hi, batch):
        b1 = min(hi, b0 + batch)
        xs = [row_block(np.arange(b0, b1) + strand * n, x[:b1 - b0]) for strand, x in ((0, blk), (1, blk2))]
        for j in order:
            w = writers[shifts[j]]
            jobs = []
            for strand in (0, 1):
                x = xs[strand]
                for di, name in enumerate(DATASETS):
                    if pool is None:
                        x[:, 0] = j * 4 + di
                        w.write_rows(name, b0 + strand * n, x)
                    else:
                        t = tagged[strand * len(DATASETS) + di][:b1 - b0]
                        t[:] = x
                        t[:, 0] = j * 4 + di
                        jobs.append(pool.submit(w.write_rows, name, b0 + strand * n, t))
                    nbytes += x.nbytes
            for f in jobs:
                f.result()
    el = time.perf_counter() - t0
    for w in writers.values():
        w.close()
    q.put((rank, el, nbytes))


def run(d: str, ranks: int = 8, n: int = 100_000, shifts=(0, -200, -400, -600, -800, 200, 400, 600, 800),
        batch: int = 4096, stagger: bool = False, threads: int = 1) -> dict:
    os.makedirs(d, exist_ok=True)
    shifts = list(shifts)
    specs = {k: ((2 * n, F), np.float32) for k in DATASETS}
    for p in _files(d, shifts).values():
        w = h5.RowWriter(p, specs)
        w.sync()
        w.close()
    ctx = mp.get_context("spawn")
    barrier, q = ctx.Barrier(ranks), ctx.Queue()
    procs = [ctx.Process(target=_rank, args=(r, ranks, n, shifts, batch, d, stagger, barrier, q, threads))
             for r in range(ranks)]
    for p in procs:
        p.start()
    res = [q.get(timeout=3600) for _ in procs]
    for p in procs:
        p.join()
        if p.exitcode != 0:
            raise RuntimeError(f"a writer rank failed (exit {p.exitcode})")
    el = max(r[1] for r in res)
    total = sum(r[2] for r in res)
    return {"ranks": ranks, "variants": n, "shifts": len(shifts), "batch": batch, "stagger": stagger, "threads": threads,
            "bytes": total, "slowest_rank_s": el, "fastest_rank_s": min(r[1] for r in res),
            "aggregate_GB_per_s": total / el / 1e9}


def check(d: str, n: int, shifts) -> None:
    """Every row of every file holds its f(global row, shift, dataset)."""
    want = np.empty((2 * n, F), np.float32)
    row_block(np.arange(2 * n), want)
    for j, s in enumerate(shifts):
        got = h5.read(_files(d, shifts)[s])
        for di, name in enumerate(DATASETS):
            want[:, 0] = j * 4 + di
            if not np.array_equal(got[name], want):
                bad = np.nonzero((got[name] != want).any(1))[0]
                raise AssertionError(f"shift {s} {name}: rows {bad[:5].tolist()} differ")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--variants", type=int, default=100_000)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--dir", required=True)
    ap.add_argument("--stagger", action="store_true")
    ap.add_argument("--threads", type=int, default=1, help="write threads per rank (the CLI's --write-threads)")
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--keep", action="store_true")
    a = ap.parse_args()
    shifts = [0, -200, -400, -600, -800, 200, 400, 600, 800]
    try:
        r = run(a.dir, a.ranks, a.variants, shifts, a.batch, a.stagger, a.threads)
        if a.check:
            check(a.dir, a.variants, shifts)
            r["checked"] = True
        print(json.dumps(r), flush=True)
    finally:
        if not a.keep:
            for p in _files(a.dir, shifts).values():
                if os.path.exists(p):
                    os.unlink(p)


if __name__ == "__main__":
    main()
