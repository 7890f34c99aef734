"""Per-dispatch HBM bytes and rate of one kernel from three rocprofv3 runs of the same command.

The runs (separate passes: FETCH_SIZE and WRITE_SIZE do not fit one TCC pass; durations from a
trace-only run, since counter passes stretch kernels):

    cd /tmp && export TMPDIR=/tmp
    rocprofv3 --pmc FETCH_SIZE --kernel-include-regex fk_seq --output-format csv -d OUT/pmc -o run -- python3 bench.py ...
    rocprofv3 --pmc WRITE_SIZE --kernel-include-regex fk_seq --output-format csv -d OUT/pmcw -o run -- python3 bench.py ...
    rocprofv3 --kernel-trace --kernel-include-regex fk_seq --output-format csv -d OUT/kt -o run -- python3 bench.py ...

    python tools/dispatch_traffic.py OUT fk_seq_h2 > profiles/rNN/fk_seq_pmc.csv

Dispatches are matched in order. FETCH_SIZE is doubled (gfx950 reports half the bytes of a wide
coalesced read, MI355X_MICROARCH.md "HBM"); WRITE_SIZE is exact for 16-B-per-lane stores.
"""
from __future__ import annotations

import csv
import sys


def _counter(path: str, name: str, kernel: str) -> list[float]:
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == name and kernel in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    return [float(r["Counter_Value"]) for r in rows]


def main(out: str, kernel: str) -> None:
    fetch = _counter(f"{out}/pmc/run_counter_collection.csv", "FETCH_SIZE", kernel)
    write = _counter(f"{out}/pmcw/run_counter_collection.csv", "WRITE_SIZE", kernel)
    trace = [r for r in csv.DictReader(open(f"{out}/kt/run_kernel_trace.csv")) if kernel in r["Kernel_Name"]]
    trace.sort(key=lambda r: int(r["Dispatch_Id"]))
    n = min(len(fetch), len(write), len(trace))
    w = csv.writer(sys.stdout)
    w.writerow(["dispatch", "grid_size", "read_bytes", "write_bytes", "duration_ns", "tb_per_s"])
    for i in range(n):
        rd, wr = fetch[i] * 1024 * 2, write[i] * 1024
        ns = int(trace[i]["End_Timestamp"]) - int(trace[i]["Start_Timestamp"])
        w.writerow([i, trace[i]["Grid_Size_X"], int(rd), int(wr), ns, round((rd + wr) / ns / 1e3, 3)])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
