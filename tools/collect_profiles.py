"""Turn one tools/profile_round.sh run (gpurun_out/) into the committed profiles/<tag>/ summaries.

    python tools/collect_profiles.py r01 [--bench-log gpurun_out/bench.log]

Writes
  kernel_stats.csv    rocprofv3 --kernel-trace --stats of the headline bench command
  pmc_traffic.csv     per-kernel FETCH_SIZE / WRITE_SIZE per dispatch (separate --pmc passes)
  pmc_sq.csv          per-kernel GRBM_GUI_ACTIVE / SQ_* per dispatch
  traffic.json        HBM bytes per launch for every kernel, keyed by kernel name, plus the
                      bench configuration it was measured on; bench.py reads it to fill
                      roofline.traffic when its own configuration matches
  bench_profiled.json the bench line printed under rocprofv3 (kernel-trace pass)

FETCH_SIZE is doubled: on gfx950 it reports half the bytes of 16-B-per-lane streaming reads
(MI355X_MICROARCH.md "HBM").  WRITE_SIZE is taken as is (calibrated: conv1's WRITE_SIZE equals
its output bytes exactly).  Counter values are KB.
"""
import argparse
import csv
import json
import os
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_kernel(path):
    acc = {}
    for r in csv.DictReader(open(path)):
        acc.setdefault(r["Kernel_Name"], {}).setdefault(r["Counter_Name"], {})
        # one row per (dispatch, counter); sum over dimension instances of a dispatch
        d = acc[r["Kernel_Name"]][r["Counter_Name"]]
        d[r["Dispatch_Id"]] = d.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return {k: {c: (sum(v.values()) / len(v), len(v)) for c, v in cs.items()} for k, cs in acc.items()}


def bench_line(path):
    for line in open(path):
        if line.startswith("{"):
            return json.loads(line)
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--src", default=os.path.join(ROOT, "gpurun_out"))
    ap.add_argument("--bench-log", default=None, help="full default bench log to keep as bench.json")
    a = ap.parse_args()
    src, dst = a.src, os.path.join(ROOT, "profiles", a.tag)
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, f"prof_{a.tag}", "run_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
    fetch = per_kernel(os.path.join(src, f"pmc_fetch_{a.tag}", "run_counter_collection.csv"))
    write = per_kernel(os.path.join(src, f"pmc_write_{a.tag}", "run_counter_collection.csv"))
    sq = per_kernel(os.path.join(src, f"pmc_sq_{a.tag}", "run_counter_collection.csv"))
    prof_bench = bench_line(os.path.join(src, f"prof_{a.tag}.log"))
    traffic = {}
    with open(os.path.join(dst, "pmc_traffic.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "dispatches", "FETCH_SIZE_KB", "WRITE_SIZE_KB", "read_bytes_est", "write_bytes",
                    "hbm_bytes_per_launch"])
        for k in sorted(fetch, key=lambda k: -fetch[k]["FETCH_SIZE"][0]):
            fk, n = fetch[k]["FETCH_SIZE"]
            wk = write.get(k, {}).get("WRITE_SIZE", (0.0, 0))[0]
            rd, wr = 2 * fk * 1024, wk * 1024
            traffic[k] = {"read_bytes": rd, "write_bytes": wr, "hbm_bytes": rd + wr, "dispatches": n}
            w.writerow([k, n, f"{fk:.1f}", f"{wk:.1f}", f"{rd:.4g}", f"{wr:.4g}", f"{rd + wr:.4g}"])
    names = ["GRBM_GUI_ACTIVE", "SQ_BUSY_CYCLES", "SQ_WAVE_CYCLES", "SQ_VALU_MFMA_BUSY_CYCLES"]
    with open(os.path.join(dst, "pmc_sq.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "dispatches"] + names)
        for k in sorted(sq, key=lambda k: -sq[k].get("GRBM_GUI_ACTIVE", (0, 0))[0]):
            w.writerow([k, sq[k][names[0]][1]] + [f"{sq[k].get(c, (0, 0))[0]:.6g}" for c in names])
    cfg = None
    if prof_bench is not None:
        json.dump(prof_bench, open(os.path.join(dst, "bench_profiled.json"), "w"), indent=1)
        cfg = prof_bench.get("profile_key")
    json.dump({"profile_key": cfg, "source": f"profiles/{a.tag}/pmc_traffic.csv", "kernels": traffic},
              open(os.path.join(dst, "traffic.json"), "w"), indent=1)
    if a.bench_log:
        b = bench_line(a.bench_log)
        json.dump(b, open(os.path.join(dst, "bench.json"), "w"), indent=1)
    print("wrote", dst)


if __name__ == "__main__":
    main()
