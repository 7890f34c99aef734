"""Turn one tools/gpu_session.sh prof,pmc run (gpurun_out/) into the committed profiles/<tag>/ summaries.

    python tools/collect_profiles.py r01 [--bench-log gpurun_out/bench.log]

Writes
  kernel_stats.csv    rocprofv3 --kernel-trace --stats of the headline bench command
  pmc_traffic.csv     per-kernel FETCH_SIZE / WRITE_SIZE per dispatch (separate --pmc passes)
  pmc_sq.csv          per-kernel GRBM_GUI_ACTIVE / SQ_* per dispatch
  traffic.json        HBM bytes per launch for every kernel, keyed by kernel name, plus the
                      bench configuration it was measured on; bench.py reads it to fill
                      roofline.traffic when its own configuration matches.  Per kernel also
                      the "main" launches (the largest grid: a layer's full launches, where the
                      same kernel also runs the small alt-delta launches) and their bytes
  launch_groups.csv   per kernel and grid size: dispatches and mean duration from the kernel
                      trace (the full-size launches' duration, comparable to the HIP-event
                      per-launch time the bench line reports for a layer)
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


def per_dispatch(path):
    """{kernel: {counter: {dispatch: (value, grid)}}} (values summed over dimension instances)."""
    acc = {}
    for r in csv.DictReader(open(path)):
        d = acc.setdefault(r["Kernel_Name"], {}).setdefault(r["Counter_Name"], {})
        v, g = d.get(r["Dispatch_Id"], (0.0, int(r["Grid_Size"])))
        d[r["Dispatch_Id"]] = (v + float(r["Counter_Value"]), g)
    return acc


def per_kernel(path, main_only=False):
    """{kernel: {counter: (mean per dispatch, dispatches)}}; main_only: the largest-grid dispatches."""
    out = {}
    for k, cs in per_dispatch(path).items():
        out[k] = {}
        for c, v in cs.items():
            vals = list(v.values())
            if main_only:
                g = max(x[1] for x in vals)
                vals = [x for x in vals if x[1] == g]
            out[k][c] = (sum(x[0] for x in vals) / len(vals), len(vals))
    return out


def launch_groups(trace_csv, out_csv):
    groups = {}
    for r in csv.DictReader(open(trace_csv)):
        g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        e = groups.setdefault((r["Kernel_Name"], g), [0, 0.0])
        e[0] += 1
        e[1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    with open(out_csv, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "grid_size", "dispatches", "avg_ns", "total_ns"])
        for (k, g), (n, t) in sorted(groups.items(), key=lambda kv: -kv[1][1]):
            w.writerow([k, g, n, f"{t / n:.0f}", f"{t:.0f}"])


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
    fetch_m = per_kernel(os.path.join(src, f"pmc_fetch_{a.tag}", "run_counter_collection.csv"), main_only=True)
    write_m = per_kernel(os.path.join(src, f"pmc_write_{a.tag}", "run_counter_collection.csv"), main_only=True)
    trace = os.path.join(src, f"prof_{a.tag}", "run_kernel_trace.csv")
    if os.path.exists(trace):
        launch_groups(trace, os.path.join(dst, "launch_groups.csv"))
    # SQ / GRBM counters of the full-size launches (the held clock and MFMA-busy of a layer's
    # launch; the alt-delta launches share the kernel)
    sq = per_kernel(os.path.join(src, f"pmc_sq_{a.tag}", "run_counter_collection.csv"), main_only=True)
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
            fm, nm = fetch_m[k]["FETCH_SIZE"]
            wm = write_m.get(k, {}).get("WRITE_SIZE", (0.0, 0))[0]
            traffic[k] = {"read_bytes": rd, "write_bytes": wr, "hbm_bytes": rd + wr, "dispatches": n,
                          "main_read_bytes": 2 * fm * 1024, "main_write_bytes": wm * 1024,
                          "main_hbm_bytes": 2 * fm * 1024 + wm * 1024, "main_dispatches": nm}
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
