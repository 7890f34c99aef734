"""Kernels of one Beluga.forward per batch size from a rocprofv3 kernel trace of
tools/small_batch_probe.py --trace (the 23rd forward of each batch: 3 warm-ups + 20 timed).
    python tools/small_batch_trace.py gpurun_out/sbt/run_kernel_trace.csv"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
rows = [r for r in rows]   # (the blit kernels of hipMemsetAsync / hipMemcpyAsync included)
starts = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith("onehot_codes") or "::onehot_codes(" in r["Kernel_Name"]]
# forwards in order: 23 per batch (onehot_codes opens every forward of exact one-hot input)
for b, B in enumerate((32, 200, 512)):
    k = 23 * b + 22
    if k + 1 >= len(starts) + 1 or k >= len(starts):
        break
    i0, i1 = starts[k], (starts[k + 1] if k + 1 < len(starts) else len(rows))
    ks = rows[i0:i1]
    t0, t1 = int(ks[0]["Start_Timestamp"]), int(ks[-1]["End_Timestamp"])
    prev_end = int(rows[i0 - 1]["End_Timestamp"]) if i0 > 0 else t0
    print(f"batch {B}: first kernel start -> last kernel end {(t1 - t0) / 1e3:.1f} us; host gap before it "
          f"{(t0 - prev_end) / 1e3:.1f} us")
    for r in ks:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        g = int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"])
        print(f"  {d:8.1f} us {g:7d} workgroups  {r['Kernel_Name'].split('(')[0]}")
