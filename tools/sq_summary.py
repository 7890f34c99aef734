"""Summarise gemm_bench SQ counter passes (tools/gpu_session.sh step gbpmc) for one variant's kernel.
    python tools/sq_summary.py <variant> [kernel-substring]"""
import csv
import glob
import sys

v = sys.argv[1]
ks = sys.argv[2] if len(sys.argv) > 2 else None
vals = {}
for path in sorted(glob.glob(f"gpurun_out/pmc_gb_{v}_[0-9]/run_counter_collection.csv")):
    acc = {}
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if "x6_wm4" in name or "beluga_gemm_x6<" in name or (ks and ks not in name):
            continue
        d = acc.setdefault(r["Counter_Name"], {})
        d[r["Dispatch_Id"]] = d.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    for c, d in acc.items():
        vals[c] = sum(d.values()) / len(d)
for c in sorted(vals):
    print(f"{c:28s} {vals[c]:.4g}")
wc = vals.get("SQ_WAVE_CYCLES")
if wc:
    for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_MFMA",
              "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_VALU"):
        if c in vals:
            print(f"  {c:26s} / WAVE_CYCLES = {vals[c] / wc:.3f}")
if "GRBM_GUI_ACTIVE" in vals and "SQ_VALU_MFMA_BUSY_CYCLES" in vals:
    print(f"  MFMA busy per SIMD-cycle = {vals['SQ_VALU_MFMA_BUSY_CYCLES'] / 1024 / (vals['GRBM_GUI_ACTIVE'] / 8):.3f}")
