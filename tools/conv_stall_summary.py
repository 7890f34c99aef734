"""Summarise the SQ stall counter passes of the headline's conv kernels (tools/gpu_session.sh step
convpmc) over their MAIN launches (the largest grid of each kernel: one per strand), per SIMD:
    python tools/conv_stall_summary.py gpurun_out r06 > profiles/r06/conv_sq_stall.txt
SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles over all waves (the 4 MFMA waves AND
the 4 producer waves of each workgroup); SQ_VALU_MFMA_BUSY_CYCLES counts cycles (16 per
v_mfma_f32_16x16x32_f16); GRBM_GUI_ACTIVE is summed over the 8 XCDs (MI355X_MICROARCH.md)."""
import collections
import csv
import glob
import sys

out, tag = sys.argv[1], sys.argv[2]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for path in sorted(glob.glob(f"{out}/convpmc_[0-9]_{tag}/run_counter_collection.csv")):
    rows = list(csv.DictReader(open(path)))
    big = collections.defaultdict(int)
    for r in rows:
        big[r["Kernel_Name"]] = max(big[r["Kernel_Name"]], int(r["Grid_Size"]))
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in rows:
        if int(r["Grid_Size"]) == big[r["Kernel_Name"]]:
            per[(r["Kernel_Name"], r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    for (k, _), d in per.items():
        for c, v in d.items():
            vals[k][c].append(v)
for k in sorted(vals):
    v = {c: sum(x) / len(x) for c, x in vals[k].items()}
    name = k.split("(")[0].replace("void expecto::", "")
    print(f"== {name}: main launches ({len(vals[k]['SQ_WAVE_CYCLES'])} in the wave-cycle pass)")
    clk = v["GRBM_GUI_ACTIVE"] / 8
    print(f"  clock cycles per launch {clk:.4g}; MFMA busy per SIMD-cycle {v['SQ_VALU_MFMA_BUSY_CYCLES'] / 1024 / clk:.3f}")
    wc = v["SQ_WAVE_CYCLES"]
    for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_LDS",
              "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_MISC"):
        if c in v:
            print(f"  {c:24s} {v[c] / wc:.3f} of all waves' cycles")
    mf = v.get("SQ_INSTS_MFMA")
    if mf:
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM", "SQ_INSTS_SMEM"):
            if c in v:
                print(f"  {c:24s} {v[c] / mf:.3f} per MFMA")
    if "SQ_LDS_IDX_ACTIVE" in v:
        print(f"  LDS bank conflict cycles / LDS-array cycles {v['SQ_LDS_BANK_CONFLICT'] / v['SQ_LDS_IDX_ACTIVE']:.4f}")
    if "SQ_VALU_MFMA_COEXEC_CYCLES" in v:
        print(f"  VALU-MFMA co-exec cycles / MFMA busy {v['SQ_VALU_MFMA_COEXEC_CYCLES'] / v.get('SQ_VALU_MFMA_BUSY_CYCLES', 1):.3f}")
