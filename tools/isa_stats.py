"""Instruction counts and resource usage per kernel from a hipcc -save-temps .s file.

    python tools/isa_stats.py file.s [name-substring]"""
import re
import sys

s = open(sys.argv[1]).read()
pat = sys.argv[2] if len(sys.argv) > 2 else ""
for m in re.finditer(r"^(_Z\S+):\s*;", s, re.M):
    name = m.group(1)
    if pat not in name:
        continue
    end = s.index(".Lfunc_end", m.end())
    body = s[m.end():end]
    print(name, "lines", body.count("\n"))
    for k in ["v_mfma", "global_load_lds", "global_load", "ds_read_b128", "ds_read", "ds_write", "s_waitcnt",
              "s_barrier", "v_cvt", "scratch_", "v_accvgpr_read", "v_accvgpr_write", "s_cbranch"]:
        print(f"   {k:18s} {len(re.findall(k, body))}")
    i = s.index(".amdhsa_kernel " + name)
    meta = s[i:i + 4000]
    for k in ["next_free_vgpr", "accum_offset", "group_segment_fixed_size", "private_segment_fixed_size"]:
        mm = re.search(r"\.amdhsa_" + k + r" (\d+)", meta)
        print(f"   {k:26s} {mm and mm.group(1)}")
