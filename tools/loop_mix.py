"""Instruction mix of the hottest basic block(s) (most MFMAs) of one kernel in a .s file.

    python tools/loop_mix.py file.s kernel-substring [min_mfma]"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
pat = sys.argv[2]
lim = int(sys.argv[3]) if len(sys.argv) > 3 else 50
for m in re.finditer(r"^(_Z\S+):\s*;", s, re.M):
    if pat not in m.group(1):
        continue
    end = s.index(".Lfunc_end", m.end())
    for b in re.split(r"\n(?=\.LBB)", s[m.end():end]):
        if len(re.findall("v_mfma", b)) < lim:
            continue
        c = collections.Counter()
        for line in b.split("\n"):
            line = line.split(";")[0].strip()
            if line and not line.startswith("."):
                c[line.split()[0]] += 1
        print(m.group(1), b.split("\n")[0][:30])
        for k, v in c.most_common(30):
            print(f"{v:6d} {k}")
