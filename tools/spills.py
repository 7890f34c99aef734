"""Where a kernel in a -save-temps .s file touches scratch: line offsets and the branch labels
around them (loop bodies are the blocks with backward branches).  Usage: spills.py file.s symbol"""
import re
import sys

s = open(sys.argv[1]).read()
name = sys.argv[2]
a = s.index(name + ':')
b = s.index('.Lfunc_end', a)
f = s[a:b].split('\n')
lbl = {l.rstrip(':'): i for i, l in enumerate(f) if re.match(r'\.LBB\d+_\d+:', l)}
sc = [i for i, l in enumerate(f) if 'scratch_' in l]
print(len(f), 'lines; scratch ops at', sc)
for i, l in enumerate(f):
    m = re.search(r's_c?branch\w*\s+(\.LBB\d+_\d+)', l)
    if m and m.group(1) in lbl and lbl[m.group(1)] < i:
        n_sc = sum(1 for j in sc if lbl[m.group(1)] <= j <= i)
        print(f'loop {m.group(1)} lines {lbl[m.group(1)]}..{i}: {n_sc} scratch ops inside')
