"""Per-kernel launch durations from a rocprofv3 kernel-trace CSV, split by grid size
(separates the ref-window launches from the small alt-delta launches of the pair path)."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
d = collections.defaultdict(list)
for r in rows:
    n = r['Kernel_Name']
    dur = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6
    d[(n[:72], int(r['Grid_Size_X']))].append(dur)
tot = sum(sum(v) for v in d.values())
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1]))[:int(sys.argv[2]) if len(sys.argv) > 2 else 30]:
    print(f"{k[0]:72s} grid {k[1]:10d} n {len(v):3d} avg {sum(v) / len(v):7.3f} ms  {100 * sum(v) / tot:5.1f} %")
