"""Summarise rocprofv3 --pmc counter CSVs per kernel (average per dispatch).

FETCH_SIZE / WRITE_SIZE are in KB.  On gfx950 FETCH_SIZE reads half the bytes of wide
coalesced streaming reads (MI355X_MICROARCH.md "HBM"); hbm_bytes_est doubles it."""
import csv, sys
rows = {}
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        rows.setdefault((k, r["Counter_Name"]), []).append(float(r["Counter_Value"]))
w = csv.writer(sys.stdout)
w.writerow(["kernel", "counter", "dispatches", "avg_value_KB", "avg_bytes_est"])
for (k, c), v in sorted(rows.items(), key=lambda kv: -sum(kv[1]) / len(kv[1])):
    avg = sum(v) / len(v)
    est = avg * 1024 * (2 if c == "FETCH_SIZE" else 1)
    w.writerow([k, c, len(v), f"{avg:.1f}", f"{est:.4g}"])
