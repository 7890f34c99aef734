"""Stand-in for natsort.natsorted (default key: digit runs compare as integers)."""
import re


def natsorted(items):
    key = lambda s: [(0, int(t), "") if t.isdigit() else (1, 0, t) for t in re.split(r"(\d+)", str(s)) if t != ""]
    return sorted(items, key=key)
