#!/usr/bin/env python3
"""Per-launch durations (us) of the pass kernels from a rocprofv3 kernel_trace.csv, in launch
order, one line per sort:  python tools/trace_passes.py <kernel_trace.csv> [max_sorts]"""
import csv
import re
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
limit = int(sys.argv[2]) if len(sys.argv) > 2 else 20
line, sorts = [], 0
for r in rows:
    n = r["Kernel_Name"]
    m = re.search(r"rs::(k_\w+)(<[^(]*>)?", n)
    if not m or m.group(1) in ("k_fill_random", "k_fill_iota", "k_is_sorted"):
        continue
    us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    if m.group(1) in ("k_pass_totals",) and line:
        print(" ".join(line)); sorts += 1; line = []
        if sorts >= limit:
            break
    line.append(f"{m.group(1)[2:]}{(m.group(2) or '').replace(' ', '')}={us:.0f}")
if line and sorts < limit:
    print(" ".join(line))
