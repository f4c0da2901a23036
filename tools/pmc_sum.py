#!/usr/bin/env python3
"""Sum rocprofv3 --pmc counters per kernel (short name) over a counter_collection.csv.
python tools/pmc_sum.py <dir-with-counter_collection.csv> [name_filter]"""
import csv
import glob
import re
import sys
from collections import defaultdict

agg = defaultdict(lambda: defaultdict(float))
calls = defaultdict(set)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        m = re.search(r"rs::(k_\w+)(<[^(]*>)?", r["Kernel_Name"])
        if not m:
            continue
        name = m.group(1) + (m.group(2) or "").replace(" ", "")
        if len(sys.argv) > 2 and sys.argv[2] not in name:
            continue
        agg[name][r["Counter_Name"]] += float(r["Counter_Value"])
        calls[name].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
for name, cs in agg.items():
    n = max(1, len(calls[name]))
    print(name, f"dispatches={n}", " ".join(f"{k}={v / n:.4g}" for k, v in sorted(cs.items())))
