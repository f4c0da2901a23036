#!/usr/bin/env python3
"""Per-kernel HBM traffic (FETCH_SIZE, WRITE_SIZE: separate rocprofv3 --pmc passes) of one
prof_driver.py workload, averaged per launch: a diagnostic for any kernel (tools/pmc_traffic.py
covers the bench line's kernels).  FETCH_SIZE is doubled (gfx950 reports half of a coalesced
read, MI355X_MICROARCH.md §HBM).  Runs rocprofv3 with the driver as a child process.

    python3 tools/r05/pmc_kernels.py config4 out.json
"""
import csv
import glob
import json
import os
import subprocess
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(counter, wl, outdir):
    d = os.path.join(outdir, counter.lower())
    cmd = ["rocprofv3", "--pmc", counter, "--output-format", "csv", "-d", d, "-o", "pmc", "--",
           sys.executable, os.path.join(ROOT, "tools", "prof_driver.py"), wl, "2"]
    subprocess.run(cmd, check=True, timeout=300, stdout=subprocess.DEVNULL)
    acc = defaultdict(lambda: [0.0, 0])
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0][:80]
            acc[k][0] += float(r["Counter_Value"])
            acc[k][1] += 1
    return {k: v[0] / max(v[1], 1) for k, v in acc.items()}


def main():
    wl = sys.argv[1]
    out = sys.argv[2]
    outdir = os.path.join(ROOT, "gpurun_out", "pmc_" + wl)
    fe = run("FETCH_SIZE", wl, outdir)
    wr = run("WRITE_SIZE", wl, outdir)
    rows = {k: {"read_MB": 2 * fe.get(k, 0) / 1024, "write_MB": wr.get(k, 0) / 1024} for k in set(fe) | set(wr)}
    json.dump(rows, open(out, "w"), indent=1, sort_keys=True)
    for k, v in sorted(rows.items(), key=lambda kv: -(kv[1]["read_MB"] + kv[1]["write_MB"]))[:25]:
        print(f'{v["read_MB"]:10.1f} {v["write_MB"]:10.1f}  {k}')


if __name__ == "__main__":
    main()
