#!/usr/bin/env python3
"""SQ (and TCC request) counters per kernel of one workload, from rocprofv3 PMC passes (GPU box).

One `rocprofv3 --pmc` pass per counter group (each group within the per-block limits of
MI355X_MICROARCH.md: at most 8 SQ_, 4 TCC_ counters), each under its own SIGKILL limit, over
tools/prof_driver.py's sorts.  Per kernel of interest (the MSD pass, the bucket sort, the 16-bit
histogram, the keys-only one-sweep pass) the counters are summed over its launches and reported
per launch, with the derived fractions DESIGN.md §5 cites: SQ_WAIT_ANY / SQ_WAVE_CYCLES (waves
parked on s_waitcnt / barriers), SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES (issue stalls), LDS bank
conflicts per LDS instruction, and TCC write requests by size.

    python3 tools/pmc_sq.py [config3|config2] [out_dir]    ->  <out_dir>/summary.json

This script never touches the GPU itself: rocprofv3 runs tools/prof_driver.py as a child.
"""
import csv
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GROUPS = {
    "cycles": ["SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_BUSY_CYCLES"],
    "active": ["SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_SALU", "SQ_ACTIVE_INST_VMEM",
               "SQ_WAIT_INST_LDS"],
    "lds": ["SQ_LDS_BANK_CONFLICT", "SQ_LDS_ADDR_CONFLICT", "SQ_LDS_IDX_ACTIVE", "SQ_INSTS_LDS"],
    "insts": ["SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_WAVES"],
    "tcc_wr": ["TCC_EA0_WRREQ_sum", "TCC_EA0_WRREQ_64B_sum"],
    "tcc_rd": ["TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_32B_sum"],
}
KERNELS = {"k_msd_pass": "msd_pass", "k_bucket_sort<": "bucket_sort", "k_bucket_sort_wide": "bucket_wide",
           "k_hist16_in": "hist16_in",
           "k_onesweep<8, 512, 32": "onesweep_keys", "k_bucket_sort_keys_wave": "bucket_keys_wave"}


def kernel_key(name: str):
    for pat, key in KERNELS.items():
        if pat in name:
            return key
    return None


def run_group(wl: str, outdir: str, group: str, counters: list) -> dict:
    d = os.path.join(outdir, group)
    cmd = ["timeout", "-s", "KILL", "120", "rocprofv3", "--pmc"] + counters + [
        "--output-format", "csv", "-d", d, "-o", "p", "--",
        sys.executable, os.path.join(ROOT, "tools", "prof_driver.py"), wl, "2"]
    rc = subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL).returncode
    acc = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = kernel_key(r["Kernel_Name"])
            if k is None:
                continue
            e = acc.setdefault(k, {"dispatches": set()})
            e["dispatches"].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
            e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    out = {}
    for k, e in acc.items():
        nd = max(1, len(e.pop("dispatches")))
        out[k] = {c: v / nd for c, v in e.items()}
        out[k]["launches"] = nd
    return {"rc": rc, "kernels": out}


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "config3"
    outdir = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "gpurun_out", "pmc_sq_" + wl)
    os.makedirs(outdir, exist_ok=True)
    per = {}
    status = {}
    for g, cs in GROUPS.items():
        r = run_group(wl, outdir, g, cs)
        status[g] = r["rc"]
        for k, v in r["kernels"].items():
            per.setdefault(k, {}).update(v)
        if r["rc"] not in (0,):
            break   # a pass that failed or was killed: stop (nothing more on the GPU in this call)
    summary = {"workload": wl, "status": status, "per_launch": per, "derived": {}}
    for k, c in per.items():
        d = {}
        wc = c.get("SQ_WAVE_CYCLES")
        if wc:
            for nm in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                       "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VMEM", "SQ_WAIT_INST_LDS"):
                if nm in c:
                    d[nm.lower() + "_frac"] = round(c[nm] / wc, 4)
        if c.get("SQ_INSTS_LDS"):
            d["lds_bank_conflicts_per_lds_inst"] = round(c.get("SQ_LDS_BANK_CONFLICT", 0.0) / c["SQ_INSTS_LDS"], 3)
            d["lds_addr_conflicts_per_lds_inst"] = round(c.get("SQ_LDS_ADDR_CONFLICT", 0.0) / c["SQ_INSTS_LDS"], 3)
        if c.get("TCC_EA0_WRREQ_sum"):
            d["write_requests_64B_frac"] = round(c.get("TCC_EA0_WRREQ_64B_sum", 0.0) / c["TCC_EA0_WRREQ_sum"], 4)
        if c.get("TCC_EA0_RDREQ_sum"):
            d["read_requests_32B_frac"] = round(c.get("TCC_EA0_RDREQ_32B_sum", 0.0) / c["TCC_EA0_RDREQ_sum"], 4)
        summary["derived"][k] = d
    with open(os.path.join(outdir, "summary.json"), "w") as f:
        json.dump(summary, f, indent=1)
    print(json.dumps(summary["derived"]))


if __name__ == "__main__":
    main()
