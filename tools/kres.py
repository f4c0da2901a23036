#!/usr/bin/env python3
"""Per-kernel resource table (VGPRs, scratch, spills, LDS) of librsort's gfx950 code object.

    python tools/kres.py [substring ...]
"""
import re
import subprocess
import sys

SRC = "webgpu-radix-sort_amd/csrc/rsort.hip"
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden", "--offload-arch=gfx950",
       "-c", "-o", "/tmp/kres.o", SRC, "-Rpass-analysis=kernel-resource-usage"] + \
      [a for a in sys.argv[1:] if a.startswith("-D")]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
pats = [a for a in sys.argv[1:] if not a.startswith("-D")]
cur = None
rows = []
for line in out.splitlines():
    m = re.search(r"remark: Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"remark:\s+([A-Za-z \[\]/]+?):\s+(\S+)", line)
    if m and cur is not None:
        cur[m.group(1).strip()] = m.group(2)
for r in rows:
    n = subprocess.run(["c++filt", r["name"]], capture_output=True, text=True).stdout.strip()
    n = re.sub(r"\(.*", "", n).replace("rs::", "")
    if pats and not any(p in n for p in pats):
        continue
    print(f"{n:60s} vgpr={r.get('VGPRs','?'):>4} scratch={r.get('ScratchSize [bytes/lane]','?'):>5} "
          f"vspill={r.get('VGPRs Spill','?'):>4} lds={r.get('LDS Size [bytes/block]','?'):>6} occ={r.get('Occupancy [waves/SIMD]','?')}")
