#!/bin/bash
# Per-kernel VGPR / scratch / occupancy of rsp_kernels.hip (hipcc resource-usage remarks), one line each.
cd "$(dirname "$0")/../../radar-signal-simulation-and-target-detection_amd/csrc"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../../include -Wno-unused-function -x hip -c ${1:-rsp_kernels.hip} ${@:2} \
  -o /dev/null -Rpass-analysis=kernel-resource-usage 2>&1 | python3 -c '
import sys, re, subprocess
cur = None
rows = []
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        name = subprocess.run(["c++filt", m.group(1)], capture_output=True, text=True).stdout.strip()
        name = re.sub(r"\(anonymous namespace\)::", "", name).split("(")[0]
        cur = {"name": name}; rows.append(cur); continue
    for key, pat in (("vgpr", r"VGPRs: (\d+)"), ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)"), ("occ", r"Occupancy \[waves/SIMD\]: (\d+)")):
        m = re.search(pat, line)
        if m and cur is not None: cur[key] = m.group(1)
for r in rows:
    print("%-45s vgpr %4s scratch %4s occ %s" % (r["name"], r.get("vgpr"), r.get("scratch"), r.get("occ")))
'
