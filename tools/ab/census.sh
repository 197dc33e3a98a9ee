#!/bin/bash
# Instruction census of one K2 job type (tools/ab/k2_census.hip; 1: 2560 block, 2: 1024 block) with
# extra defines: tools/ab/census.sh 1 [-DFOO=1 ...]
c=$1; shift
cd "$(dirname "$0")"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../../include -I../../radar-signal-simulation-and-target-detection_amd/csrc \
  -Wno-unused-function "$@" -x hip -S --cuda-device-only k2_census.hip -o /tmp/k2census.s 2>&1 | grep -v warning
python3 asm_counts.py /tmp/k2census.s "k2_census<$c>"
python3 - $c <<'PY'
import re, sys
s = open('/tmp/k2census.s').read()
for m in re.finditer(r'\.amdhsa_kernel (\S+)\n(.*?)\.end_amdhsa_kernel', s, re.S):
    if 'k2_censusILi%sE' % sys.argv[1] in m.group(1):
        b = m.group(2)
        print('   vgpr', re.search(r'next_free_vgpr (\d+)', b).group(1), 'scratch', re.search(r'private_segment_fixed_size (\d+)', b).group(1))
PY
