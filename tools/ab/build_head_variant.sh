#!/bin/bash
# Build exp/ab/librsp_<name>.so from the kernels/plan sources of git revision REV (default HEAD),
# against the current headers and host objects: the "before" side of an A/B (tools/ab.sh).
# usage: tools/ab/build_head_variant.sh NAME [REV]
set -e
name=$1; rev=${2:-HEAD}
C=radar-signal-simulation-and-target-detection_amd/csrc
d=/tmp/rsp_variant_$name
rm -rf $d && mkdir -p $d exp/ab
for f in rsp_kernels.hip rsp_plan.cpp rsp_internal.h; do git show $rev:$C/$f > $d/$f; done
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Iinclude -I$d -Wall -Wno-unused-function"
/opt/rocm/bin/hipcc $F -x hip -c $d/rsp_kernels.hip -o $d/k.o &
/opt/rocm/bin/hipcc $F -x hip -c $d/rsp_plan.cpp -o $d/p.o &
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o exp/ab/librsp_$name.so $d/k.o $d/p.o $C/build/rsp_music.hip.o $C/build/rsp_mat.cpp.o $C/build/rsp_host.cpp.o -lz -lpthread
echo built exp/ab/librsp_$name.so from $rev
