# K2 row padding one complex per 64 (SH 6) and without the XOR swizzle, at 3 workgroups per CU
set -o pipefail
o=gpurun_out/r05ac; mkdir -p $o
bash tools/ab/gpu_ab_stages.sh $o 3 "x2:c128:50" base sh6 noxor || exit $?
