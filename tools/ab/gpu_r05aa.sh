# K1: the next tile's sub-tile u - 1 issued right after sub-tile u's MFMAs (complex double too)
set -o pipefail
o=gpurun_out/r05aa; mkdir -p $o
bash tools/ab/gpu_ab_stages.sh $o 3 "x2:c128:50 x2:c64:50" base lag || exit $?
bash tools/ab/ab_bench.sh "--steps 300" lag || exit $?
