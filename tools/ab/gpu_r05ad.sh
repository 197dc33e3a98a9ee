# K2 2560-point workgroups at raised wave priority until their loads are issued
set -o pipefail
o=gpurun_out/r05ad; mkdir -p $o
bash tools/ab/gpu_ab_stages.sh $o 3 "x2:c128:50" base prio || exit $?
