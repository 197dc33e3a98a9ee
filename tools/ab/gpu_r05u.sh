# K2 2560-point blocks with the filter spectrum loaded before the fused pass's forward DFT: A/B
set -o pipefail
o=gpurun_out/r05u; mkdir -p $o
bash tools/ab/gpu_ab_stages.sh $o 3 "x2:c128:50" base hearly || exit $?
