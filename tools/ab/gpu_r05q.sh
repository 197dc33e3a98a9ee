# x4 K1 with the second MFMA row block's operands re-read per sub-tile (no scratch): A/B
set -o pipefail
o=gpurun_out/r05q; mkdir -p $o
bash tools/ab/gpu_ab_stages.sh $o 3 "x4:c128:10" base arel || exit $?
