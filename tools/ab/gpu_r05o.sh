# K2 1024-point blocks as 8 x 16 x 8 in the 3-per-CU plans: parity, then stage + bench A/B vs 16 x 4 x 16
set -o pipefail
o=gpurun_out/r05o; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_queue_paths.py -m gpu -x -q --timeout 300 --timeout-method thread > $o/parity.log 2>&1; rc=$?; tail -3 $o/parity.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab/gpu_ab_stages.sh $o 3 "x2:c128:50" base m16 || exit $?
bash tools/ab/ab_bench.sh "--steps 300" m16 || exit $?
