# persistent 3-per-CU K2 (k2_pcp): parity, then stage + bench A/B vs the launch-per-item form and HEAD
set -o pipefail
o=gpurun_out/r05r; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_queue_paths.py tests/test_detection_capacity.py -m gpu -x -q --timeout 300 --timeout-method thread > $o/parity.log 2>&1; rc=$?; tail -3 $o/parity.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab/gpu_ab_stages.sh $o 3 "x2:c128:50" base nopers old || exit $?
bash tools/ab/ab_bench.sh "--steps 300" nopers old || exit $?
