# narrow-segment rows through per-row buffer windows: parity, then stage A/B
set -o pipefail
o=gpurun_out/r05z; mkdir -p $o
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_k2_blocks.py tests/test_queue_paths.py -m gpu -x -q --timeout 300 --timeout-method thread > $o/parity.log 2>&1; rc=$?; tail -3 $o/parity.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab/gpu_ab_stages.sh $o 3 "x2:c128:50 x4:c128:10" base nofirwin || exit $?
