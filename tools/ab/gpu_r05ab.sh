# K3 tile loads through buffer resources (branch-free): parity, then stage + bench A/B
set -o pipefail
o=gpurun_out/r05ab; mkdir -p $o
timeout -k 10 800 python -u -m pytest tests/test_gpu_parity.py tests/test_k3_prefilter.py tests/test_detection_capacity.py tests/test_k2_blocks.py -m gpu -x -q --timeout 300 --timeout-method thread > $o/parity.log 2>&1; rc=$?; tail -3 $o/parity.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab/gpu_ab_stages.sh $o 3 "x2:c128:50 x2:c64:50 x4:c128:10" base k3old || exit $?
