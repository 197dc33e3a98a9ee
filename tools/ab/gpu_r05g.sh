set -o pipefail
o=gpurun_out/r05g; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_k3_prefilter.py tests/test_monopulse_complex.py -x -q --timeout 300 --timeout-method thread > $o/parity.log 2>&1; rc=$?; tail -3 $o/parity.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab/gpu_ab_stages.sh $o 2 "x2:c128:50 p256:c128:20 x4:c128:10" base m4k old || exit 1
