#!/bin/bash
# Fast GPU iteration: parity subset (-k expression) + per-stage HIP-event times of x2 (both precisions).
# usage: tools/ab/quick.sh [pytest -k expr]
set -o pipefail
mkdir -p gpurun_out
k=${1:-"x2 or small"}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "$k" > gpurun_out/quick_test.log 2>&1
rc=$?; tail -n 5 gpurun_out/quick_test.log
if [ $rc -ne 0 ]; then exit $rc; fi
for prec in c128 c64; do
  timeout -k 10 120 python3 tools/prof_stages.py x2 50 8 $prec | tee -a gpurun_out/quick_stages.log || exit $?
done
