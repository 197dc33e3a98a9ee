#!/bin/bash
# K2 iteration: x2/small/reference parity subset, then per-stage A/B against exp/ab variants.
# usage: tools/gpu_k2ab.sh variant...
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_amplitude_kat.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/t1.log 2>&1 || { tail -30 gpurun_out/t1.log; exit 1; }
tail -2 gpurun_out/t1.log
bash tools/ab/ab.sh x2 c128 "$@"
