#!/bin/bash
# Full GPU check: every gpu test (one process), smoke(), then the x2 bench (driver's command).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/full_test.log 2>&1 || { tail -40 gpurun_out/full_test.log; exit 1; }
tail -3 gpurun_out/full_test.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/bench_driver.json 2> gpurun_out/bench_driver.err || { tail -20 gpurun_out/bench_driver.err; exit 1; }
tail -1 gpurun_out/bench_driver.json | cut -c1-400
