#!/bin/bash
# Round-3 secondary bench lines: complex single, config #3 (512 frames, 1 GPU), end to end.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/lines
timeout -k 10 300 python3 bench.py --precision c64 > gpurun_out/lines/c64.json 2> gpurun_out/lines/c64.err || exit $?
timeout -k 10 300 python3 bench.py --frames-total 512 > gpurun_out/lines/config3.json 2> gpurun_out/lines/config3.err || exit $?
timeout -k 10 300 python3 bench.py --e2e --steps 100 --no-cpu-baseline > gpurun_out/lines/e2e.json 2> gpurun_out/lines/e2e.err || exit $?
for f in c64 config3 e2e; do tail -1 gpurun_out/lines/$f.json | cut -c1-200; done
