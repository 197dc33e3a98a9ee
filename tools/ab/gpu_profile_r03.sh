#!/bin/bash
# Round-3 evidence: x2 and x4 profile rounds (bench line, kernel trace + stats, traffic, SQ counters),
# MUSIC (config #5, complex double) bench + trace.  Outputs under gpurun_out/.
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r03b}
bash tools/profile_round.sh ${tag}x2 x2 c128 || exit $?
bash tools/profile_round.sh ${tag}x4 x4 c128 --steps 200 --warmup 10 || exit $?
mkdir -p gpurun_out/${tag}music
timeout -k 10 240 python3 bench.py --config music5 > gpurun_out/${tag}music/bench.json 2> gpurun_out/${tag}music/bench.err || exit $?
tail -1 gpurun_out/${tag}music/bench.json | cut -c1-300
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}music/trace -o run -- python3 bench.py --config music5 --no-cpu-baseline > gpurun_out/${tag}music/trace.log 2>&1 || exit $?
echo done
