# round 6: kernel trace of the per-call bench (x2) on the current tree: host gaps between calls
set -o pipefail
o=gpurun_out/r06v; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $o/trace -o run -- python3 bench.py --per-call --config x2 --steps 100 --warmup 5 --no-cpu-baseline > $o/trace.log 2>&1 || exit $?
