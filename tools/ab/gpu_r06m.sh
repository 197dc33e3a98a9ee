# round 6: per-call latency breakdown + kernel trace of the per-call bench
set -o pipefail
o=gpurun_out/r06m; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 200 python3 tools/ab/percall_breakdown.py x2 200 > $o/percall_breakdown_x2.txt 2>&1 || exit $?
timeout -k 10 200 python3 tools/ab/percall_breakdown.py reference 50 > $o/percall_breakdown_ref.txt 2>&1 || exit $?
cat $o/percall_breakdown_*.txt
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $o/trace -o run -- python3 bench.py --per-call --config x2 --steps 50 --warmup 5 --no-cpu-baseline > $o/trace.log 2>&1 || exit $?
