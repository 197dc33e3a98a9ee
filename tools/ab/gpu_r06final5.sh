# round 6 closing rehearsal of the driver's round-end steps on the final tree: the GPU suite,
# smoke(), and bench.py with no flags
set -o pipefail
o=gpurun_out/r06final5; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/gputest.log 2>&1 || { tail -30 $o/gputest.log; exit 1; }
tail -2 $o/gputest.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { tail -20 $o/smoke.log; exit 1; }
tail -2 $o/smoke.log
timeout -k 10 300 python3 bench.py > $o/bench_default.json 2> $o/bench_default.err || { tail -20 $o/bench_default.err; exit 1; }
cat $o/bench_default.json
