# final tree: the full GPU suite, smoke, and the driver's bench command
set -o pipefail
o=gpurun_out/r05final; mkdir -p $o
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $o/gputest.log 2>&1; rc=$?; tail -3 $o/gputest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit $?
cat $o/smoke.log
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $o/bench_driver_cmd.json 2> $o/bench_driver_cmd.err || exit $?
cut -c1-220 $o/bench_driver_cmd.json
