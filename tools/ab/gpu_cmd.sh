set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r04i
mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/tests.log 2>&1; rc=$?; tail -3 $o/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit 1
cat $o/smoke.log
timeout -k 10 300 python3 bench.py > $o/bench.json 2> $o/bench.err || exit 1
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $o/bench_driver_cmd.json 2> $o/bench_driver_cmd.err || exit 1
timeout -k 10 300 python3 bench.py --config x4 --steps 100 --no-cpu-baseline > $o/bench_x4.json 2> $o/bench_x4.err || exit 1
for f in $o/bench*.json; do echo "$f $(cut -c1-200 $f)"; done
