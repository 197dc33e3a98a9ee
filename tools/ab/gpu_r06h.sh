# round 6: k1p with Atab in LDS for 16 beams (x4 without scratch); full GPU suite; x4 line
set -o pipefail
o=gpurun_out/r06h; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 1500 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $o/gputest.log 2>&1; rc=$?; tail -3 $o/gputest.log
timeout -k 10 300 python3 bench.py --config x4 --steps 20 --no-cpu-baseline > $o/bench_x4.json 2> $o/bench_x4.err || exit $?
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $o/bench_x2_driver_cmd.json 2> $o/bench_x2.err || exit $?
for f in $o/bench_*.json; do cut -c1-250 $f; done
exit $rc
