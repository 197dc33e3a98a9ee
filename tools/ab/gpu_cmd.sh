set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r04m
mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/tests.log 2>&1; rc=$?; tail -3 $o/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --precision c64 > $o/bench_c64.json 2> $o/bench_c64.err || exit 1
timeout -k 10 300 python3 bench.py --steps 300 --no-cpu-baseline > $o/bench.json 2> $o/bench.err || exit 1
for f in $o/bench*.json; do echo "$f $(cut -c1-200 $f)"; done
