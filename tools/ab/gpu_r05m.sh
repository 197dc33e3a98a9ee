# round-5 HEAD check: the full GPU suite, smoke, and the secondary bench lines
set -o pipefail
o=gpurun_out/r05m; mkdir -p $o
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $o/gputest.log 2>&1; rc=$?; tail -3 $o/gputest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit $?
cat $o/smoke.log
timeout -k 10 300 python3 bench.py --config music5 > $o/bench_music5.json 2> $o/bench_music5.err || exit $?
timeout -k 10 300 python3 bench.py --config x4 --steps 20 > $o/bench_x4.json 2> $o/bench_x4.err || exit $?
timeout -k 10 240 python3 bench.py --precision c64 --steps 500 > $o/bench_c64.json 2> $o/bench_c64.err || exit $?
timeout -k 10 240 python3 bench.py --want-rdm --steps 500 > $o/bench_want_rdm.json 2> $o/bench_want_rdm.err || exit $?
timeout -k 10 240 python3 tools/ab/steps_sweep.py x2 c128 8 > $o/steps_sweep.txt 2>&1 || exit $?
for f in $o/bench_*.json; do cut -c1-160 $f; done
