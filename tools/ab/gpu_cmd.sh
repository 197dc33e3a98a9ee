set -o pipefail
# Round evidence on HEAD: GPU suite, smoke, x2 profile round, secondary bench lines.
export TMPDIR=/tmp
o=gpurun_out/r04c
mkdir -p $o
timeout -k 10 200 python3 tools/ab/c64_cells.py x2 c64 cfar 2>&1 | head -8
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/tests.log 2>&1; rc=$?; tail -3 $o/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit 1
cat $o/smoke.log
bash tools/profile_round.sh r04c x2 c128 --steps 500 || exit 1
for c in "x4 c128" "x2 c64"; do set -- $c
  timeout -k 10 300 python3 bench.py --config $1 --precision $2 > $o/bench_$1_$2.json 2> $o/bench_$1_$2.err || exit 1
  cut -c1-300 $o/bench_$1_$2.json
done
timeout -k 10 300 python3 bench.py --want-rdm --steps 200 > $o/bench_rdm.json 2> $o/bench_rdm.err || exit 1
timeout -k 10 300 python3 bench.py --config music5 > $o/bench_music5.json 2> $o/bench_music5.err || exit 1
cut -c1-300 $o/bench_rdm.json $o/bench_music5.json
bash tools/pmc_pass.sh x4 c128 || exit 1
