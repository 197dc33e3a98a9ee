set -o pipefail
# Round-end evidence on HEAD: GPU suite, smoke, x2 profile round, secondary lines with their PMC files.
export TMPDIR=/tmp
o=gpurun_out/r04f
mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/tests.log 2>&1; rc=$?; tail -3 $o/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit 1
cat $o/smoke.log
bash tools/profile_round.sh r04f x2 c128 --steps 500 || exit 1
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $o/bench_driver_cmd.json 2> $o/bench_driver_cmd.err || exit 1
bash tools/pmc_pass.sh x2 c128 rdm > /dev/null || exit 1
cp gpurun_out/pmc_x2_c128_rdm/pmc_traffic_x2_c128_rdm.json profiles/
timeout -k 10 300 python3 bench.py --want-rdm --steps 200 > $o/bench_rdm.json 2> $o/bench_rdm.err || exit 1
for c in "x4 c128" "x2 c64"; do set -- $c
  timeout -k 10 300 python3 bench.py --config $1 --precision $2 > $o/bench_$1_$2.json 2> $o/bench_$1_$2.err || exit 1
done
timeout -k 10 300 python3 bench.py --config music5 > $o/bench_music5.json 2> $o/bench_music5.err || exit 1
for f in $o/bench_*.json; do echo "$f $(cut -c1-160 $f)"; done
