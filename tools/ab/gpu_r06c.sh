# round 6: persistent factored-DFT K1 (k1q_dbf_mtd) -- reference-frame parity, bit identity with the tiled K1, timing
set -o pipefail
o=gpurun_out/r06c; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "reference or profile_stages" -x -v --timeout 300 --timeout-method thread > $o/gputest_ref.log 2>&1; rc=$?; tail -3 $o/gputest_ref.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --config reference --steps 50 --warmup 2 --no-cpu-baseline > $o/bench_ref.json 2> $o/bench_ref.err || exit $?
timeout -k 10 300 python3 bench.py --per-call --config reference --steps 100 --warmup 5 --no-cpu-baseline > $o/percall_ref.json 2> $o/percall_ref.err || exit $?
timeout -k 10 300 python3 bench.py --per-call --config x2 --steps 300 --warmup 10 --no-cpu-baseline > $o/percall_x2.json 2> $o/percall_x2.err || exit $?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/prof_ref -o run -- python3 bench.py --config reference --steps 20 --warmup 2 --no-cpu-baseline > $o/prof_ref.log 2>&1 || exit $?
for f in $o/*.json; do cut -c1-300 $f; done
