# round 6 baseline: the reference frame (P = 332, O(P^2) DFT K1) and per-call latency lines before the change
set -o pipefail
o=gpurun_out/r06a; mkdir -p $o
timeout -k 10 300 python3 bench.py --per-call --config x2 --steps 200 --warmup 10 --no-cpu-baseline > $o/percall_x2.json 2> $o/percall_x2.err || exit $?
timeout -k 10 300 python3 bench.py --per-call --config reference --steps 50 --warmup 5 --no-cpu-baseline > $o/percall_ref.json 2> $o/percall_ref.err || exit $?
timeout -k 10 400 python3 bench.py --config reference --steps 10 --warmup 2 --no-cpu-baseline > $o/bench_ref.json 2> $o/bench_ref.err || exit $?
for f in $o/*.json; do cut -c1-400 $f; done
timeout -k 10 600 python -u -m pytest tests/test_music.py tests/test_k2_blocks.py -m gpu -x -v --timeout 120 --timeout-method thread > $o/gputest_music_k2.log 2>&1; rc=$?; tail -3 $o/gputest_music_k2.log; exit $rc
