# round 6: factored P = 4 x 83 slow-time DFT in the tiled K1 -- reference-frame parity and timing
set -o pipefail
o=gpurun_out/r06b; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "reference" -x -v --timeout 300 --timeout-method thread > $o/gputest_ref.log 2>&1; rc=$?; tail -3 $o/gputest_ref.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --config reference --steps 20 --warmup 2 --no-cpu-baseline > $o/bench_ref.json 2> $o/bench_ref.err || exit $?
timeout -k 10 300 python3 bench.py --per-call --config reference --steps 50 --warmup 5 --no-cpu-baseline > $o/percall_ref.json 2> $o/percall_ref.err || exit $?
timeout -k 10 600 python -u -m pytest tests/test_music.py tests/test_k2_blocks.py -m gpu -x -v --timeout 120 --timeout-method thread > $o/gputest_music_k2.log 2>&1; rc=$?; tail -3 $o/gputest_music_k2.log; [ $rc -eq 0 ] || exit $rc
for f in $o/*.json; do cut -c1-300 $f; done
