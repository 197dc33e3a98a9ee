# round 6: 4096-point overlap-save blocks (x4 long segment: 2 blocks instead of 5 x 2048)
set -o pipefail
o=gpurun_out/r06l; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_k2_blocks.py -m gpu -k "x4 or reference or k2_block" -v --timeout 300 --timeout-method thread > $o/gputest.log 2>&1; rc=$?; tail -3 $o/gputest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --config x4 --steps 20 --no-cpu-baseline > $o/bench_x4.json 2> $o/bench_x4.err || exit $?
timeout -k 10 300 python3 bench.py --config reference --steps 50 --warmup 2 --no-cpu-baseline > $o/bench_ref.json 2> $o/bench_ref.err || exit $?
for f in $o/bench_*.json; do cut -c1-250 $f; done
