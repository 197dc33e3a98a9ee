# round 6: k1q with loader / store wave roles (RQ_RK = 4)
set -o pipefail
o=gpurun_out/r06k; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "reference" -v --timeout 300 --timeout-method thread > $o/gputest_ref.log 2>&1; rc=$?; tail -3 $o/gputest_ref.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --config reference --steps 50 --warmup 2 --no-cpu-baseline > $o/bench_ref.json 2> $o/bench_ref.err || exit $?
cut -c1-300 $o/bench_ref.json
