set -o pipefail
o=gpurun_out/r05e; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_k3_prefilter.py -x -q --timeout 300 --timeout-method thread > $o/parity.log 2>&1; rc=$?; tail -3 $o/parity.log; [ $rc -eq 0 ] || exit $rc
for prec in c128 c64; do timeout -k 10 120 python3 tools/prof_stages.py x2 50 8 $prec | tee -a $o/stages.log || exit 1; done
timeout -k 10 120 python3 tools/prof_stages.py x4 10 8 c128 | tee -a $o/stages.log || exit 1
timeout -k 10 240 python3 bench.py --steps 500 --no-cpu-baseline > $o/bench.json 2> $o/bench.err || exit 1
cut -c1-200 $o/bench.json
