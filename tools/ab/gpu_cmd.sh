set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04p
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04p/tests.log 2>&1; rc=$?; tail -2 gpurun_out/r04p/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1 || exit 1
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r04p/bench_driver_cmd.json 2> gpurun_out/r04p/bench_driver_cmd.err || exit 1
cut -c1-200 gpurun_out/r04p/bench_driver_cmd.json
