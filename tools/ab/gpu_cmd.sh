set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_queue_paths.py -x -q --timeout 200 --timeout-method thread -k "x2 or small or p256 or rdm or x4" > gpurun_out/par.log 2>&1; rc=$?; tail -3 gpurun_out/par.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab/ab.sh x2 c128 nowl p3072 || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl_base -o run -- python3 bench.py --steps 100 --no-cpu-baseline > gpurun_out/tl_base.json 2>gpurun_out/tl_base.err || exit 1
python3 tools/timeline.py gpurun_out/tl_base
