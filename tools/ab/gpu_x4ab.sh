set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k x4 --timeout 200 --timeout-method thread > gpurun_out/t_x4.log 2>&1 || { tail -30 gpurun_out/t_x4.log; exit 1; }
tail -2 gpurun_out/t_x4.log
bash tools/ab/ab.sh x4 c128 old
