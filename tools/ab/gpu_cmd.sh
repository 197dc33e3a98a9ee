set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_monopulse_complex.py -x -v -m gpu --timeout 300 --timeout-method thread 2>&1 | grep -E "PASS|FAIL|Error|assert|passed|failed" | head -20
