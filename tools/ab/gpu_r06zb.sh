# round 6: the new GPU tests (64-target synthesis, small-N spectrum calls) with their files
set -o pipefail
o=gpurun_out/r06zb; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_music.py > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -2 $o/tests.log
