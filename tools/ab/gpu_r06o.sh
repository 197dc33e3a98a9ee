# round 6: synthesis with 32-bit index math -- synthesis parity + per-call breakdown
set -o pipefail
o=gpurun_out/r06o; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_golden.py tests/test_queue_paths.py > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -2 $o/tests.log
timeout -k 10 200 python3 tools/ab/percall_breakdown.py x2 200 > $o/percall_breakdown_x2.txt 2>&1 || exit $?
timeout -k 10 200 python3 tools/ab/percall_breakdown.py reference 50 > $o/percall_breakdown_ref.txt 2>&1 || exit $?
cat $o/percall_breakdown_*.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $o/trace -o run -- python3 tools/ab/percall_breakdown.py x2 50 > $o/trace.log 2>&1 || exit $?
