# round 6 final evidence, part A: the whole GPU suite
set -o pipefail
o=gpurun_out/r06final; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $o/gputest.log 2>&1; rc=$?
tail -5 $o/gputest.log
exit $rc
