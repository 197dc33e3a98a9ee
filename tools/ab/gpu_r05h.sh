set -o pipefail
o=gpurun_out/r05h; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/gputest.log 2>&1; rc=$?; tail -3 $o/gputest.log; [ $rc -eq 0 ] || exit $rc
for round in 1 2 3; do
  for v in base exp/ab/librsp_old.so; do
    timeout -k 10 200 python3 tools/ab/ab_bench.py $v --steps 300 | sed "s/^/$round /" | tee -a $o/ab_bench.log || exit 1
  done
done
