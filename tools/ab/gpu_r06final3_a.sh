# round 6, K2 at 4 workgroups per CU shipped: the whole GPU suite, the x2 profile round (500-step
# bench, kernel trace, FETCH/WRITE and SQ passes) and fresh PMC traffic for every file holding k2_pc
set -o pipefail
o=gpurun_out/r06final3; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/gputest.log 2>&1 || { tail -30 $o/gputest.log; exit 1; }
tail -2 $o/gputest.log
bash tools/profile_round.sh r06final3 x2 c128 --steps 500 || exit $?
for a in "x2 c64" "x4 c128" "reference c128" "x2 c128 rdm"; do
  echo "=== pmc $a"
  bash tools/pmc_pass.sh $a > /dev/null || exit $?
done
ls gpurun_out/pmc_*/
