# round 6 final evidence, part B: x2 profile round (500-step bench, kernel trace, FETCH/WRITE and
# SQ passes) and fresh PMC traffic files for x2 c64, x4, the reference frame and x2 --want-rdm
set -o pipefail
bash tools/profile_round.sh r06final x2 c128 --steps 500 || exit $?
for a in "x2 c64" "x4 c128" "reference c128" "x2 c128 rdm"; do
  echo "=== pmc $a"
  bash tools/pmc_pass.sh $a > /dev/null || exit $?
done
ls gpurun_out/pmc_*/
