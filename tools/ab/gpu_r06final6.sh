# round 6 final: the profile round of the x4 line (kernel trace + stats, FETCH/WRITE and SQ passes)
# and of the reference frame on the final tree
set -o pipefail
export TMPDIR=/tmp
bash tools/profile_round.sh r06final4_x4 x4 c128 || exit $?
bash tools/profile_round.sh r06final4_ref reference c128 || exit $?
