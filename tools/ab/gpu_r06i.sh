# round 6: MUSIC eigensolver phase stamps (diagnostic build) for the three forms of call
set -o pipefail
o=gpurun_out/r06i; mkdir -p $o
for w in peaks spectrum eigenvalues; do
  AB_LIB=exp/ab/librsp_diag.so RSP_MUSIC_TRACE=1 timeout -k 10 120 python3 tools/music_prof.py 4096 3 c128 $w > $o/music_phases_$w.txt 2>&1 || exit $?
  cat $o/music_phases_$w.txt
done
