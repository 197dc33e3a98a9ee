# MUSIC eigensolver sized for 3 waves per SIMD (161 VGPRs, no scratch) vs 4 (128 + 52 B scratch)
set -o pipefail
o=gpurun_out/r05af; mkdir -p $o
for i in 1 2 3; do
  for v in base wps3; do
    if [ $v = base ]; then lib=""; else lib=exp/ab/librsp_$v.so; fi
    AB_LIB=$lib timeout -k 10 120 python3 tools/music_prof.py 4096 | sed "s/^/$i $v /" | tee -a $o/ab.log || exit $?
  done
done
