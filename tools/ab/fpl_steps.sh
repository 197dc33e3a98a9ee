set -o pipefail
for r in 1 2; do
for spec in "base 8" "f16 8" "f16 12" "f16 16"; do
  set -- $spec
  if [ $1 = base ]; then lib=""; else lib=exp/ab/librsp_$1.so; fi
  AB_LIB=$lib timeout -k 10 200 python3 -u tools/steps_sweep.py x2 c128 $2 > gpurun_out/fs_$1_$2.log 2>&1 || exit $?
  echo "$r $1 F=$2: $(grep back gpurun_out/fs_$1_$2.log | awk '{print $3":"$4}' | tr '\n' ' ')"
done; done
