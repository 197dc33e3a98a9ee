# round 6: per-call host gap -- harvest by spinning on hipEventQuery (RSP_HARVEST_SPIN) vs hipEventSynchronize
set -o pipefail
o=gpurun_out/r06w; mkdir -p $o
export TMPDIR=/tmp
for r in 1 2 3; do
  for v in base spin; do
    if [ $v = base ]; then lib=""; else lib=exp/ab/librsp_$v.so; fi
    echo "$r $v $(AB_LIB=$lib timeout -k 10 120 python3 tools/ab/percall_breakdown.py x2 300)" | tee -a $o/ab.log || exit 1
  done
done
