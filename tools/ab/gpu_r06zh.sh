# round 6: K2 with the RD map written (--want-rdm), buffer-resource twiddles (shipped) vs 64-bit
# twiddle addresses (notw = the previous commit's kernels), 3 interleaved rounds, x2 c128 rdm
set -o pipefail
o=gpurun_out/r06zh; mkdir -p $o
export TMPDIR=/tmp
for round in 1 2 3; do
  for v in base notw; do
    if [ $v = base ]; then lib=""; else lib=exp/ab/librsp_$v.so; fi
    out=$(AB_LIB=$lib timeout -k 10 120 python3 tools/prof_stages.py x2 50 8 c128 rdm) || exit $?
    echo "$round $v $out" | python3 -c 'import sys,json; r,v,j=sys.stdin.read().split(" ",2); print(r, v, " ".join("%s %.1f" % (s["stage"], s["ms"]*1e3) for s in json.loads(j)))' | tee -a $o/ab_rdm.log
  done
done
