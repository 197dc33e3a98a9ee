#!/bin/bash
# Interleaved per-stage A/B (HIP events, tools/prof_stages.py) over configs and variants.
# usage: tools/ab/gpu_ab_stages.sh OUTDIR ROUNDS "cfg:prec:iters ..." base name...
set -o pipefail
o=$1; rounds=$2; cfgs=$3; shift 3
mkdir -p $o
for round in $(seq 1 $rounds); do
  for c in $cfgs; do IFS=: read cfg prec it <<< "$c"
    for v in "$@"; do
      if [ $v = base ]; then lib=""; else lib=exp/ab/librsp_$v.so; fi
      out=$(AB_LIB=$lib timeout -k 10 150 python3 tools/prof_stages.py $cfg $it 8 $prec) || exit $?
      echo "$round $cfg $prec $v $out" | python3 -c 'import sys,json; r,c,p,v,j=sys.stdin.read().split(" ",4); print(r, c, p, v, " ".join("%s %.1f" % (s["stage"], s["ms"]*1e3) for s in json.loads(j)))' | tee -a $o/ab.log
    done
  done
done
