#!/bin/bash
# A/B timing on one GPU box: per-stage HIP-event times of the shipped library and each variant
# (exp/ab/librsp_<name>.so, built by `make -C csrc ab NAME=<name> DEFS=...`), interleaved 3 rounds.
# usage: tools/ab.sh CONFIG PREC name...
set -o pipefail
cfg=$1; prec=$2; shift 2
mkdir -p gpurun_out
for round in 1 2 3; do
  for v in base "$@"; do
    if [ $v = base ]; then lib=""; else lib=exp/ab/librsp_$v.so; fi
    out=$(AB_LIB=$lib timeout -k 10 120 python3 tools/prof_stages.py $cfg 50 8 $prec) || exit $?
    echo "$round $v $out" | python3 -c 'import sys,json; r,v,j=sys.stdin.read().split(" ",2); print(r, v, " ".join("%s %.1f" % (s["stage"], s["ms"]*1e3) for s in json.loads(j)))' | tee -a gpurun_out/ab.log
  done
done
