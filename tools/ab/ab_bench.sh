#!/bin/bash
# Interleaved A/B of whole-bench throughput: base library vs exp/ab/librsp_<name>.so, 3 rounds.
# usage: tools/ab_bench.sh "bench args" name...
set -o pipefail
args=$1; shift
mkdir -p gpurun_out
for round in 1 2 3; do
  for v in base "$@"; do
    if [ $v = base ]; then lib=base; else lib=exp/ab/librsp_$v.so; fi
    timeout -k 10 200 python3 tools/ab/ab_bench.py $lib $args | sed "s/^/$round /" | tee -a gpurun_out/ab_bench.log || exit $?
  done
done
