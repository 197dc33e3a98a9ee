#!/bin/bash
# Interleaved A/B of the queue's timed-region behaviour (tools/steps_sweep.py) for the shipped
# library and exp/ab/librsp_<name>.so variants, 2 rounds.   usage: tools/ab_steps.sh CONFIG PREC F name...
set -o pipefail
cfg=$1; prec=$2; F=$3; shift 3
mkdir -p gpurun_out
for round in 1 2; do
  for v in base "$@"; do
    if [ $v = base ]; then lib=""; else lib=exp/ab/librsp_$v.so; fi
    AB_LIB=$lib timeout -k 10 200 python3 -u tools/steps_sweep.py $cfg $prec $F > gpurun_out/ss_$v.log 2>&1 || exit $?
    grep -E "k=(20|320)|fit" gpurun_out/ss_$v.log | sed "s/^/$round $v /" | tee -a gpurun_out/ab_steps.log
  done
done
