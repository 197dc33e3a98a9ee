#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (separate rocprofv3 runs) of the stage driver -> the traffic json
# bench.py reads (profiles/pmc_traffic_<cfg>_<prec>.json).  usage: tools/pmc_pass.sh CFG PREC
set -o pipefail
cfg=$1; prec=$2; out=gpurun_out/pmc_${cfg}_${prec}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/fetch -o run -- python3 tools/prof_stages.py $cfg 10 8 $prec > $out/fetch.log 2>&1 || exit $?
timeout -k 10 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/write -o run -- python3 tools/prof_stages.py $cfg 10 8 $prec > $out/write.log 2>&1 || exit $?
python3 tools/pmc_traffic.py $out/fetch $out/write $out/pmc_traffic_${cfg}_${prec}.json $cfg 10 8
