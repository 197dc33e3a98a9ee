#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (separate rocprofv3 runs) of the stage driver -> the traffic json
# bench.py reads (profiles/pmc_traffic_<cfg>_<prec>[_rdm].json).  usage: tools/pmc_pass.sh CFG PREC [rdm]
# (rdm: K2 also writes the complex RD map, the bench's --want-rdm workload)
set -o pipefail
cfg=$1; prec=$2; rdm=$3; sfx=${rdm:+_$rdm}; out=gpurun_out/pmc_${cfg}_${prec}$sfx
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/fetch -o run -- python3 tools/prof_stages.py $cfg 10 8 $prec $rdm > $out/fetch.log 2>&1 || exit $?
timeout -k 10 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/write -o run -- python3 tools/prof_stages.py $cfg 10 8 $prec $rdm > $out/write.log 2>&1 || exit $?
python3 tools/pmc_traffic.py $out/fetch $out/write $out/pmc_traffic_${cfg}_${prec}$sfx.json $cfg 10 8
