#!/bin/bash
# GPU profiling pass for the round's evidence (run on the GPU box through gpurun):
#   the bench line, a kernel trace + stats of the same bench command, FETCH_SIZE / WRITE_SIZE
#   passes -> traffic json, and SQ counter passes of the stage driver.  Everything lands in
#   gpurun_out/prof_<tag>/.
# usage: tools/profile_round.sh TAG CONFIG PREC [bench args...]     (PREC = c128 | c64)
set -o pipefail
tag=$1; cfg=$2; prec=$3; shift 3
out=gpurun_out/prof_$tag
mkdir -p $out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name"
  timeout -k 10 $to "$@" > $out/$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 4 $out/$name.log
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step bench 240 python3 bench.py --config $cfg --precision $prec "$@"
cp $out/bench.log $out/bench.json
step trace 240 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 bench.py --config $cfg --precision $prec --no-cpu-baseline "$@"
step fetch 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/fetch -o run -- python3 tools/prof_stages.py $cfg 10 8 $prec
step write 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/write -o run -- python3 tools/prof_stages.py $cfg 10 8 $prec
python3 tools/pmc_traffic.py $out/fetch $out/write $out/pmc_traffic_${cfg}_${prec}.json $cfg 10 8 > /dev/null
step sqa 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $out/sqa -o run -- python3 tools/prof_stages.py $cfg 10 8 $prec
step sqb 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d $out/sqb -o run -- python3 tools/prof_stages.py $cfg 10 8 $prec
python3 tools/pmc_summary.py $out/sqa $out/sqb > $out/sq_summary.txt
cat $out/sq_summary.txt
find $out/trace -name '*kernel_stats.csv' -exec cp {} $out/kernel_stats.csv \;
python3 tools/rocprof_split.py $out/trace 50 $out/kernel_legs.csv
cp $out/trace.log $out/bench_under_rocprof.log
