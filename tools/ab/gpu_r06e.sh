# round 6: k1q with pipelined pass-2 operands, Atab in LDS, default-policy z stores
set -o pipefail
o=gpurun_out/r06e; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "reference" -x -v --timeout 300 --timeout-method thread > $o/gputest_ref.log 2>&1; rc=$?; tail -3 $o/gputest_ref.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --config reference --steps 50 --warmup 2 --no-cpu-baseline > $o/bench_ref.json 2> $o/bench_ref.err || exit $?
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $o/sqa -o run -- python3 tools/prof_stages.py reference 5 8 c128 > $o/sqa.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d $o/sqb -o run -- python3 tools/prof_stages.py reference 5 8 c128 > $o/sqb.log 2>&1 || exit $?
python3 tools/pmc_summary.py $o/sqa $o/sqb > $o/sq_summary.txt
bash tools/pmc_pass.sh reference c128 || exit $?
grep k1q $o/sq_summary.txt
head -4 gpurun_out/pmc_reference_c128/pmc_traffic_reference_c128.json
cut -c1-300 $o/bench_ref.json
