# round 6: SQ / LDS / traffic counters of the reference frame's kernels (k1q_dbf_mtd first)
set -o pipefail
o=gpurun_out/r06d; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $o/sqa -o run -- python3 tools/prof_stages.py reference 5 8 c128 > $o/sqa.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d $o/sqb -o run -- python3 tools/prof_stages.py reference 5 8 c128 > $o/sqb.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_WR SQ_INSTS_MFMA --output-format csv -d $o/sqc -o run -- python3 tools/prof_stages.py reference 5 8 c128 > $o/sqc.log 2>&1 || exit $?
python3 tools/pmc_summary.py $o/sqa $o/sqb $o/sqc > $o/sq_summary.txt
bash tools/pmc_pass.sh reference c128 || exit $?
cat $o/sq_summary.txt
cat gpurun_out/pmc_reference_c128/pmc_traffic_reference_c128.json
