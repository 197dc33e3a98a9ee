# x4 K2 at 3 workgroups per CU (2048-point blocks one row per workgroup) A/B, and SQ counters of
# the MUSIC step with the peaks-only eigensolver
set -o pipefail
o=gpurun_out/r05p; mkdir -p $o
export TMPDIR=/tmp
bash tools/ab/gpu_ab_stages.sh $o 2 "x4:c128:10 p256:c128:20" base m3all || exit $?
m=$o/music_sq; mkdir -p $m
timeout -k 10 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $m/sqa -o run -- python3 tools/music_prof.py 1024 > $m/sqa.log 2>&1 || exit $?
timeout -k 10 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d $m/sqb -o run -- python3 tools/music_prof.py 1024 > $m/sqb.log 2>&1 || exit $?
python3 tools/pmc_summary.py $m/sqa $m/sqb > $m/sq_summary.txt
cat $m/sq_summary.txt
