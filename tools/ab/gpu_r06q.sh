# round 6: synthesis strip length A/B (SYNTH_NS 4 / 8 / 16) + SQ counters of k_synth
set -o pipefail
o=gpurun_out/r06q; mkdir -p $o
export TMPDIR=/tmp
for r in 1 2; do
  for v in base ns4 ns16; do
    if [ $v = base ]; then lib=""; else lib=exp/ab/librsp_$v.so; fi
    echo "$r $v $(AB_LIB=$lib timeout -k 10 120 python3 tools/ab/synth_prof.py 50)" | tee -a $o/ab.log || exit 1
  done
done
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d $o/sqa -o run -- python3 tools/ab/synth_prof.py 5 > $o/sqa.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SMEM GRBM_GUI_ACTIVE --output-format csv -d $o/sqb -o run -- python3 tools/ab/synth_prof.py 5 > $o/sqb.log 2>&1 || exit $?
python3 tools/pmc_summary.py $o/sqa $o/sqb > $o/sq_summary.txt 2>&1; grep -i synth $o/sq_summary.txt || true
