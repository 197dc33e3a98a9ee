# round 6 final: MFMA counters of K1 (x2 / x4 / reference) and the MUSIC covariance on the final
# kernels (k1p_dbf_mtd changed with the P = 256 DIF), with their kernel hashes
set -o pipefail
o=gpurun_out/r06ze; mkdir -p $o
export TMPDIR=/tmp
for cfg in x2 x4 reference; do
  timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE --output-format csv -d $o/mfma_$cfg -o run -- python3 tools/prof_stages.py $cfg 5 8 c128 > $o/mfma_$cfg.log 2>&1 || exit $?
done
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE --output-format csv -d $o/mfma_music5 -o run -- python3 tools/music_prof.py 4096 5 c128 > $o/mfma_music5.log 2>&1 || exit $?
python3 tools/mfma_summary.py x2:$o/mfma_x2 x4:$o/mfma_x4 reference:$o/mfma_reference music5:$o/mfma_music5 > $o/r06_mfma_counters.txt
cat $o/r06_mfma_counters.txt | cut -c1-160
