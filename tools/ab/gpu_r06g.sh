# round 6: MFMA counters (K1 at x2 / x4 / reference, MUSIC covariance), MUSIC lines (peaks, --want-eig), x4 line
set -o pipefail
o=gpurun_out/r06g; mkdir -p $o
export TMPDIR=/tmp
for cfg in x2 x4 reference; do
  timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE --output-format csv -d $o/mfma_$cfg -o run -- python3 tools/prof_stages.py $cfg 5 8 c128 > $o/mfma_$cfg.log 2>&1 || exit $?
done
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE --output-format csv -d $o/mfma_music5 -o run -- python3 tools/music_prof.py 4096 5 c128 > $o/mfma_music5.log 2>&1 || exit $?
python3 tools/mfma_summary.py x2:$o/mfma_x2 x4:$o/mfma_x4 reference:$o/mfma_reference music5:$o/mfma_music5 > $o/r06_mfma_counters.txt
cat $o/r06_mfma_counters.txt | cut -c1-200
timeout -k 10 300 python3 bench.py --config music5 --no-cpu-baseline > $o/bench_music5.json 2> $o/bench_music5.err || exit $?
timeout -k 10 300 python3 bench.py --config music5 --want-eig --no-cpu-baseline > $o/bench_music5_eig.json 2> $o/bench_music5_eig.err || exit $?
timeout -k 10 300 python3 bench.py --config x4 --steps 20 --no-cpu-baseline > $o/bench_x4.json 2> $o/bench_x4.err || exit $?
for f in $o/bench_*.json; do cut -c1-250 $f; done
