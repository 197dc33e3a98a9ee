set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r05i; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_k3_prefilter.py tests/test_detection_capacity.py -x -q --timeout 300 --timeout-method thread > $o/parity.log 2>&1; rc=$?; tail -3 $o/parity.log; [ $rc -eq 0 ] || exit $rc
for cfg in x2 x4; do for v in base old; do
  if [ $v = base ]; then lib=""; else lib=exp/ab/librsp_$v.so; fi
  AB_LIB=$lib timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_WAVES --output-format csv -d $o/sq_${cfg}_$v -o run -- python3 tools/prof_stages.py $cfg 5 8 c128 > $o/sq_${cfg}_$v.log 2>&1 || exit 1
  python3 tools/pmc_summary.py $o/sq_${cfg}_$v | tee -a $o/sq_summary.txt
done; done
bash tools/ab/gpu_ab_stages.sh $o 2 "x2:c128:50 x4:c128:10" base old || exit 1
timeout -k 10 600 python -u -m pytest tests/test_music.py -x -q --timeout 300 --timeout-method thread -m gpu > $o/music_tests.log 2>&1; rc=$?; tail -3 $o/music_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do timeout -k 10 120 python3 tools/music_prof.py | tail -n 1 | tee -a $o/music_prof.txt || exit 1; AB_LIB=exp/ab/librsp_old.so timeout -k 10 120 python3 tools/music_prof.py | tail -n 1 | sed 's/^/old /' | tee -a $o/music_prof.txt || exit 1; done
