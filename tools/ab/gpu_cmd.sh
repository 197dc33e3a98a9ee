set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 tools/ab/ab_pytest.py exp/ab/librsp_msect.so tests/test_music.py -x -q -m gpu -p no:cacheprovider 2>&1 | tail -2 || exit 1
RSP_MUSIC_TRACE=1 AB_LIB=exp/ab/librsp_mtrace.so timeout -k 10 120 python3 tools/music_prof.py 1024 5 c128 2>&1 | cut -c1-300 || exit 1
for r in 1 2 3; do for v in base msect; do
  if [ $v = base ]; then lib=""; else lib=exp/ab/librsp_$v.so; fi
  echo "$r $v $(AB_LIB=$lib timeout -k 10 120 python3 tools/music_prof.py 1024 20 c128 | cut -c1-120)" || exit 1
done; done
