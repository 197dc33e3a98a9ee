# covariance with Im R = P - P^T: MUSIC tests, stage timing, bench line
set -o pipefail
o=gpurun_out/r05y; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_music.py -m gpu -x -q --timeout 300 --timeout-method thread > $o/music_tests.log 2>&1; rc=$?; tail -3 $o/music_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do timeout -k 10 120 python3 tools/music_prof.py 1024 | tee -a $o/music_prof.txt || exit $?; timeout -k 10 120 python3 tools/music_prof.py 4096 | tee -a $o/music_prof.txt || exit $?; done
timeout -k 10 300 python3 bench.py --config music5 --no-cpu-baseline > $o/bench_music5.json 2> $o/bench_music5.err || exit $?
cut -c1-200 $o/bench_music5.json
