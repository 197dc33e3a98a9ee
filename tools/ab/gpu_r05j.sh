set -o pipefail
o=gpurun_out/r05j; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_music.py -x -v --timeout 300 --timeout-method thread -m gpu > $o/music_tests.log 2>&1; rc=$?; tail -5 $o/music_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do timeout -k 10 120 python3 tools/music_prof.py | tail -n 1 | tee -a $o/music_prof.txt || exit 1; done
timeout -k 10 300 python3 bench.py --config music5 --no-cpu-baseline > $o/music5.json 2> $o/music5.err || exit 1
cut -c1-400 $o/music5.json
