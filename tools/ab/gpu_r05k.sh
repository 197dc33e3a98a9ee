set -o pipefail
o=gpurun_out/r05k; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_music.py -x -q --timeout 300 --timeout-method thread -m gpu > $o/music_tests.log 2>&1; rc=$?; tail -5 $o/music_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --config music5 > $o/music5.json 2> $o/music5.err || exit 1
cut -c1-300 $o/music5.json
