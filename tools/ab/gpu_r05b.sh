set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r05b; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_music.py -x -q --timeout 300 --timeout-method thread -m gpu > $o/music_tests.log 2>&1; rc=$?; tail -3 $o/music_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --gpus 2 --same-device --dist-backend gloo --steps 100 --no-cpu-baseline > $o/bench_2rank.json 2> $o/bench_2rank.err || exit 1
bash tools/pmc_pass.sh x2 c128 > /dev/null || exit 1
cp gpurun_out/pmc_x2_c128/pmc_traffic_x2_c128.json $o/
python3 -c "import json; d=json.load(open('$o/bench_2rank.json')); print(d['value'], json.dumps(d['distributed'])[:400])"
