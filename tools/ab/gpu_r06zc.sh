# round 6: P = 256 through the in-place DIF FFT in K1 (persistent and tiled) instead of the Stockham
# passes -- x4 / p256 parity, then stage times: shipped lib = DIF, head = the Stockham K1, early8 =
# DIF + the next tile's loads issued right after the DBF
set -o pipefail
o=gpurun_out/r06zc; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "x4 or p256" > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -2 $o/tests.log
for cfg in x4 p256; do
  timeout -k 10 600 bash tools/ab/ab.sh $cfg c128 head early8 > $o/ab_$cfg.log 2>&1 || { tail -5 $o/ab_$cfg.log; exit 1; }
done
cp gpurun_out/ab.log $o/ab_all.log
timeout -k 10 300 python3 bench.py --config x4 > $o/bench_x4.json 2> $o/bench_x4.err || exit 1
python3 -c "import json; d=json.load(open('$o/bench_x4.json')); print('x4', round(d['value'],1), d['ms_per_step'], [(s['stage'], round(s['ms_per_launch'],3)) for s in d['roofline']['stages']])"
