# round 6: MUSIC spectrum calls on the fast path where its bound holds P_dB to 1e-8 dB
set -o pipefail
o=gpurun_out/r06s; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_music.py > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -2 $o/tests.log
for m in "spectrum --want-spectrum" "peaks" "eig --want-eig"; do
  set -- $m
  timeout -k 10 300 python3 bench.py --config music5 $2 > $o/bench_music5_$1.json 2> $o/bench_music5_$1.err || { tail -20 $o/bench_music5_$1.err; exit 1; }
  python3 -c "import json; d=json.load(open('$o/bench_music5_$1.json')); print('$1', round(d['value']), d['ms_per_step'], [(s['stage'], round(s['ms_per_launch'],3), s.get('fast_path_instances')) for s in d['roofline']['stages']], (d.get('cpu_baseline') or {}).get('value'))"
done
