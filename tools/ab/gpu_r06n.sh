# round 6: S4 synthesis with per-target phasor tables -- parity of the synthesis/target paths,
# then the per-call lines (x2, reference) with the synthesis stage timed
set -o pipefail
o=gpurun_out/r06n; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_golden.py tests/test_queue_paths.py tests/test_config3.py > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -3 $o/tests.log
timeout -k 10 200 python3 tools/ab/percall_breakdown.py x2 200 > $o/percall_breakdown_x2.txt 2>&1 || exit $?
timeout -k 10 200 python3 tools/ab/percall_breakdown.py reference 50 > $o/percall_breakdown_ref.txt 2>&1 || exit $?
cat $o/percall_breakdown_*.txt
timeout -k 10 200 python3 bench.py --per-call --config x2 --steps 200 --warmup 10 --no-cpu-baseline > $o/percall_x2.json 2> $o/percall_x2.err || exit $?
timeout -k 10 200 python3 bench.py --per-call --config reference --steps 50 --warmup 5 --no-cpu-baseline > $o/percall_ref.json 2> $o/percall_ref.err || exit $?
python3 -c "
import json
for f in ('percall_x2','percall_ref'):
    d=json.load(open('$o/'+f+'.json')); r=d['roofline']
    print(f, round(d['value'],1), 'fps', 'median ms', round(d['per_call_ms']['median'],4), [(s['stage'], round(s['ms_per_launch']*1e3,1)) for s in r['stages']])
"
