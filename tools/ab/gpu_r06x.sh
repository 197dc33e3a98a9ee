# round 6: k_synth with its phasor tables in LDS (no table kernel) -- whole GPU suite, synthesis time,
# per-call lines
set -o pipefail
o=gpurun_out/r06x; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/gputest.log 2>&1 || { tail -30 $o/gputest.log; exit 1; }
tail -2 $o/gputest.log
for r in 1 2; do echo "$r $(timeout -k 10 120 python3 tools/ab/synth_prof.py 50)" | tee -a $o/synth.log || exit 1; done
timeout -k 10 300 python3 bench.py --per-call --config x2 --steps 200 --warmup 10 > $o/percall_x2.json 2> $o/percall_x2.err || exit 1
timeout -k 10 300 python3 bench.py --per-call --config reference --steps 50 --warmup 5 > $o/percall_ref.json 2> $o/percall_ref.err || exit 1
python3 -c "
import json
for f in ('percall_x2','percall_ref'):
    d=json.load(open('$o/'+f+'.json')); r=d['roofline']
    print(f, round(d['value'],1), 'median ms', round(d['per_call_ms']['median'],4), [(s['stage'], round(s['ms_per_launch']*1e3,1)) for s in r['stages']], (d.get('cpu_baseline') or {}).get('value'))
"
