"""Print one line per bench JSON: frames/s, us/frame, dominant kernel, frac, stage ms (roofline leg / live)."""
import json
import sys

for fn in sys.argv[1:]:
    d = json.load(open(fn))
    r = d['roofline']
    print(fn.split('/')[-1], round(d['value']), round(d['ms_per_step'] * 1e3, 2), r['kernel'], round(r['frac'], 3),
          [(s['stage'][:2], round(s['ms_per_launch'] * 1e3, 1),
            round(s.get('live_overlapped_ms_per_launch', 0) * 1e3, 1)) for s in r['stages']])
