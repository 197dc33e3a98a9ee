set -e
for f in 5 6 7 8 5 8; do
  timeout -k 10 120 python bench.py --steps 3000 --warmup 300 --no-cpu-baseline --fpl $f > gpurun_out/b_fpl$f.json
  python -c "
import json
d=json.loads(open('gpurun_out/b_fpl$f.json').read().strip().splitlines()[-1])
print('fpl $f', round(d['value']), round(d['ms_per_step']*1e3,2), [round(s['ms_per_launch']*1e3/$f,2) for s in d['roofline']['stages']])"
done
