# A/B of queue/launch options on the x2 bench (usage: bash tools/cmp_queue.sh "NAME ENV=.. ..." ...)
set -e
for spec in "$@"; do
  set -- $spec; name=$1; shift
  env "$@" timeout -k 10 120 python bench.py --steps 3000 --warmup 300 --no-cpu-baseline > gpurun_out/b_$name.json
  python -c "
import json
d=json.loads(open('gpurun_out/b_$name.json').read().strip().splitlines()[-1])
print('$name', round(d['value']), round(d['ms_per_step']*1e3,2), [round(s['ms_per_launch']*1e3,1) for s in d['roofline']['stages']])"
done
