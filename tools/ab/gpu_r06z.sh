# round 6: the driver's short timed region -- ms per step at 10/20/40/100/500 steps (fixed overhead
# of the region) and a kernel trace of the --steps 20 run
set -o pipefail
o=gpurun_out/r06z; mkdir -p $o
export TMPDIR=/tmp
for s in 10 20 40 100 500 20 10; do
  timeout -k 10 200 python3 bench.py --steps $s --warmup 5 --no-cpu-baseline > $o/b$s.json 2> $o/b$s.err || exit 1
  python3 -c "import json; d=json.load(open('$o/b$s.json')); print($s, round(d['value']), round(d['ms_per_step'],4))" | tee -a $o/steps.log
done
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $o/trace -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $o/trace.log 2>&1 || exit 1
