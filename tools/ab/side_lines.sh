#!/bin/bash
# The round's secondary bench lines (one GPU): the driver's own command, complex single, config #3
# (512 distinct frames), end to end from pinned host cubes, config #4, config #5 (MUSIC).
# usage: tools/side_lines.sh TAG       -> gpurun_out/<TAG>_bench_*.json
set -o pipefail
t=$1
mkdir -p gpurun_out
run() {  # name timeout args...
  local n=$1 to=$2; shift 2
  timeout -k 10 $to python3 bench.py "$@" > gpurun_out/${t}_bench_$n.json 2> gpurun_out/${t}_bench_$n.err || { echo "$n failed rc=$?"; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/${t}_bench_$n.json').read().strip().splitlines()[-1]); print('$n', round(d['value'],1), d['unit'], d.get('roofline',{}).get('frac'))"
}
run driver_cmd 240 --gpus 1 --steps 20 --warmup 5
run c64 240 --precision c64 --steps 200 --warmup 10 --no-cpu-baseline
run config3 240 --frames-total 512 --ring 512 --steps 64 --warmup 20 --no-cpu-baseline
run e2e 240 --e2e --steps 40 --warmup 6 --no-cpu-baseline
run x4 300 --config x4 --steps 10 --warmup 4 --no-cpu-baseline
run music5 240 --config music5 --steps 50 --warmup 5
