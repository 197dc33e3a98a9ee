# round 6, K2 at 4 workgroups per CU shipped: A/B against the round-5 layout (3 per CU, pads,
# staged twiddles: exp/ab/librsp_w3.so built from the previous commit) on x2 and x4, smoke(), and
# the bench lines whose plans run k2_pc<double, 4>
set -o pipefail
o=gpurun_out/r06final3; mkdir -p $o
export TMPDIR=/tmp
rm -f gpurun_out/ab.log
timeout -k 10 400 bash tools/ab/ab.sh x2 c128 w3 > /dev/null 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
timeout -k 10 400 bash tools/ab/ab.sh x4 c128 w3 > /dev/null 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
cp gpurun_out/ab.log $o/ab_w3.log; cat $o/ab_w3.log
run() {  # name timeout args...
  local n=$1 t=$2; shift 2
  echo "=== $n $(date +%T)"
  timeout -k 10 $t python3 bench.py "$@" > $o/bench_$n.json 2> $o/bench_$n.err || { tail -20 $o/bench_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$o/bench_$n.json')); r=d['roofline']; print('$n', round(d['value'],1), d['unit'], 'ms/step', round(d['ms_per_step'],4), r.get('kernel'), 'frac', round(r['frac'],3), 'traffic', r.get('traffic'), 'cpu', (d.get('cpu_baseline') or {}).get('value'), [(s['stage'], round(s['ms_per_launch']*1e3,1)) for s in r.get('stages', [])])"
}
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { tail -20 $o/smoke.log; exit 1; }
tail -2 $o/smoke.log
run driver_cmd 300 --steps 20 --warmup 5
run steps500 300 --steps 500 --no-cpu-baseline
run reference 300 --config reference
run percall_x2 300 --per-call --config x2 --steps 200 --warmup 10
run percall_reference 300 --per-call --config reference --steps 50 --warmup 5
run x4 300 --config x4
run c64 300 --precision c64
run want_rdm 300 --want-rdm
