# round 6 final evidence after the buffer-resource twiddles in K2 (k2_pc code changed): the whole
# GPU suite, the x2 profile round, fresh PMC traffic for every file holding k2_pc, smoke() and the
# bench lines whose plans run K2
set -o pipefail
o=gpurun_out/r06final4; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/gputest.log 2>&1 || { tail -30 $o/gputest.log; exit 1; }
tail -2 $o/gputest.log
bash tools/profile_round.sh r06final4 x2 c128 --steps 500 || exit $?
for a in "x2 c64" "x4 c128" "reference c128" "x2 c128 rdm"; do
  echo "=== pmc $a"
  bash tools/pmc_pass.sh $a > /dev/null || exit $?
done
run() {  # name timeout args...
  local n=$1 t=$2; shift 2
  echo "=== $n $(date +%T)"
  timeout -k 10 $t python3 bench.py "$@" > $o/bench_$n.json 2> $o/bench_$n.err || { tail -20 $o/bench_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$o/bench_$n.json')); r=d['roofline']; print('$n', round(d['value'],1), d['unit'], 'ms/step', round(d['ms_per_step'],4), r.get('kernel'), 'frac', round(r['frac'],3), 'traffic', r.get('traffic'), (r.get('traffic_source') or {}).get('fresh'), 'cpu', (d.get('cpu_baseline') or {}).get('value'), [(s['stage'], round(s['ms_per_launch']*1e3,1)) for s in r.get('stages', [])])"
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
