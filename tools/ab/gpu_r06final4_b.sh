# round 6 final: the x4 and --want-rdm lines again with the fresh PMC files (their roofline kernel is
# k2_pc), x4 twice
set -o pipefail
o=gpurun_out/r06final4; mkdir -p $o
export TMPDIR=/tmp
run() {  # name timeout args...
  local n=$1 t=$2; shift 2
  echo "=== $n $(date +%T)"
  timeout -k 10 $t python3 bench.py "$@" > $o/bench_$n.json 2> $o/bench_$n.err || { tail -20 $o/bench_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$o/bench_$n.json')); r=d['roofline']; print('$n', round(d['value'],1), d['unit'], 'ms/step', round(d['ms_per_step'],4), r.get('kernel'), 'frac', round(r['frac'],3), 'traffic', r.get('traffic'), (r.get('traffic_source') or {}).get('fresh'), 'cpu', (d.get('cpu_baseline') or {}).get('value'), [(s['stage'], round(s['ms_per_launch']*1e3,1)) for s in r.get('stages', [])])"
}
run x4 300 --config x4
run x4_again 300 --config x4 --no-cpu-baseline
run want_rdm 300 --want-rdm
