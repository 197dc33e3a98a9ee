# round 6 final evidence on the final tree: smoke, every bench line (driver command, 500 steps,
# reference frame, per-call x2 / reference, x4, complex single, MUSIC forms, --want-rdm)
set -o pipefail
o=gpurun_out/r06final2; mkdir -p $o
export TMPDIR=/tmp
run() {  # name timeout args...
  local n=$1 t=$2; shift 2
  echo "=== $n $(date +%T)"
  timeout -k 10 $t python3 bench.py "$@" > $o/bench_$n.json 2> $o/bench_$n.err || { tail -20 $o/bench_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$o/bench_$n.json')); r=d['roofline']; print('$n', round(d['value'],1), d['unit'], 'ms/step', round(d['ms_per_step'],4), r.get('kernel'), 'frac', round(r['frac'],3), 'traffic', r.get('traffic'), 'cpu', (d.get('cpu_baseline') or {}).get('value'))"
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
run music5 300 --config music5
run music5_want_spectrum 300 --config music5 --want-spectrum
run music5_want_eig 300 --config music5 --want-eig
run want_rdm 300 --want-rdm
