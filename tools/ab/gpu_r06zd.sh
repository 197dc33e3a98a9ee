# round 6: K1 with the in-place DIF FFT at P = 256 (>= 16 channels) and the early next-tile issue --
# the whole GPU suite, fresh PMC traffic for every file holding k1p_dbf_mtd, and the x4 / x2 lines
set -o pipefail
o=gpurun_out/r06zd; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/gputest.log 2>&1 || { tail -30 $o/gputest.log; exit 1; }
tail -2 $o/gputest.log
for a in "x4 c128" "x2 c128" "x2 c64" "x2 c128 rdm"; do
  echo "=== pmc $a"
  bash tools/pmc_pass.sh $a > /dev/null || exit $?
done
mkdir -p $o/pmc; cp gpurun_out/pmc_*/pmc_traffic_*.json $o/pmc/
cp gpurun_out/pmc_x4_c128/pmc_traffic_x4_c128.json gpurun_out/pmc_x2_c128/pmc_traffic_x2_c128.json gpurun_out/pmc_x2_c64/pmc_traffic_x2_c64.json gpurun_out/pmc_x2_c128_rdm/pmc_traffic_x2_c128_rdm.json profiles/
for m in "x4 --config x4" "driver_cmd --steps 20 --warmup 5" "p256 --config p256 --no-cpu-baseline"; do
  set -- $m; n=$1; shift
  timeout -k 10 300 python3 bench.py "$@" > $o/bench_$n.json 2> $o/bench_$n.err || { tail -5 $o/bench_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$o/bench_$n.json')); r=d['roofline']; print('$n', round(d['value'],1), round(d['ms_per_step'],4), r['kernel'], round(r['frac'],3), r.get('traffic'), [(s['stage'], round(s['ms_per_launch']*1e3,1)) for s in r['stages']])"
done
