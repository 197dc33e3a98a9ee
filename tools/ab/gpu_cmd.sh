set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r04n
mkdir -p $o
timeout -k 10 300 python3 bench.py --frames-total 512 --no-cpu-baseline > $o/bench_config3.json 2> $o/bench_config3.err || exit 1
timeout -k 10 300 python3 bench.py --gpus 2 --same-device --dist-backend gloo --steps 100 > $o/bench_2rank.json 2> $o/bench_2rank.err || exit 1
timeout -k 10 300 python3 bench.py --e2e --steps 100 --no-cpu-baseline > $o/bench_e2e.json 2> $o/bench_e2e.err || exit 1
for f in $o/bench*.json; do echo "$f $(cut -c1-220 $f)"; done
