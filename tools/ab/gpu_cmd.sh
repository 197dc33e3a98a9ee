set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out; rm -f gpurun_out/ab_bench.log
bash tools/ab/ab_bench.sh "--steps 300" lanes4 lanes2 || exit 1
for r in 1 2; do for f in 8 4; do echo "$r fpl $f $(timeout -k 10 200 python3 bench.py --steps 300 --fpl $f --no-cpu-baseline | cut -c100-200)" || exit 1; done; done
