# round 6: PMC traffic refresh on the final synthesis (x2, reference frame) + 2-rank gloo rehearsal
# of the multi-GPU bench path on one GPU
set -o pipefail
export TMPDIR=/tmp
for a in "x2 c128" "reference c128"; do
  echo "=== pmc $a"
  bash tools/pmc_pass.sh $a > /dev/null || exit $?
done
o=gpurun_out/r06y; mkdir -p $o
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --same-device --dist-backend gloo --steps 100 --warmup 5 > $o/bench_2rank_gloo.json 2> $o/bench_2rank_gloo.err || { tail -20 $o/bench_2rank_gloo.err; exit 1; }
python3 -c "import json; d=json.load(open('$o/bench_2rank_gloo.json')); print(round(d['value']), d['n_gpus'], d['ms_per_step'], d['distributed']['world_size'], d['distributed']['backend'])"
