# config #5 instances per launch: 1024 vs 2048 vs 4096
set -o pipefail
o=gpurun_out/r05w; mkdir -p $o
for round in 1 2; do
  for b in 1024 2048 4096; do
    timeout -k 10 240 python3 bench.py --config music5 --batch $b --no-cpu-baseline > $o/music_b$b.json 2> $o/music_b$b.err || exit $?
    python3 -c "import json; d=json.load(open('$o/music_b$b.json')); print($round, $b, round(d['value']), round(d['ms_per_step'],4), [round(s['ms_per_launch'],4) for s in d['roofline']['stages']])" | tee -a $o/ab.log
  done
done
