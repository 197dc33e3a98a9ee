# usage: sweep.sh "name|ENV=.. ENV=..|bench args" ...
for v in "$@"; do
  n=${v%%|*}; r=${v#*|}; e=${r%%|*}; x=${r#*|}
  env $e timeout -k 10 120 python bench.py --no-cpu-baseline $x > gpurun_out/b_$n.json || exit 1
done
