#!/bin/bash
# Run GPU steps in order; stop at the first fault/abort/timeout (rc not in {0,1}).
# usage: tools/gpu_steps.sh "name|timeout|command" ...
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%|*}"; rest="${spec#*|}"; to="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== $name (timeout $to s): $cmd"
  timeout -k 10 "$to" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc"
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
done
exit 0
