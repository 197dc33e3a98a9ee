# round 6: where k_synth's time goes -- ablations (timing only; outputs not checked):
# syn1 no log/sqrt/sincos, syn2 no Philox, syn3 no targets, syn4 no sincos, syn5 no log/sqrt
set -o pipefail
o=gpurun_out/r06t; mkdir -p $o
export TMPDIR=/tmp
for r in 1 2; do
  for v in base syn1 syn2 syn3 syn4 syn5; do
    if [ $v = base ]; then lib=""; else lib=exp/ab/librsp_$v.so; fi
    echo "$r $v $(AB_LIB=$lib timeout -k 10 120 python3 tools/ab/synth_prof.py 50)" | tee -a $o/ab.log || exit 1
  done
done
