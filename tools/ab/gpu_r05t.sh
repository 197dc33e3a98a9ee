# 16 frames per launch (RSP_MAX_F = 16 build) vs 8: steady state and the driver's 20-step region
set -o pipefail
o=gpurun_out/r05t; mkdir -p $o
for round in 1 2 3; do
  timeout -k 10 200 python3 tools/ab/ab_bench.py base --steps 300 | sed "s/^/$round fpl8 s300 /" | tee -a $o/ab.log || exit $?
  timeout -k 10 200 python3 tools/ab/ab_bench.py exp/ab/librsp_f16.so --steps 150 --fpl 16 --ring 16 | sed "s/^/$round fpl16 s150 /" | tee -a $o/ab.log || exit $?
  timeout -k 10 200 python3 tools/ab/ab_bench.py base --steps 20 | sed "s/^/$round fpl8 s20 /" | tee -a $o/ab.log || exit $?
  timeout -k 10 200 python3 tools/ab/ab_bench.py exp/ab/librsp_f16.so --steps 20 --fpl 16 --ring 16 | sed "s/^/$round fpl16 s20 /" | tee -a $o/ab.log || exit $?
done
