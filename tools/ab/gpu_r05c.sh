set -o pipefail
# A/B: z stores non-temporal (base) vs default policy (zt), frames per launch 8/4/2 (MALL residency of z)
mkdir -p gpurun_out/r05c
for round in 1 2; do
  for cfg in "base 8" "exp/ab/librsp_zt.so 8" "exp/ab/librsp_zt.so 4" "exp/ab/librsp_zt.so 2" "base 4"; do
    set -- $cfg
    timeout -k 10 200 python3 tools/ab/ab_bench.py $1 --steps 300 --fpl $2 | sed "s/^/$round fpl$2 /" | tee -a gpurun_out/r05c/ab.log || exit 1
  done
done
