# persistent K1 as two 256-thread workgroups per CU (NT = 2, z chunks kept at 4 samples): RDM
# bit-identity vs the shipped build, then stage + bench A/B
set -o pipefail
o=gpurun_out/r05ae; mkdir -p $o
timeout -k 10 120 python3 tools/ab/rdm_dump.py $o/base.npy x2 c128 || exit $?
AB_LIB=exp/ab/librsp_k1t256.so timeout -k 10 120 python3 tools/ab/rdm_dump.py $o/k1t256.npy x2 c128 || exit $?
python3 -c "import numpy as np; a=np.load('$o/base.npy'); b=np.load('$o/k1t256.npy'); print('rdm max rel diff', np.abs(a-b).max()/np.abs(a).max(), 'identical', np.array_equal(a,b))"
bash tools/ab/gpu_ab_stages.sh $o 3 "x2:c128:50" base k1t256 || exit $?
bash tools/ab/ab_bench.sh "--steps 300" k1t256 || exit $?
