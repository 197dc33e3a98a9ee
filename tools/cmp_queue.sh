set -e
run() { name=$1; shift; env "$@" timeout -k 10 120 python bench.py --steps 2000 --warmup 200 --no-cpu-baseline > gpurun_out/b_$name.json; python -c "
import json,sys
d=json.loads(open('gpurun_out/b_$name.json').read().strip().splitlines()[-1]); print('$name', round(d['value']), round(d['ms_per_step']*1e3,2))
"; }
run base X=1
run pipe RSP_QUEUE=pipe
run pipe2 RSP_QUEUE=pipe RSP_NLANES=2
run pipe_nt4 RSP_QUEUE=pipe RSP_NT=4 RSP_LIB=$PWD/exp/librsp_k1_256.so
run nt4 RSP_NT=4 RSP_LIB=$PWD/exp/librsp_k1_256.so
