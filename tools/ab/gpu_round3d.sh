#!/bin/bash
# Round-3 closing evidence for HEAD: every gpu test, smoke(), the x2 profile round (bench line,
# kernel trace + stats, PMC traffic, SQ counters), the driver's bench command, and a 2-rank
# rehearsal of the torchrun bench path (gloo, both ranks on the one GPU).  Outputs under gpurun_out/.
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r03d}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/${tag}_gputest.log 2>&1 || { tail -40 gpurun_out/${tag}_gputest.log; exit 1; }
tail -2 gpurun_out/${tag}_gputest.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 || { tail -20 gpurun_out/${tag}_smoke.log; exit 1; }
tail -1 gpurun_out/${tag}_smoke.log
bash tools/profile_round.sh ${tag}x2 x2 c128 || exit $?
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/${tag}_bench_driver_cmd.json 2> gpurun_out/${tag}_bench_driver_cmd.err || { tail -20 gpurun_out/${tag}_bench_driver_cmd.err; exit 1; }
tail -1 gpurun_out/${tag}_bench_driver_cmd.json | cut -c1-300
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --dist-backend gloo --same-device --no-cpu-baseline > gpurun_out/${tag}_bench_2rank_gloo.json 2> gpurun_out/${tag}_bench_2rank_gloo.err || { tail -20 gpurun_out/${tag}_bench_2rank_gloo.err; exit 1; }
tail -1 gpurun_out/${tag}_bench_2rank_gloo.json | cut -c1-300
