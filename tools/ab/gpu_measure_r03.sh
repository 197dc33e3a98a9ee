#!/bin/bash
# Round-3 measurement pass: x4 (config #4) profile round + MFMA counters of K1 (x4 and x2),
# MUSIC (config #5, complex double) traffic passes and bench line.  Outputs under gpurun_out/.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/mfma gpurun_out/music
bash tools/profile_round.sh r03x4 x4 c128 --steps 200 --warmup 10 || exit $?
for cfg in x4 x2; do
  timeout -k 10 90 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_F64 GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/mfma/$cfg -o run -- python3 tools/prof_stages.py $cfg 10 8 c128 > gpurun_out/mfma/$cfg.log 2>&1 || exit $?
done
timeout -k 10 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/music/fetch -o run -- python3 tools/music_prof.py 1024 5 c128 > gpurun_out/music/fetch.log 2>&1 || exit $?
timeout -k 10 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/music/write -o run -- python3 tools/music_prof.py 1024 5 c128 > gpurun_out/music/write.log 2>&1 || exit $?
python3 tools/pmc_traffic.py gpurun_out/music/fetch gpurun_out/music/write gpurun_out/music/pmc_traffic_music5_c128.json music_prof 1024 5 || exit $?
timeout -k 10 90 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/music/mfma -o run -- python3 tools/music_prof.py 1024 5 c128 > gpurun_out/music/mfma.log 2>&1 || exit $?
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/music/trace -o run -- python3 bench.py --config music5 --no-cpu-baseline --steps 100 > gpurun_out/music/trace.log 2>&1 || exit $?
echo done
