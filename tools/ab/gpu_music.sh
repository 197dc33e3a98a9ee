#!/bin/bash
# MUSIC GPU check: parity tests, then the k_music_eig64 phase trace (debug build) and timings.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_music.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/mus.log 2>&1 || { tail -30 gpurun_out/mus.log; exit 1; }
tail -2 gpurun_out/mus.log
AB_LIB=exp/ab/librsp_dbg.so RSP_MUSIC_TRACE=1 timeout -k 10 120 python3 tools/music_prof.py 1024 5 c128 > gpurun_out/mtr.log 2>&1 || exit 1
timeout -k 10 120 python3 tools/music_prof.py 1024 5 c128 >> gpurun_out/mtr.log 2>&1 || exit 1
cat gpurun_out/mtr.log
