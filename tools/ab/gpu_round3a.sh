set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_amplitude_kat.py tests/test_music.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/t1.log 2>&1 || { tail -30 gpurun_out/t1.log; exit 1; }
tail -3 gpurun_out/t1.log
AB_LIB=exp/ab/librsp_dbg.so RSP_MUSIC_TRACE=1 timeout -k 10 120 python3 tools/music_prof.py 1024 5 c128 > gpurun_out/mtr.log 2>&1 || exit 1
timeout -k 10 120 python3 tools/music_prof.py 1024 5 c128 >> gpurun_out/mtr.log 2>&1 || exit 1
cat gpurun_out/mtr.log
bash tools/ab/ab.sh x2 c128 old
