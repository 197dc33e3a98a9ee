set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out; rm -f gpurun_out/ab.log
timeout -k 10 400 python -u -m pytest tests/test_music.py -x -q -m gpu --timeout 200 --timeout-method thread 2>&1 | tail -3 || exit 1
RSP_MUSIC_TRACE=1 AB_LIB=exp/ab/librsp_mtrace.so timeout -k 10 120 python3 tools/music_prof.py 1024 5 c128 2>&1 | cut -c1-300 || exit 1
for r in 1 2; do timeout -k 10 120 python3 tools/music_prof.py 1024 20 c128 | cut -c1-200 || exit 1; done
timeout -k 10 500 python3 tools/ab/ab_pytest.py exp/ab/librsp_zprune.so tests/test_gpu_parity.py tests/test_k3_prefilter.py tests/test_queue_paths.py -x -q -p no:cacheprovider 2>&1 | tail -3 || exit 1
bash tools/ab/ab.sh x2 c128 zprune || exit 1
