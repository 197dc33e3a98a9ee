set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/music_sq
timeout -k 10 400 python -u -m pytest tests/test_music.py -x -q -m gpu --timeout 200 --timeout-method thread 2>&1 | tail -3 || exit 1
RSP_MUSIC_TRACE=1 AB_LIB=exp/ab/librsp_mtrace.so timeout -k 10 120 python3 tools/music_prof.py 1024 5 c128 2>&1 | cut -c1-300 || exit 1
for r in 1 2; do timeout -k 10 120 python3 tools/music_prof.py 1024 20 c128 | cut -c1-260 || exit 1; done
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d gpurun_out/music_sq/sqa -o run -- python3 tools/music_prof.py 1024 3 c128 > gpurun_out/music_sq/sqa.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/music_sq/sqb -o run -- python3 tools/music_prof.py 1024 3 c128 > gpurun_out/music_sq/sqb.log 2>&1 || exit 1
python3 tools/pmc_summary.py gpurun_out/music_sq/sqa gpurun_out/music_sq/sqb
