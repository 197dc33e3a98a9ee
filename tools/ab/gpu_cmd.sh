set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out; rm -f gpurun_out/ab.log
for v in m2pf8 m2pf16; do
timeout -k 10 300 python3 tools/ab/ab_pytest.py exp/ab/librsp_$v.so tests/test_gpu_parity.py tests/test_k3_prefilter.py -x -q -k "x2 or small or x4" -p no:cacheprovider 2>&1 | tail -2 || exit 1
done
bash tools/ab/ab.sh x2 c128 m2pf0 m2pf4 m2pf8 m2pf16 || exit 1
