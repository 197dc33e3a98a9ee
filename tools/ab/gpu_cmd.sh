set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out; rm -f gpurun_out/ab.log
bash tools/ab/ab.sh x2 c128 e2f e2s || exit 1
