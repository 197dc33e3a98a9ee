# round 6: K2 dispatch order with the long segment's units moved earlier (key x 0.85 / 0.7,
# RSP_K2_LONGBIAS), so that the launch's tail holds the shorter FIR / medium workgroups
set -o pipefail
o=gpurun_out/r06zi; mkdir -p $o
export TMPDIR=/tmp
rm -f gpurun_out/ab.log
timeout -k 10 500 bash tools/ab/ab.sh x2 c128 lb085 lb07 > /dev/null 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
timeout -k 10 500 bash tools/ab/ab.sh x4 c128 lb085 lb07 > /dev/null 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
cp gpurun_out/ab.log $o/ab.log; cat $o/ab.log
