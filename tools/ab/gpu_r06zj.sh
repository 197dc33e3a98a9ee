# round 6: power-of-two complex-double plans (the reference frame, p256) in the 4-per-CU K2
# workgroups (w4p, RSP_K2_W4_POW2) -- RD-map identity, then stage times
set -o pipefail
o=gpurun_out/r06zj; mkdir -p $o
export TMPDIR=/tmp
for c in reference p256; do
  timeout -k 10 120 python3 tools/ab/rdm_dump.py /tmp/rdm_base.npy $c c128 > $o/dump_base_$c.log 2>&1 || exit 1
  AB_LIB=exp/ab/librsp_w4p.so timeout -k 10 120 python3 tools/ab/rdm_dump.py /tmp/rdm_v.npy $c c128 > $o/dump_v_$c.log 2>&1 || exit 1
  python3 -c "import numpy as np; a=np.load('/tmp/rdm_base.npy'); b=np.load('/tmp/rdm_v.npy'); print('$c w4p rdm identical', np.array_equal(a,b), float(np.abs(a-b).max()))" | tee -a $o/rdm_identity.txt
done
rm -f gpurun_out/ab.log
timeout -k 10 500 bash tools/ab/ab.sh reference c128 w4p > /dev/null 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
timeout -k 10 300 bash tools/ab/ab.sh p256 c128 w4p > /dev/null 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
cp gpurun_out/ab.log $o/ab.log; cat $o/ab.log
