# round 6: power-of-two rows in the 4-per-CU K2 workgroups padded with LDS twiddles where they fit
# (w4pad, RSP_K2_W4PAD; the 2560-point row stays unpadded) -- x2 RD-map identity and stage times;
# the same kernels with the reference frame's power-of-two plan at 4 per CU (w4ppad)
set -o pipefail
o=gpurun_out/r06zk; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/ab/rdm_dump.py /tmp/rdm_base.npy x2 c128 > $o/dump_base.log 2>&1 || exit 1
AB_LIB=exp/ab/librsp_w4pad.so timeout -k 10 120 python3 tools/ab/rdm_dump.py /tmp/rdm_v.npy x2 c128 > $o/dump_v.log 2>&1 || exit 1
python3 -c "import numpy as np; a=np.load('/tmp/rdm_base.npy'); b=np.load('/tmp/rdm_v.npy'); print('x2 w4pad rdm identical', np.array_equal(a,b), float(np.abs(a-b).max()))" | tee -a $o/rdm_identity.txt
rm -f gpurun_out/ab.log
timeout -k 10 500 bash tools/ab/ab.sh x2 c128 w4pad > /dev/null 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
timeout -k 10 500 bash tools/ab/ab.sh reference c128 w4ppad > /dev/null 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
cp gpurun_out/ab.log $o/ab.log; cat $o/ab.log
