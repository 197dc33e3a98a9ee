# round 6: K2 at 4 workgroups per CU (2560-point rows without pads or staged twiddles, 40 KB; 128
# VGPRs with 44 B of scratch) vs the shipped 3 per CU -- RD-map identity, then x2 stage times
set -o pipefail
o=gpurun_out/r06zf; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/ab/rdm_dump.py $o/rdm_base.npy x2 c128 > $o/dump_base.log 2>&1 || exit 1
AB_LIB=exp/ab/librsp_w4.so timeout -k 10 120 python3 tools/ab/rdm_dump.py $o/rdm_w4.npy x2 c128 > $o/dump_w4.log 2>&1 || exit 1
python3 -c "import numpy as np; a=np.load('$o/rdm_base.npy'); b=np.load('$o/rdm_w4.npy'); print('rdm identical', np.array_equal(a,b), 'max diff', float(np.abs(a-b).max()))"
timeout -k 10 600 bash tools/ab/ab.sh x2 c128 w4 > $o/ab.log 2>&1 || { tail -5 $o/ab.log; exit 1; }
cp gpurun_out/ab.log $o/ab_stages.log; cat $o/ab_stages.log
