# round 6: K2 phase timeline of the final kernel (k2_pc<double, 4>, diagnostic build); A/B of K2
# variants: non-temporal z sample loads (znt, RSP_K2_ZAUX=2) and twiddles outside LDS read through a
# buffer resource (twbuf, RSP_K2_TWBUF=1; RD map must stay bit-identical)
set -o pipefail
o=gpurun_out/r06zg; mkdir -p $o
export TMPDIR=/tmp
AB_LIB=exp/ab/librsp_diag.so timeout -k 10 120 python3 tools/ab/k2_phases.py x2 c128 > $o/k2_phases.txt 2>&1 || { tail -20 $o/k2_phases.txt; exit 1; }
cat $o/k2_phases.txt
for c in x2 x4; do
  timeout -k 10 120 python3 tools/ab/rdm_dump.py /tmp/rdm_base.npy $c c128 > $o/dump_base_$c.log 2>&1 || exit 1
  AB_LIB=exp/ab/librsp_twbuf.so timeout -k 10 120 python3 tools/ab/rdm_dump.py /tmp/rdm_tw.npy $c c128 > $o/dump_tw_$c.log 2>&1 || exit 1
  python3 -c "import numpy as np; a=np.load('/tmp/rdm_base.npy'); b=np.load('/tmp/rdm_tw.npy'); print('$c twbuf rdm identical', np.array_equal(a,b))" | tee -a $o/rdm_identity.txt
done
rm -f gpurun_out/ab.log
timeout -k 10 500 bash tools/ab/ab.sh x2 c128 znt twbuf > /dev/null 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
timeout -k 10 500 bash tools/ab/ab.sh x4 c128 twbuf > /dev/null 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
cp gpurun_out/ab.log $o/ab.log; cat $o/ab.log
