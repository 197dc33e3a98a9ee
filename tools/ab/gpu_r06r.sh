# round 6: MUSIC full path A/B -- wave-role rotation (ME_ROT 1-4) and bisection by lane (ME_BIS)
# on the eigenvalues form: outputs vs the shipped library, HIP-event times, phase stamps
set -o pipefail
o=gpurun_out/r06r; mkdir -p $o
export TMPDIR=/tmp
V="base rot1 rot2 rot3 rot4 bis bisrot4"
lib() { if [ $1 = base ]; then echo ""; else echo exp/ab/librsp_$1.so; fi; }
for v in $V; do
  AB_LIB=$(lib $v) timeout -k 10 120 python3 tools/ab/music_eig_check.py $o/out_$v.npz > $o/check_$v.log 2>&1 || { tail -5 $o/check_$v.log; exit 1; }
done
for r in 1 2; do
  for v in $V; do
    echo "$r $v $(AB_LIB=$(lib $v) timeout -k 10 120 python3 tools/music_prof.py 4096 10 c128 eigenvalues)" | tee -a $o/ab.log || exit 1
  done
done
for v in $V; do
  echo "$v $(RSP_MUSIC_TRACE=1 AB_LIB=$(lib $v) timeout -k 10 120 python3 tools/music_prof.py 4096 3 c128 eigenvalues 2>&1 | grep phases | tail -1)" | tee -a $o/phases.log || exit 1
done
python3 - <<'PY'
import numpy as np
o='gpurun_out/r06r'
b=np.load(o+'/out_base.npz')
for v in ('rot1','rot2','rot3','rot4','bis','bisrot4'):
    d=np.load(o+'/out_%s.npz'%v)
    print(v, {k: (float(np.abs(d[k]-b[k]).max()) if d[k].dtype.kind in 'fc' else bool((d[k]==b[k]).all())) for k in b.files})
PY
