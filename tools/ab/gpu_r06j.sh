# round 6: k1q phase stamps at the reference frame (diagnostic build)
set -o pipefail
o=gpurun_out/r06j; mkdir -p $o
AB_LIB=exp/ab/librsp_diag.so timeout -k 10 180 python3 tools/ab/k1_phases.py reference c128 > $o/k1q_phases.txt 2>&1 || exit $?
cat $o/k1q_phases.txt
AB_LIB=exp/ab/librsp_diag.so timeout -k 10 180 python3 tools/ab/k1_phases.py x2 c128 > $o/k1p_phases_x2.txt 2>&1 || exit $?
cat $o/k1p_phases_x2.txt
