# K2 phase timeline at 3 workgroups per CU, x4 with the 2560-point long block (A/B), and hashed
# PMC traffic for the secondary lines (x4, complex single, --want-rdm)
set -o pipefail
o=gpurun_out/r05n; mkdir -p $o
export TMPDIR=/tmp
AB_LIB=exp/ab/librsp_dbg.so timeout -k 10 120 python3 tools/ab/k2_phases.py x2 c128 > $o/k2_phases.txt 2>&1 || exit $?
cat $o/k2_phases.txt
bash tools/ab/gpu_ab_stages.sh $o 2 "x4:c128:10 x2:c128:50" base x4mix || exit $?
bash tools/pmc_pass.sh x4 c128 || exit $?
bash tools/pmc_pass.sh x2 c64 || exit $?
bash tools/pmc_pass.sh x2 c128 rdm || exit $?
