set -o pipefail
mkdir -p gpurun_out/r05d
AB_LIB=exp/ab/librsp_dbg.so timeout -k 10 120 python3 tools/ab/k2_phases.py x2 c128 gpurun_out/r05d/k2_phases.npz > gpurun_out/r05d/k2_phases.txt 2>&1; rc=$?; cat gpurun_out/r05d/k2_phases.txt; exit $rc
