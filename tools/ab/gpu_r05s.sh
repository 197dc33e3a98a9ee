# persistent K2 diagnosis: HBM traffic of k2_pcp (locality of the z-line pairs)
set -o pipefail
bash tools/pmc_pass.sh x2 c128 || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/pmc_x2_c128/pmc_traffic_x2_c128.json')); print({k: v for k, v in d['_raw'].items()})"
