# round 6: host-side split of the short timed region
set -o pipefail
o=gpurun_out/r06za; mkdir -p $o
export TMPDIR=/tmp
for s in 20 100 20; do timeout -k 10 200 python3 tools/ab/region_breakdown.py $s 5 | tee -a $o/region.log || exit 1; done
