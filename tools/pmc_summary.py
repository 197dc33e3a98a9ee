"""Average rocprofv3 --pmc counters per kernel (usage: pmc_summary.py dir...)."""
import collections
import csv
import sys

for d in sys.argv[1:]:
    rows = list(csv.DictReader(open(d + '/p_counter_collection.csv')))
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in rows:
        kn = r['Kernel_Name'].replace('void ', '').replace('(anonymous namespace)::', '').split('(')[0]
        agg[kn][r['Counter_Name']].append(float(r['Counter_Value']))
    for kn, cs in agg.items():
        if kn.startswith('k'):
            print(d, kn, {c: '%.4g' % (sum(v) / len(v)) for c, v in cs.items()})
