"""Average rocprofv3 --pmc counters per kernel (usage: pmc_summary.py dir...).

Reads every *counter_collection.csv under each directory (rocprofv3 --output-format csv)."""
import collections
import csv
import glob
import sys

for d in sys.argv[1:]:
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for fn in glob.glob(d + '/**/*counter_collection.csv', recursive=True):
        for r in csv.DictReader(open(fn)):
            kn = r['Kernel_Name'].replace('void ', '').replace('(anonymous namespace)::', '').split('(')[0]
            agg[kn][r['Counter_Name']].append(float(r['Counter_Value']))
    for kn, cs in sorted(agg.items()):
        if kn.startswith('k'):
            print(d, kn, {c: '%.4g' % (sum(v) / len(v)) for c, v in sorted(cs.items())})
