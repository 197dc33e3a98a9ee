"""Split a rocprofv3 kernel trace of `bench.py` into its two legs and summarise each.

bench.py runs (1) the throughput queue -- warm-up + the timed region, consecutive batches
overlapping on the device -- and then (2) the roofline leg: rsp_profile_stages launches each
stage once untimed and then `iters` timed times, one stage after the other, chip otherwise idle.
The last `iters` dispatches of each hot-path kernel are therefore the roofline leg; every earlier
dispatch belongs to the queue.  Prints a CSV: leg, kernel, calls, average / min / max ns.

usage: rocprof_split.py TRACE_DIR ITERS [OUT_CSV]
"""
import collections
import csv
import glob
import statistics
import sys


def short(name):
    n = name.replace('void ', '').replace('(anonymous namespace)::', '')
    return n.split('(')[0]


def main():
    d, iters = sys.argv[1], int(sys.argv[2])
    rows = []
    for fn in glob.glob(d + '/**/*kernel_trace.csv', recursive=True):
        rows += list(csv.DictReader(open(fn)))
    by = collections.defaultdict(list)
    for r in rows:
        by[short(r['Kernel_Name'])].append((int(r['Start_Timestamp']), int(r['End_Timestamp'])))
    out = [('leg', 'kernel', 'calls', 'avg_ns', 'min_ns', 'max_ns')]
    for k in sorted(by):
        if not k.startswith('k'):
            continue
        ds = sorted(by[k])
        legs = [('queue', ds[:-iters]), ('roofline_leg', ds[-iters:])] if k.split('<')[0] in (
            'k1_dbf_mtd', 'k1p_dbf_mtd', 'k1q_dbf_mtd', 'k2_pc', 'k3_cfar') and len(ds) > iters else [('all', ds)]
        for leg, v in legs:
            if not v:
                continue
            dur = [e - s for s, e in v]
            out.append((leg, k, len(dur), round(statistics.mean(dur)), min(dur), max(dur)))
    text = '\n'.join(','.join(str(x) for x in r) for r in out)
    print(text)
    if len(sys.argv) > 3:
        open(sys.argv[3], 'w').write(text + '\n')


if __name__ == '__main__':
    main()
