"""Overlap of the queue's kernels in a rocprofv3 kernel trace of bench.py (steady state).

For every K1 launch of the timed region: how long it shares the device with the previous
batch's K2 / K3, and the device-busy union vs the sum of kernel durations.
usage: timeline.py TRACE_DIR [n_skip]"""
import csv
import glob
import sys

d = sys.argv[1]
rows = []
for fn in glob.glob(d + '/**/*kernel_trace.csv', recursive=True):
    rows += list(csv.DictReader(open(fn)))
ev = []
for r in rows:
    n = r['Kernel_Name']
    k = 'K1' if 'k1' in n else 'K2' if 'k2_pc' in n else 'K3' if 'k3_cfar' in n else None
    if k:
        ev.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), k))
ev.sort()
# the queue leg: the longest run of K1/K2/K3 with gaps < 50 us
runs, cur = [], [ev[0]]
for e in ev[1:]:
    if e[0] - max(x[1] for x in cur[-6:]) < 50000:
        cur.append(e)
    else:
        runs.append(cur)
        cur = [e]
runs.append(cur)
q = max(runs, key=len)
skip = int(sys.argv[2]) if len(sys.argv) > 2 else len(q) // 4
q = q[skip:]
t0, t1 = q[0][0], max(e[1] for e in q)
tot = {k: sum(e[1] - e[0] for e in q if e[2] == k) for k in ('K1', 'K2', 'K3')}
cnt = {k: sum(1 for e in q if e[2] == k) for k in ('K1', 'K2', 'K3')}
# union of busy time
busy, end = 0, t0
for s, e, _ in sorted(q):
    if e > end:
        busy += e - max(s, end)
        end = e
# pairwise overlap
def ov(a, b):
    o = 0
    A = [e for e in q if e[2] == a]
    B = [e for e in q if e[2] == b]
    for s1, e1, _ in A:
        for s2, e2, _ in B:
            o += max(0, min(e1, e2) - max(s1, s2))
    return o
print('launches', cnt, 'span %.1f us' % ((t1 - t0) / 1e3))
print('per-launch mean us', {k: round(tot[k] / max(cnt[k], 1) / 1e3, 1) for k in tot})
print('sum of durations %.1f us, busy union %.1f us, overlap %.1f us' % (sum(tot.values()) / 1e3, busy / 1e3,
                                                                         (sum(tot.values()) - busy) / 1e3))
print('pairwise overlap us per batch', {a + b: round(ov(a, b) / max(cnt['K1'], 1) / 1e3, 1)
                                        for a, b in (('K1', 'K2'), ('K1', 'K3'), ('K2', 'K3'), ('K2', 'K2'))})
