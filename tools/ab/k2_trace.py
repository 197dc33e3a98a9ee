"""K2 per-job-type workgroup phase times from an RSP_TRACE_FILE dump (x2 job layout:
narrow 0..127, medium 128..383, long block 0 384..895, long block 1 896..1407)."""
import sys

import numpy as np

rows = [l.strip().split(',') for l in open(sys.argv[1]) if l.strip().startswith('k2')]
a = np.array([[int(x) for x in r[1:]] for r in rows], float)
idx = a[:, 0].astype(int)
t = a[:, 1:]
ok = (t > 0).all(1)
tt = (t - t[ok, 0].min()) / 100.0
wg = idx % 1408
dur = tt[:, 3] - tt[:, 0]
for name, lo, hi in [('narrow', 0, 128), ('med', 128, 384), ('long b0', 384, 896), ('long b1', 896, 1408)]:
    m = ok & (wg >= lo) & (wg < hi)
    print('%-8s n=%4d dur %.2f phases %s start med %.1f' % (name, m.sum(), dur[m].mean(),
                                                          np.round(np.diff(tt[m], axis=1).mean(0), 2),
                                                          np.median(tt[m, 0])))
span = tt[ok, 3].max()
ts = np.linspace(0, span, 16)
print('span %.1f conc %s' % (span, [int(((tt[ok, 0] <= x) & (tt[ok, 3] > x)).sum()) for x in ts]))
