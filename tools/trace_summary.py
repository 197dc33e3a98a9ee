"""Summarise RSP_TRACE_FILE per-workgroup phase stamps (100 MHz clock -> us)."""
import collections
import sys

import numpy as np

rows = [l.strip().split(',') for l in open(sys.argv[1]) if l.strip()]
by = collections.defaultdict(list)
for r in rows:
    by[r[0]].append([int(x) for x in r[2:]])
for st, v in by.items():
    a = np.array(v, dtype=np.float64)
    a[a == 0] = np.nan
    t0 = np.nanmin(a[:, 0])
    a = (a - t0) / 100.0
    dur = a[:, 3] - a[:, 0]
    print('%s n=%d kernel span %.1f us' % (st, len(a), np.nanmax(a[:, 3])))
    print('   start: med %.1f max %.1f' % (np.nanmedian(a[:, 0]), np.nanmax(a[:, 0])))
    for i, name in [(1, 'ph1'), (2, 'ph2'), (3, 'ph3')]:
        d = a[:, i] - a[:, i - 1]
        print('   %s: med %.2f p90 %.2f max %.2f' % (name, np.nanmedian(d), np.nanpercentile(d, 90), np.nanmax(d)))
    print('   wg dur: med %.2f max %.2f' % (np.nanmedian(dur), np.nanmax(dur)))
