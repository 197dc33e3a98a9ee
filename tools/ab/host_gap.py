"""Host-side gaps of the throughput queue from a rocprofv3 --kernel-trace --hip-trace run:
per batch, when the last kernel (K3) of lane batch i ended vs when the next K1 launched on
that stream started, and the HIP API calls in between.   usage: host_gap.py TRACE_DIR"""
import csv
import glob
import sys

d = sys.argv[1]
kt = list(csv.DictReader(open(glob.glob(d + '/**/*kernel_trace.csv', recursive=True)[0])))
ht = list(csv.DictReader(open(glob.glob(d + '/**/*hip_api_trace.csv', recursive=True)[0])))


def nm(n):
    for k in ('k1p', 'k2_pc', 'k3_cfar'):
        if k in n:
            return k
    return None


ks = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), nm(r['Kernel_Name']), r['Stream_Id'])
            for r in kt if nm(r['Kernel_Name']))
api = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Function']) for r in ht)
# take the last 60 chain kernels (a steady region)
ks = ks[-120:]
t0 = ks[0][0]
for s, e, n, q in ks[:45]:
    print('%9.1f %9.1f %7.1f %-8s stream %s' % ((s - t0) / 1e3, (e - t0) / 1e3, (e - s) / 1e3, n, q))
print('--- API calls in the same window')
tend = ks[44][1]
for s, e, f in api:
    if t0 <= s <= tend and f not in ('hipGetLastError',):
        print('%9.1f %9.1f %7.1f %s' % ((s - t0) / 1e3, (e - t0) / 1e3, (e - s) / 1e3, f))
