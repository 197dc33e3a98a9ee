"""MFMA utilisation from rocprofv3 --pmc passes (usage: mfma_summary.py LABEL:DIR ... > file).

Per kernel (mean over its launches): flops = SQ_INSTS_VALU_MFMA_MOPS_F64 x 512 (f64) or
SQ_INSTS_VALU_MFMA_MOPS_F32 x 512 (f32); MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE /
8 XCDs x 1024 SIMDs) (MI355X_MICROARCH.md).  Each line carries the code hash of the kernel in the
built library (rsp/kernel_hashes.json, tools/kernel_hashes.py), so the file states which code
its counters describe."""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
hp = os.path.join(ROOT, 'radar-signal-simulation-and-target-detection_amd', 'rsp', 'kernel_hashes.json')
hashes = json.load(open(hp)) if os.path.exists(hp) else {}
print('MFMA counters (rocprofv3 --pmc, one pass per config; means over launches).  flops = MOPS x 512;')
print('MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs).  kernel hash = rsp/kernel_hashes.json.')
for arg in sys.argv[1:]:
    label, d = arg.split(':', 1)
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for fn in glob.glob(d + '/**/*counter_collection.csv', recursive=True):
        for r in csv.DictReader(open(fn)):
            kn = r['Kernel_Name'].replace('void ', '').replace('(anonymous namespace)::', '').split('(')[0]
            agg[kn][r['Counter_Name']].append(float(r['Counter_Value']))
    for kn, cs in sorted(agg.items()):
        c = {k: sum(v) / len(v) for k, v in cs.items()}
        mops = c.get('SQ_INSTS_VALU_MFMA_MOPS_F64', 0.0) + c.get('SQ_INSTS_VALU_MFMA_MOPS_F32', 0.0)
        if mops <= 0:
            continue
        gui = c.get('GRBM_GUI_ACTIVE', 0.0)
        busy = c.get('SQ_VALU_MFMA_BUSY_CYCLES', 0.0) / (gui / 8 * 1024) if gui else float('nan')
        base = kn.split('<')[0]
        print('%-9s %-46s MOPS %.4g -> %.4g flop/launch; MFMA busy %.3f; kernel hash %s; raw %s' % (
            label, kn, mops, mops * 512, busy, hashes.get(base), {k: '%.4g' % v for k, v in sorted(c.items())}))
