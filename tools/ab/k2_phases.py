"""K2 phase timeline of one 8-frame x2 launch (diagnostic builds, -DRSP_DEBUG_KNOBS only).

usage: AB_LIB=exp/ab/librsp_dbg.so python3 tools/ab/k2_phases.py [CONFIG] [PREC] [OUT.npz]
Runs the roofline leg's K1/K2/K3 launches (profile_stages) with rsp_k2_trace set, so the last K2
launch leaves, per workgroup, s_memrealtime stamps (100 MHz) at its phase boundaries, its job
type and its hardware position; prints per-job-type phase means and the CU-level occupancy.
"""
import collections
import ctypes as ct
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, 'radar-signal-simulation-and-target-detection_amd'))
from rsp import _abi  # noqa: E402
if os.environ.get('AB_LIB'):
    _abi.LIB_PATH = os.environ['AB_LIB']
from rsp import config as C  # noqa: E402
from rsp.precompute import precompute  # noqa: E402
from rsp.plan import Plan  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else 'x2'
    prec = sys.argv[2] if len(sys.argv) > 2 else 'c128'
    out = sys.argv[3] if len(sys.argv) > 3 else None
    nf = 8
    cfg, cfar, clus, W, ang, k = C.named_config(name)
    pre = precompute(cfg, W, ang, k, C.V8_FIR)
    plan = Plan(cfg, cfar, clus, pre, frames_per_launch=nf, precision=prec)
    cubes = [plan.device_alloc(plan.cube_bytes) for _ in range(8)]
    tg = C.v8_2_targets()
    for i, p in enumerate(cubes):
        plan.synthesize_device(p, tg, 1 + i)
        tg = C.evolve_targets(tg, cfg)
    nwg_max = 8 * 40000
    tb = plan.device_alloc(nwg_max * 8 * 8)
    L = _abi.lib()
    L.rsp_debug_set_k2_trace.argtypes = [ct.c_void_p]
    L.rsp_debug_set_k2_trace.restype = ct.c_int
    assert L.rsp_debug_set_k2_trace(tb) == 0
    st = plan.profile_stages(cubes, iters=5)
    assert L.rsp_debug_set_k2_trace(None) == 0
    raw = plan.device_download(tb, nwg_max * 8 * 8 // 8, np.uint64).reshape(-1, 8)
    used = raw[:, 0] != 0
    t = raw[used].astype(np.int64)
    t0 = t[:, 0].min()
    tt = (t[:, :6] - t0) / 100.0   # us
    typ = t[:, 6]
    hw = t[:, 7]
    xcc = (hw >> 32) & 0xF
    cu = (hw >> 8) & 0xF
    sh = (hw >> 12) & 0x1
    se = (hw >> 13) & 0x7
    cuid = ((xcc * 8 + se) * 2 + sh) * 16 + cu
    print('stages', [(s['stage'], round(s['ms'] * 1e3, 1)) for s in st])
    print('workgroups', len(t), 'span %.1f us' % (tt[:, 5].max()))
    names = {0: 'FIR', 16: 'mix2560'}
    for ty in sorted(set(typ.tolist())):
        m = typ == ty
        nm = names.get(ty, 'pow2 lg%d' % (ty - 16))
        d = tt[m]
        ph = [np.mean(d[:, i + 1] - d[:, i]) if np.all(d[:, i + 1] > 0) else float('nan') for i in range(5)]
        print('%-10s n=%5d  span %.2f us  phases %s' % (nm, m.sum(), np.mean(d[:, 5] - d[:, 0]),
                                                       ' '.join('%.2f' % x for x in ph)))
    # phase breakdown where stamps exist (mix: 0..5; pow2: 0,1,3,5; FIR: 0,1,5)
    for ty in sorted(set(typ.tolist())):
        m = typ == ty
        d = tt[m]
        print(names.get(ty, 'pow2'), 'load->first barrier %.2f' % np.mean(d[:, 1] - d[:, 0]),
              'rest %.2f' % np.mean(d[:, 5] - d[:, 1]))
    # occupancy: workgroups resident per CU over time (time-weighted mean)
    ncu = len(set(cuid.tolist()))
    occ = []
    for c in set(cuid.tolist()):
        m = cuid == c
        ev = sorted([(a, 1) for a in tt[m, 0]] + [(b, -1) for b in tt[m, 5]])
        cur = 0
        last = ev[0][0]
        acc = collections.Counter()
        for x, dlt in ev:
            acc[cur] += x - last
            cur += dlt
            last = x
        occ.append(acc)
    tot = collections.Counter()
    for a in occ:
        tot.update(a)
    s = sum(tot.values())
    print('CUs', ncu, 'resident-WG time fractions', {k: round(v / s, 3) for k, v in sorted(tot.items())})
    gaps = []
    if out:
        np.savez(out, tt=tt, typ=typ, cuid=cuid)
    plan.device_free(tb)
    for p in cubes:
        plan.device_free(p)
    plan.close()


if __name__ == '__main__':
    main()
