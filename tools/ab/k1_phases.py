"""Persistent K1 phase timeline of one 8-frame launch (diagnostic builds, -DRSP_DEBUG_KNOBS only).

usage: AB_LIB=exp/ab/librsp_dbg.so python3 tools/ab/k1_phases.py [CONFIG] [PREC]
Runs the roofline leg's launches (profile_stages) with rsp_k1_trace set, so the last K1 launch
leaves, per workgroup and loop iteration, wave 0's s_memrealtime stamps (100 MHz): loop top, after
the slow-time FFT + z stores of tile n, after the DBF of tile n + 1 (its loads' wait, the MFMAs,
the LDS stores) and the next load issue, after the tile barrier.  Prints the mean phase lengths.
"""
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
    cfg, cfar, clus, W, ang, k = C.named_config(name)
    pre = precompute(cfg, W, ang, k, C.V8_FIR)
    plan = Plan(cfg, cfar, clus, pre, frames_per_launch=8, precision=prec)
    cubes = [plan.device_alloc(plan.cube_bytes) for _ in range(8)]
    tg = C.v8_2_targets()
    for i, p in enumerate(cubes):
        plan.synthesize_device(p, tg, 1 + i)
        tg = C.evolve_targets(tg, cfg)
    nwg, nit = 1024, 64
    nbytes = nwg * nit * 4 * 8
    tb = plan.device_alloc(nbytes)
    L = _abi.lib()
    L.rsp_debug_set_k1_trace.argtypes = [ct.c_void_p]
    L.rsp_debug_set_k1_trace.restype = ct.c_int
    assert L.rsp_debug_set_k1_trace(tb) == 0
    st = plan.profile_stages(cubes, iters=3)
    assert L.rsp_debug_set_k1_trace(None) == 0
    raw = plan.device_download(tb, nbytes // 8, np.uint64).reshape(nwg, nit, 4).astype(np.int64)
    used = raw[:, :, 0] != 0
    print('stages', [(s['stage'], round(s['ms'] * 1e3, 1)) for s in st])
    print('workgroups %d, iterations per workgroup %.1f' % (int(used.any(axis=1).sum()), used.sum() / max(used.any(axis=1).sum(), 1)))
    full = used & (raw[:, :, 3] != 0)
    d = raw[full]
    ph = (d[:, 1:] - d[:, :-1]) / 100.0   # us
    nxt = []
    for w in range(nwg):   # loop top to the next top (includes the loop overhead)
        r = raw[w][used[w]]
        if len(r) > 1:
            nxt.extend(((r[1:, 0] - r[:-1, 0]) / 100.0).tolist())
    if plan.sizes.P & (plan.sizes.P - 1):   # k1q_dbf_mtd (factored DFT): stamps at DBF | barrier | DFT
        print('per tile (wave 0, us): DBF (load wait, MFMA, LDS) + next issue %.2f | barrier %.2f | pass 1 + pass 2 '
              '(+ z stores) %.2f | top to top %.2f' % (ph[:, 0].mean(), ph[:, 1].mean(), ph[:, 2].mean(), np.mean(nxt)))
    else:
        print('per tile (wave 0, us): FFT + z stores %.2f | DBF of the next tile (load wait, MFMA, LDS) + next issue %.2f | '
              'barrier %.2f | top to top %.2f' % (ph[:, 0].mean(), ph[:, 1].mean(), ph[:, 2].mean(), np.mean(nxt)))
    for q in (10, 50, 90):
        print('  p%d: %.2f %.2f %.2f' % (q, np.percentile(ph[:, 0], q), np.percentile(ph[:, 1], q), np.percentile(ph[:, 2], q)))
    t0 = raw[used][:, 0].min()
    first = raw[:, 0, 0]
    print('launch span %.1f us; first-iteration start spread %.1f us' % ((raw[full][:, 3].max() - t0) / 100.0,
                                                                        (first[first > 0].max() - first[first > 0].min()) / 100.0))


if __name__ == '__main__':
    main()
