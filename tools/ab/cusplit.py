"""CU-split experiment: K1 of one batch and K2 of another on disjoint CU sets at the same time
(rsp_profile_split).  Prints per split: wall ms per pair, K1 and K2 stream ms.  The CUs of K1 are
spread over the 8 XCDs (CU ids c with c % 32 < n1 / 8 in each 32-CU XCD block -- placement is for
speed only).  usage: cusplit.py [CONFIG] [PREC]"""
import ctypes as ct
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, 'radar-signal-simulation-and-target-detection_amd'))
if os.environ.get('AB_LIB'):
    from rsp import _abi  # noqa: E402
    _abi.LIB_PATH = os.environ['AB_LIB']
from rsp import config as C  # noqa: E402
from rsp._abi import lib, check  # noqa: E402
from rsp.precompute import precompute  # noqa: E402
from rsp.plan import Plan  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else 'x2'
prec = sys.argv[2] if len(sys.argv) > 2 else 'c128'
cfg, cfar, clus, W, ang, k = C.named_config(name)
plan = Plan(cfg, cfar, clus, precompute(cfg, W, ang, k, C.V8_FIR), frames_per_launch=8, precision=prec)
cubes = [plan.device_alloc(plan.cube_bytes) for _ in range(8)]
tg = C.v8_2_targets()
for i, p in enumerate(cubes):
    plan.synthesize_device(p, tg, 1 + i)
arr = (ct.c_void_p * 8)(*cubes)
NCU = 256


def mask(sel):
    m = (ct.c_uint32 * (NCU // 32))()
    for c in range(NCU):
        if sel(c):
            m[c // 32] |= 1 << (c % 32)
    return m


out = []
for n1 in (0, 256, 64, 96, 128, 160):
    for mode in ('xcd', 'lin'):
        if n1 in (0, 256) and mode == 'lin':
            continue
        per = n1 // 8
        if mode == 'xcd':   # the same number of K1 CUs in every XCD (CU id c -> XCD c // 32, assumed)
            s1 = (lambda c, per=per: c % 32 < per)
        else:               # K1 on every (256 / n1)-th CU id
            s1 = (lambda c, n1=n1: (c * n1) // NCU != ((c + 1) * n1) // NCU)
        m1 = mask(s1) if n1 else None
        m2 = mask(lambda c: not s1(c)) if n1 < 256 else None
        ms = (ct.c_float * 3)()
        check(lib().rsp_profile_split(plan.h, arr, 8, m1, m2, NCU // 32, 20, ms))
        out.append({'k1_cus': n1, 'mode': mode, 'wall_ms': ms[0], 'k1_ms': ms[1], 'k2_ms': ms[2]})
        print(json.dumps(out[-1]), flush=True)
for p in cubes:
    plan.device_free(p)
plan.close()
