"""Dump the complex RD map of one synthesised frame (x2 by default) computed by a librsp variant
(AB_LIB) to an .npy file, for bit-level comparisons between A/B builds.
usage: AB_LIB=exp/ab/librsp_x.so rdm_dump.py OUT.npy [CONFIG] [PREC]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, 'radar-signal-simulation-and-target-detection_amd'))
if os.environ.get('AB_LIB'):
    from rsp import _abi  # noqa: E402
    _abi.LIB_PATH = os.environ['AB_LIB']
from rsp import config as C  # noqa: E402
from rsp.precompute import precompute  # noqa: E402
from rsp.plan import Plan  # noqa: E402

name = sys.argv[2] if len(sys.argv) > 2 else 'x2'
prec = sys.argv[3] if len(sys.argv) > 3 else 'c128'
cfg, cfar, clus, W, ang, k = C.named_config(name)
plan = Plan(cfg, cfar, clus, precompute(cfg, W, ang, k, C.V8_FIR), frames_per_launch=2, precision=prec)
d = plan.device_alloc(plan.cube_bytes)
m = plan.device_alloc(plan.sizes.rdm_elems * plan.sizes.elem_bytes)
plan.synthesize_device(d, C.v8_2_targets(), 1)
plan.enqueue_many([d, d], [1, 2], rdms=[m, m])
plan.drain()
np.save(sys.argv[1], plan.rdm_from_device(m))
plan.close()
