"""Device time of the S4 + S4.1 synthesis (rsp_profile_synthesis) at x2 and the reference frame.
usage: [AB_LIB=exp/ab/librsp_<v>.so] synth_prof.py [ITERS]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'radar-signal-simulation-and-target-detection_amd'))
from rsp import config as C, _abi  # noqa: E402
if os.environ.get('AB_LIB'):   # timing experiments only: an A/B variant of librsp.so
    _abi.LIB_PATH = os.environ['AB_LIB']
from rsp.precompute import precompute  # noqa: E402
from rsp.plan import Plan  # noqa: E402
import bench  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 50
out = {}
for name in ('x2', 'reference'):
    cfg, cfar, clus, W, ang, k = C.named_config(name)
    plan = Plan(cfg, cfar, clus, precompute(cfg, W, ang, k, C.V8_FIR), frames_per_launch=1)
    d = plan.device_alloc(plan.cube_bytes)
    r = plan.profile_synthesis(d, bench.scene(cfg), iters=iters)
    out[name] = round(r['ms'] * 1e3, 1)
    plan.device_free(d)
    plan.close()
print(json.dumps(out))
