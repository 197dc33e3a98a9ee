"""Profiling driver: time/profile each device stage of one config #2 frame N times.

Used under rocprofv3 (kernel trace / PMC passes); prints the in-process HIP-event
stage times as JSON.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'radar-signal-simulation-and-target-detection_amd'))

from rsp import config as C  # noqa: E402
from rsp.precompute import precompute  # noqa: E402
from rsp.plan import Plan  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else 'x2'
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    cfg, cfar, clus, W, ang, k = C.named_config(name)
    pre = precompute(cfg, W, ang, k, C.V8_FIR)
    plan = Plan(cfg, cfar, clus, pre)
    p = plan.device_alloc(plan.sizes.cube_elems * 8)
    plan.synthesize_device(p, C.v8_2_targets(), 1)
    st = plan.profile_stages(p, iters=iters)
    print(json.dumps(st))
    plan.device_free(p)
    plan.close()


if __name__ == '__main__':
    main()
