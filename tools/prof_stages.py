"""Profiling driver: time/profile each device stage of one config #2 frame N times.

Used under rocprofv3 (kernel trace / PMC passes); prints the in-process HIP-event
stage times as JSON.  usage: prof_stages.py [CONFIG] [ITERS] [FRAMES_PER_LAUNCH] [PREC] [rdm]
(rdm: K2 also writes every frame's complex RD map, as rsp_enqueue_device_rdm)
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'radar-signal-simulation-and-target-detection_amd'))
if os.environ.get('AB_LIB'):   # timing experiments only (tools/ab/ab.sh): an A/B variant of librsp.so
    from rsp import _abi  # noqa: E402
    _abi.LIB_PATH = os.environ['AB_LIB']

from rsp import config as C  # noqa: E402
from rsp.precompute import precompute  # noqa: E402
from rsp.plan import Plan  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else 'x2'
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    nf = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    cfg, cfar, clus, W, ang, k = C.named_config(name)
    pre = precompute(cfg, W, ang, k, C.V8_FIR)
    prec = sys.argv[4] if len(sys.argv) > 4 else 'c128'
    plan = Plan(cfg, cfar, clus, pre, frames_per_launch=nf, precision=prec)
    # a ring of >= 8 cubes (> the 256 MiB Infinity Cache at x2), rotated over by the launches
    cubes = [plan.device_alloc(plan.cube_bytes) for _ in range(max(nf, 8))]
    tg = C.v8_2_targets()
    for i, p in enumerate(cubes):
        plan.synthesize_device(p, tg, 1 + i)
        tg = C.evolve_targets(tg, cfg)
    rdms = None
    if len(sys.argv) > 5 and sys.argv[5] == 'rdm':
        rdms = [plan.device_alloc(plan.sizes.rdm_elems * plan.sizes.elem_bytes) for _ in range(nf)]
    st = plan.profile_stages(cubes, iters=iters, d_rdms=rdms)
    print(json.dumps(st))
    for p in rdms or []:
        plan.device_free(p)
    for p in cubes:
        plan.device_free(p)
    plan.close()


if __name__ == '__main__':
    main()
