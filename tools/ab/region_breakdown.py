"""Host-side split of bench.py's timed region at x2 (the driver's --steps 20): enqueue_many,
drain, results_rows, sync -- where the region's fixed ~0.3 ms goes.  usage: region_breakdown.py [STEPS] [REPS]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'radar-signal-simulation-and-target-detection_amd'))
from rsp import config as C, _abi  # noqa: E402
if os.environ.get('AB_LIB'):   # timing experiments only: an A/B variant of librsp.so
    _abi.LIB_PATH = os.environ['AB_LIB']
from rsp.precompute import precompute  # noqa: E402
from rsp.plan import Plan  # noqa: E402
import bench  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
cfg, cfar, clus, W, ang, k = C.named_config('x2')
plan = Plan(cfg, cfar, clus, precompute(cfg, W, ang, k, C.V8_FIR), frames_per_launch=8)
tg = bench.scene(cfg)
ring = [plan.device_alloc(plan.cube_bytes) for _ in range(8)]
for i, p in enumerate(ring):
    plan.synthesize_device(p, tg, frame_idx=i + 1)
plan.sync()
seq = [ring[i % 8] for i in range(steps * 8)]
plan.enqueue_many([ring[i % 8] for i in range(800)], range(800))   # warm-up: 100 batches
plan.drain()
plan.results_rows(clear=True)
acc = np.zeros(5)
for r in range(reps):
    plan.sync()
    t0 = time.perf_counter()
    plan.enqueue_many(seq, range(1, 1 + len(seq)))
    t1 = time.perf_counter()
    plan.drain()
    t2 = time.perf_counter()
    rows = plan.results_rows(clear=True)
    t3 = time.perf_counter()
    plan.sync()
    t4 = time.perf_counter()
    acc += np.array([t1 - t0, t2 - t1, t3 - t2, t4 - t3, t4 - t0]) * 1e3
acc /= reps
print('steps %d: enqueue_many %.3f ms, drain %.3f, results_rows %.3f, sync %.3f, total %.3f (%.4f ms/step)' % (
    steps, acc[0], acc[1], acc[2], acc[3], acc[4], acc[4] / steps))
