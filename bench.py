#!/usr/bin/env python3
"""Throughput bench of the per-frame radar chain on MI355X (BASELINE.json config #2).

Workload: 16-channel x 8-beam x 4096-sample x 128-pulse echo cubes (BASELINE config #2,
``named_config('x2')``), synthetic: the v8_2 five-target scene (v8_2:28-51) evolved per
frame (v8:170-173) plus Philox noise, synthesised ON the device into a ring of distinct
frame cubes (ring > 256 MiB Infinity Cache, so every step reads its cube from HBM).
One step = one frame through DBF -> MTD -> pulse compression -> GOCA-CFAR -> S9
estimation (device) -> S10/S11 clustering (host).  Frames are batched
``--fpl`` per launch and alternate over two HIP streams.

Multi-GPU: one process per GPU (torchrun); frames are sharded (each rank processes its
own K frames, weak scaling); the only collective is an RCCL all-gather of the
detection lists at the end (inside the timed region).

Prints ONE JSON line (rank 0).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, 'radar-signal-simulation-and-target-detection_amd')
for _p in (ROOT, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=4000)
    ap.add_argument('--warmup', type=int, default=200)
    ap.add_argument('--config', default='x2')
    ap.add_argument('--fpl', type=int, default=4, help='frames per launch')
    ap.add_argument('--ring', type=int, default=8, help='distinct device-resident frame cubes')
    ap.add_argument('--profile-iters', type=int, default=50)
    ap.add_argument('--cpu-frames', type=int, default=0, help='oracle frames for cpu_baseline (0 = auto ~15 s)')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--stage-timing', action='store_true',
                    help='HIP events around every kernel in the timed region (diagnostic: overlapped durations)')
    return ap.parse_args()


def scene(cfg):
    from rsp import config as C
    sc = cfg['Sig_Config']
    G = sum(sc['point_prt_segments'])
    rmax = 0.9 * G * sc['c'] / (2 * sc['fs'])
    return [t for t in C.v8_2_targets() if t['Range'] < rmax]


def cpu_baseline(cfg, cfar, clus, W, ang, k, targets, budget_s=15.0, nframes=0):
    """The oracle (numpy/scipy restatement, complex128 like MATLAB) timed on this host."""
    import scipy.fft as sfft
    from rsp import config as C
    from oracle import chain, precompute as op
    cores = min(16, len(os.sched_getaffinity(0)))
    pre = op.precompute(cfg, W, ang, k, C.V8_FIR)
    cube = chain.synthesize_echo(targets, cfg, pre) + chain.philox_noise(cfg, 1, 20250101)
    times = []
    with sfft.set_workers(cores):
        chain.process_cube(cube, cfg, cfar, clus, pre)   # warm-up
        t_start = time.perf_counter()
        while True:
            t0 = time.perf_counter()
            chain.process_cube(cube, cfg, cfar, clus, pre)
            times.append(time.perf_counter() - t0)
            if nframes and len(times) >= nframes:
                break
            if not nframes and (time.perf_counter() - t_start > budget_s or len(times) >= 50):
                break
    med = float(np.median(times))
    return {'value': 1.0 / med, 'unit': 'frames/s', 'cores': cores, 'kind': 'port',
            'sample': '%d frames of the same %s cube, median of per-frame times (%.3f s/frame); oracle = '
                      'numpy/scipy complex128 restatement of fsf S5-S11, CFAR vectorised '
                      '(the MATLAB scalar CFAR loop fsf:192-213 would be slower)' % (len(times), 'x2', med)}


def main():
    a = parse()
    rank = int(os.environ.get('RANK', 0))
    world = int(os.environ.get('WORLD_SIZE', 1))
    local = int(os.environ.get('LOCAL_RANK', 0))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group('nccl', device_id=torch.device('cuda', local))

    from rsp import config as C
    from rsp.precompute import precompute
    from rsp.plan import Plan

    cfg, cfar, clus, W, ang, k = C.named_config(a.config)
    pre = precompute(cfg, W, ang, k, C.V8_FIR)
    plan = Plan(cfg, cfar, clus, pre, device=local if world > 1 else 0, frames_per_launch=a.fpl)
    sz = plan.sizes
    targets = scene(cfg)
    cube_bytes = sz.cube_elems * 8
    ring = [plan.device_alloc(cube_bytes) for _ in range(a.ring)]
    tg = targets
    for i, p in enumerate(ring):
        plan.synthesize_device(p, tg, frame_idx=1 + i + 1000 * rank, seed=20250101 + rank)
        tg = C.evolve_targets(tg, cfg)
    plan.sync()

    def run(nframes, base):
        for i in range(nframes):
            plan.enqueue(ring[i % a.ring], base + i)
        plan.drain()

    run(a.warmup, 0)
    plan.results(clear=True)

    if dist is not None:
        dist.barrier()
    plan.sync()
    plan.set_stage_timing(a.stage_timing)   # optional live HIP events around K1/K2/K3 of every batch
    t0 = time.perf_counter()
    run(a.steps, 1)
    res = plan.results(clear=True)
    n_targets_local = sum(len(r['final_targets']) for r in res)
    if dist is not None:
        # the one collective: gather every rank's detection list (RCCL over xGMI)
        from rsp.dist import gather_targets
        gathered = gather_targets(res, rank, world, device=local)
        n_targets_all = sum(len(r['final_targets']) for r in gathered)
    else:
        n_targets_all = n_targets_local
    plan.sync()
    if dist is not None:
        dist.barrier()
    t1 = time.perf_counter()
    live = plan.stage_times()
    plan.set_stage_timing(False)
    el = t1 - t0
    if dist is not None:
        import torch
        t = torch.tensor([el], dtype=torch.float64, device='cuda')
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())

    frames = a.steps * world
    fps = frames / el
    cells = sz.B * sz.G * sz.P
    out = None
    if rank == 0:
        # Roofline leg (after the timed region): each stage re-launched `profile_iters` times on
        # the same F-frame batch with HIP events on the kernel's stream, chip otherwise idle.  In the
        # timed region consecutive batches overlap on the device (lanes), so a kernel's span there
        # is shared with the neighbouring batch's kernels; --stage-timing records those spans too.
        prof = plan.profile_stages(ring, iters=a.profile_iters)
        stages = []
        for lv, pr in zip(live, prof):
            st = {'stage': pr['stage'], 'ms_per_launch': pr['ms'], 'frames_per_launch': pr['frames'],
                  'alg_bytes_per_launch': pr['bytes'], 'achieved_GBps': pr['bytes'] / (pr['ms'] * 1e-3) / 1e9}
            if lv['launches']:
                st['live_overlapped_ms_per_launch'] = lv['ms_total'] / lv['launches']
                st['live_frames_per_launch'] = lv['frames'] / lv['launches']
            stages.append(st)
        dom = max(stages, key=lambda s: s['ms_per_launch'])
        achieved = dom['achieved_GBps']
        traffic = None
        tf = os.path.join(ROOT, 'profiles', 'pmc_traffic_%s.json' % a.config)
        if os.path.exists(tf):
            with open(tf) as f:
                tr = json.load(f).get(dom['stage'])
            if tr is not None:   # the PMC passes run frames_per_launch = 4 like the default bench
                traffic = tr * dom['frames_per_launch'] / 4.0
                dom['pmc_traffic_bytes'] = traffic
        frame_alg_bytes = sz.C * sz.N * sz.P * 8 + cells * 8
        out = {
            'metric': 'frames/sec + range-Doppler cells/sec, 16ch×8beam×4096samp×128pulse',
            'value': fps, 'unit': 'frames/s', 'n_gpus': world, 'steps': a.steps, 'warmup': a.warmup,
            'ms_per_step': el / a.steps * 1e3, 'higher_is_better': True, 'scaling': 'weak',
            'vs_baseline': None, 'dtype': 'fp32 (complex64)', 'data': 'synthetic (device Philox noise + v8_2 targets)',
            'cells_per_s': fps * cells,
            'achieved_GBps_frame': fps * frame_alg_bytes / 1e9,
            'config': {'workload': 'BASELINE config #2: %s C=%d B=%d N=%d P=%d G=%d' % (
                a.config, sz.C, sz.B, sz.N, sz.P, sz.G), 'frames_per_launch': a.fpl, 'ring': a.ring,
                'parallelism': 'frame-sharded x%d' % world, 'used_samples': sz.used_samples,
                'targets_reported': n_targets_all},
            'roofline': {'bound': 'hbm', 'kernel': dom['stage'], 'achieved': achieved, 'peak': HBM_PEAK_GBS,
                         'unit': 'GB/s', 'frac': achieved / HBM_PEAK_GBS, 'traffic': traffic,
                         'kernel_ms': dom['ms_per_launch'], 'alg_bytes_per_launch': dom['alg_bytes_per_launch'],
                         'frames_per_launch': dom['frames_per_launch'],
                         'timing': 'roofline leg: %d isolated launches per stage, HIP events on the kernel stream '
                                   '(tools/rocprof_split.py separates them from the timed region in the rocprof '
                                   'trace)' % a.profile_iters,
                         'stages': stages},
        }
        if world == 1 and not a.no_cpu_baseline:
            out['cpu_baseline'] = cpu_baseline(cfg, cfar, clus, W, ang, k, targets, nframes=a.cpu_frames)
        else:
            out['cpu_baseline'] = None
    for p in ring:
        plan.device_free(p)
    plan.close()
    if dist is not None:
        dist.destroy_process_group()
    if out is not None:
        print(json.dumps(out))


if __name__ == '__main__':
    main()
