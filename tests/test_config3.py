"""BASELINE config #3 on the GPU: a batch of 512 independent x2 frames, sharded, with the
detection-list gather (main_simulate_echoes_with_array_v8.m:164-190 loops over
independent frames, each evolved per v8:170-173 and processed by fun_process_single_frame).

Two sharded drivers are checked, each against paths the parity suite pins to the oracle:

* ``rsp_process_targets_multi`` (one process, one host thread per plan; the MEX / loadlibrary
  form of config #3): 512 frames split over 8 plans -- eight shares of 64 frames as on the 8 GPUs
  of a node, here all on the box's one GPU.  Every frame's gathered final targets must equal the
  synchronous per-frame ``rsp_process_targets`` result (same kernels, so identical, not close),
  in frame order; frames 1, 64, 65, 300 and 512 (first / last of shares, one in the middle) are
  also checked against ``oracle.chain`` on the very cube the device synthesised (c128 tolerance
  of test_gpu_parity: every field within 1e-9).
* one process per rank (the bench's torchrun form): 2 ranks on the one GPU, each pushing its
  contiguous shard of frames through the device queue, packing ``Plan.results_rows`` and
  gathering with ``rsp.dist.gather_rows`` (gloo here; the same call runs over RCCL on 8 GPUs).
  Rank 0 checks the gathered rows, frame by frame, against the per-frame path.
"""
import os
import socket

import numpy as np
import pytest

from _scen import scenario, targets_for, device_cube
from oracle import chain
from rsp import config as C
from rsp.plan import Plan, process_targets_multi

pytestmark = pytest.mark.gpu

N_FRAMES = 512
N_PLANS = 8
ORACLE_FRAMES = (1, 64, 65, 300, 512)


def _frames(s, n):
    """(targets, frame_idx) of frames 1..n: the v8_2 scene evolved per frame (v8:170-173)."""
    t = targets_for('x2')
    out = []
    for f in range(1, n + 1):
        out.append((t, f))
        t = C.evolve_targets(t, s['cfg'])
    return out


def _close(a, b):
    assert len(a) == len(b)
    for x, y in zip(a, b):
        for f in ('Range', 'Velocity', 'Angle', 'Power'):
            assert y[f] == pytest.approx(x[f], rel=1e-9, abs=1e-9), f


def test_config3_512_frames_multi_plan():
    s = scenario('x2')
    frames = _frames(s, N_FRAMES)
    plans = [Plan(s['cfg'], s['cfar'], s['clus'], s['pre_p'], frames_per_launch=8) for _ in range(N_PLANS)]
    try:
        got = process_targets_multi(plans, frames)
        ref_plan = plans[0]
        ref = [ref_plan.process_targets(t, frame_idx=f)['final_targets'] for t, f in frames]
        assert len(got) == N_FRAMES
        assert sum(len(r) for r in ref) >= N_FRAMES   # every frame sees targets
        for j in range(N_FRAMES):
            assert got[j] == ref[j], 'frame %d' % (j + 1)
        for f in ORACLE_FRAMES:   # the device's own cube through the oracle
            t, fi = frames[f - 1]
            cube = device_cube(ref_plan, t, frame_idx=fi)
            fin = chain.process_cube(cube, s['cfg'], s['cfar'], s['clus'], s['pre_o'])
            _close(fin, got[f - 1])
    finally:
        for p in plans:
            p.close()


def _free_port():
    so = socket.socket()
    so.bind(('127.0.0.1', 0))
    port = so.getsockname()[1]
    so.close()
    return port


RANK_FRAMES = 96


def _rank_worker(rank, world, port, q):
    import torch.distributed as dist
    from rsp.dist import gather_rows, shard_frames
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        s = scenario('x2')
        frames = _frames(s, RANK_FRAMES)
        mine = shard_frames(RANK_FRAMES, rank, world)
        plan = Plan(s['cfg'], s['cfar'], s['clus'], s['pre_p'], device=0, frames_per_launch=8)
        ring = [plan.device_alloc(plan.cube_bytes) for _ in mine]
        for p, f in zip(ring, mine):
            plan.synthesize_device(p, frames[f - 1][0], frame_idx=f)
        plan.sync()
        plan.enqueue_many(ring, mine)
        plan.drain()
        rows = plan.results_rows(clear=True)
        counts, bufs = gather_rows(rows, rank, world)
        out = None
        if rank == 0:
            gathered = np.concatenate([b[:c] for c, b in zip(counts, bufs)])
            want = []
            for t, f in frames:
                r = plan.process_targets(t, frame_idx=f)['final_targets']
                want += [(f, x['Range'], x['Velocity'], x['Angle'], x['Power']) for x in r] or [(f,) + (np.nan,) * 4]
            out = (gathered, np.asarray(want, np.float64))
        for p in ring:
            plan.device_free(p)
        plan.close()
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def test_config3_two_ranks_gather_rows():
    import torch.multiprocessing as mp
    world = 2
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    gathered, want = outs[0]
    assert gathered.shape == want.shape
    assert [int(f) for f in gathered[:, 0]] == [int(f) for f in want[:, 0]]   # frame order across ranks
    np.testing.assert_array_equal(gathered, want)
