"""Multi-process (gloo, world_size 2, CPU) test of the frame-sharded path.

Each rank takes its contiguous shard of frames (rsp.dist.shard_frames), produces
final_targets for them, and the detection lists are gathered with the same code the
bench runs over RCCL (rsp.dist.gather_targets).  Without a GPU the per-frame work is
done by the oracle; the thing under test is the sharding + gather, which must give
every rank the single-process result for all frames, in frame order.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from rsp.dist import shard_frames

N_FRAMES = 5


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _frame_results(frames):
    """Per-frame final_targets of the 'small' scene (targets evolved per frame, v8:170-173) via the oracle."""
    from oracle import chain
    from _scen import scenario, targets_for, noisy_cube
    from rsp import config as C
    s = scenario('small')
    tg = targets_for('small')
    out = []
    for f in range(1, max(frames) + 1 if frames else 1):
        if f in frames:
            cube = noisy_cube(s, tg, frame_idx=f)
            fin = chain.process_cube(cube.astype(np.complex128), s['cfg'], s['cfar'], s['clus'], s['pre_o'])
            out.append({'frame_idx': f, 'final_targets': fin})
        tg = C.evolve_targets(tg, s['cfg'])
    return out


def _worker(rank, world, port, q):
    import torch.distributed as dist
    from rsp.dist import gather_targets
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        mine = shard_frames(N_FRAMES, rank, world)
        res = _frame_results(mine)
        got = gather_targets(res, rank, world)
        q.put((rank, [(g['rank'], g['frame_idx'], [(t['Range'], t['Velocity'], t['Angle'], t['Power'])
                                                   for t in g['final_targets']]) for g in got]))
    finally:
        dist.destroy_process_group()


def test_shard_frames_partition():
    for n in (0, 1, 5, 64, 512):
        for w in (1, 2, 3, 8):
            parts = [shard_frames(n, r, w) for r in range(w)]
            assert sum(parts, []) == list(range(1, n + 1))
            assert max(map(len, parts)) - min(map(len, parts)) <= 1


def test_gather_two_ranks_equals_single_process():
    world = 2
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert outs[0] == outs[1]                       # every rank holds the same gathered list
    want = _frame_results(list(range(1, N_FRAMES + 1)))
    got = outs[0]
    assert [f for _, f, _ in got] == list(range(1, N_FRAMES + 1))
    assert [r for r, _, _ in got] == [0, 0, 0, 1, 1]
    for (_, f, tl), w in zip(got, want):
        assert len(tl) == len(w['final_targets'])
        for t, u in zip(tl, w['final_targets']):
            assert t == pytest.approx((u['Range'], u['Velocity'], u['Angle'], u['Power']), rel=1e-12)
    assert sum(len(tl) for _, _, tl in got) > 0


def _census_worker(rank, world, port, q):
    import sys
    import torch.distributed as dist
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), LOCAL_RANK=str(rank))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        q.put((rank, bench.rank_census(dist, rank)))
    finally:
        dist.destroy_process_group()


def test_bench_rank_census_two_ranks():
    """The census bench.py puts in an N > 1 line: world size and backend from torch.distributed
    itself, and every rank's device ordinal, gathered (gloo here; RCCL on the node)."""
    world = 2
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_census_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        c = outs[r]
        assert c['world_size'] == world and c['backend'] == 'gloo'
        assert [x['rank'] for x in c['ranks']] == [0, 1]
        assert [x['device'] for x in c['ranks']] == [0, 1]
        assert c['distinct_devices'] == 2


CONFIG3_FRAMES, CONFIG3_WORLD = 512, 8


def _config3_results(frames):
    """Deterministic stand-in final_targets per frame id (0..3 targets; frames with none keep
    their NaN marker row): what each rank's plan returns for its frames, without the chain."""
    out = []
    for f in frames:
        n = (f * 7) % 4
        out.append({'frame_idx': f, 'final_targets': [
            {'Range': 1000.0 + 3.5 * f + j, 'Velocity': 0.25 * (f % 17) - j, 'Angle': 0.01 * f + j,
             'Power': 1.0 / (f + j)} for j in range(n)]})
    return out


def _config3_worker(rank, world, port, q):
    import torch.distributed as dist
    from rsp.dist import gather_rows, shard_frames as shard, _pack
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        mine = shard(CONFIG3_FRAMES, rank, world)
        counts, bufs = gather_rows(_pack(_config3_results(mine)), rank, world)
        rows = np.concatenate([b[:c] for c, b in zip(counts, bufs)])
        q.put((rank, len(mine), counts, rows))
    finally:
        dist.destroy_process_group()


def test_config3_split_eight_ranks_equals_single_process():
    """BASELINE config #3's actual split rehearsed as 8 processes (gloo, CPU): 512 frame ids
    sharded by shard_frames (64 per rank, v8:164-190 frames are independent), each rank's packed
    (frame_idx, Range, Velocity, Angle, Power) rows all-gathered through gather_rows -- the code
    bench.py runs over RCCL.  Every rank must hold the one-process rows of frames 1..512, in frame
    order, bit for bit."""
    world = CONFIG3_WORLD
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_config3_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = dict((r, (n, c, rows)) for r, n, c, rows in (q.get(timeout=300) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from rsp.dist import _pack
    want = _pack(_config3_results(list(range(1, CONFIG3_FRAMES + 1))))
    assert [outs[r][0] for r in range(world)] == [CONFIG3_FRAMES // world] * world
    for r in range(world):
        n, counts, rows = outs[r]
        assert sum(counts) == want.shape[0]
        assert np.array_equal(rows, want, equal_nan=True)
    f = want[:, 0]
    assert np.all(np.diff(f) >= 0) and set(f.astype(int)) == set(range(1, CONFIG3_FRAMES + 1))
