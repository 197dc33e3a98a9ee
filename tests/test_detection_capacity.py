"""Detection lists without a capacity limit (fsf:215-221 appends every CFAR hit with
all_raw_detections(end+1, :)).

At a very low T_CFAR nearly every cell under test is a hit: one K3 tile then holds more than
its 1024-entry LDS queue (the hits past it reserve their slots and run S9 in place), and a
frame holds far more than the lanes' initial lists (4096 on the device, 1024 in the pinned
read-back), which grow on demand -- the device list by running K3 again on the batch.  The
device list must still be the oracle's, cell for cell and in find() order (complex double),
with S9 estimates to the parity tolerance on a sample, and the throughput queue (batched frames,
read back by k_dets_to_host) must give the synchronous path's results.
"""
import numpy as np
import pytest

from oracle import chain
from rsp.plan import Plan

from _scen import scenario, targets_for, noisy_cube

pytestmark = pytest.mark.gpu

T_LOW = 0.3


def _tile_max(keys, rc0, rt):
    """Most hits in one K3 tile (pair, range tile): tiles start at (rc0 & ~3) + k rt."""
    cnt = {}
    for v, r, p in keys:
        t = (p, (r - 1 - (rc0 & ~3)) // rt)
        cnt[t] = cnt.get(t, 0) + 1
    return max(cnt.values())


def test_dense_hits_match_oracle_and_queue():
    s = scenario('small')
    cube = noisy_cube(s, targets_for('small'), dtype=np.complex128)
    cfar = dict(s['cfar'], T_CFAR=T_LOW)
    pre = s['pre_o']
    rdm = chain.mtd(chain.pulse_compress(chain.dbf(cube, pre['DBF_coeffs_data_C']), pre), pre)
    dets, S_all = chain.goca_cfar(rdm, cfar)
    want = [(int(d[0]), int(d[1]), int(d[2])) for d in dets]
    rc0 = cfar['refCells_R'] + cfar['guardCells_R']
    assert len(want) > 20000
    assert _tile_max(want, rc0, 32) > 1024, 'no K3 tile past its LDS queue'

    plan = Plan(s['cfg'], cfar, s['clus'], s['pre_p'], frames_per_launch=2)
    try:
        gpu = plan.process_cube(cube, frame_idx=1)
        got = gpu['detections']
        assert [(d['v_idx'], d['r_idx'], d['pair_idx']) for d in got] == want
        amp = np.array([d['amp'] for d in got])
        # the map tolerance of test_gpu_parity (1e-12 of the maximum): most of these are noise cells
        np.testing.assert_allclose(amp, dets[:, 3], rtol=0, atol=1e-12 * np.abs(dets[:, 3]).max())
        rng = np.random.default_rng(7)
        idx = np.sort(rng.choice(len(want), 300, replace=False))
        est = chain.parameter_estimation(dets[idx], S_all, rdm, pre)
        for i, e in zip(idx, est):
            for f in ('Range', 'Velocity', 'Angle'):
                assert got[i][f] == pytest.approx(e[f], abs=1e-9), (i, f)
        sync_targets = gpu['final_targets']
        assert len(sync_targets) > 0

        # the same frame through the queue: batches of 2, lists read back by k_dets_to_host
        d = plan.device_alloc(plan.cube_bytes)
        try:
            plan.upload_cube(d, cube)
            plan.enqueue_many([d] * 6, range(10, 16))
            plan.drain()
            res = plan.results()
        finally:
            plan.device_free(d)
        assert [r['frame_idx'] for r in res] == list(range(10, 16))
        for r in res:
            assert r['n_dets'] == len(want)
            assert r['final_targets'] == sync_targets
    finally:
        plan.close()


def test_dense_hits_complex_single_queue_equals_sync():
    """Complex single (64-cell halo-less tiles): the queue's lists equal the synchronous path's,
    and the detection count is the oracle's up to near-threshold flips."""
    s = scenario('x2')
    cube = noisy_cube(s, targets_for('x2'), dtype=np.complex64)
    cfar = dict(s['cfar'], T_CFAR=1.5)
    plan = Plan(s['cfg'], cfar, s['clus'], s['pre_p'], frames_per_launch=4, precision='c64')
    try:
        sync = plan.process_cube(cube, frame_idx=1)
        n = len(sync['detections'])
        assert n > 5000
        d = plan.device_alloc(plan.cube_bytes)
        try:
            plan.upload_cube(d, cube)
            plan.enqueue_many([d] * 8, range(8))
            plan.drain()
            res = plan.results()
        finally:
            plan.device_free(d)
        for r in res:
            assert r['n_dets'] == n
            assert r['final_targets'] == sync['final_targets']
    finally:
        plan.close()


def test_between_readback_and_device_capacity():
    """A frame with more detections than the pinned read-back holds (1024) but fewer than the
    device list (4096): harvest takes the first 1024 from the read-back and the rest by a direct
    copy, without regrowing the device list.  On a fresh plan the queue must give the synchronous
    path's lists (counts and final targets) for every frame."""
    s = scenario('small')
    cube = noisy_cube(s, targets_for('small'), dtype=np.complex128)
    cfar = dict(s['cfar'], T_CFAR=2.0)
    qplan = Plan(s['cfg'], cfar, s['clus'], s['pre_p'], frames_per_launch=2)   # fresh: initial capacities
    splan = Plan(s['cfg'], cfar, s['clus'], s['pre_p'])
    try:
        d = qplan.device_alloc(qplan.cube_bytes)
        try:
            qplan.upload_cube(d, cube)
            qplan.enqueue_many([d] * 4, range(20, 24))
            qplan.drain()
            res = qplan.results()
        finally:
            qplan.device_free(d)
        sync = splan.process_cube(cube, frame_idx=1)
        n = len(sync['detections'])
        assert 1024 < n <= 4096, n
        for r in res:
            assert r['n_dets'] == n
            assert r['final_targets'] == sync['final_targets']
    finally:
        qplan.close()
        splan.close()
