"""GPU tests of the end-to-end queue (rsp_enqueue_host) and the in-process multi-plan driver
(rsp_process_targets_multi, BASELINE config #3 for a MEX host).

Both are checked against paths the parity suite already pins to the oracle: the device-resident
queue (rsp_enqueue_device) and the synchronous rsp_process_targets.  Same cubes through the same
kernels, so the final targets must be identical, not just close.
"""
import numpy as np
import pytest

from _scen import scenario, targets_for
from rsp import config as C
from rsp.plan import Plan, process_targets_multi

pytestmark = pytest.mark.gpu


def _same(a, b):
    assert [r['frame_idx'] for r in a] == [r['frame_idx'] for r in b]
    for ra, rb in zip(a, b):
        assert ra['final_targets'] == rb['final_targets'], ra['frame_idx']


@pytest.mark.parametrize('prec', ['c128', 'c64'])
def test_enqueue_host_equals_device_queue(prec):
    """x2 frames (several used-sample intervals) uploaded from pinned host cubes through the plan's
    ring, which wraps (F = 2: 8 slots for 20 frames), give the device queue's results."""
    s = scenario('x2')
    tg = targets_for('x2')
    plan = Plan(s['cfg'], s['cfar'], s['clus'], s['pre_p'], frames_per_launch=2, precision=prec)
    nb = plan.cube_bytes
    dev = [plan.device_alloc(nb) for _ in range(3)]
    host = [plan.host_alloc(nb) for _ in range(3)]
    try:
        t = tg
        for i in range(3):
            plan.synthesize_device(dev[i], t, frame_idx=i + 1)
            t = C.evolve_targets(t, s['cfg'])
            plan.host_cube(host[i])[...] = plan.device_download(dev[i], nb // np.dtype(plan.cdtype).itemsize,
                                                                plan.cdtype).reshape(plan.host_cube(host[i]).shape,
                                                                                     order='F')
        plan.sync()
        for k in range(20):
            plan.enqueue(dev[k % 3], 100 + k)
        plan.drain()
        ref = plan.results()
        for k in range(20):
            plan.enqueue_host(host[k % 3], 100 + k)
        plan.drain()
        got = plan.results()
        assert sum(len(r['final_targets']) for r in ref) > 0
        _same(got, ref)
        with pytest.raises(Exception):   # no converting uploads on the queue
            other = np.zeros((plan.P, plan.N, plan.sizes.C), np.complex64 if prec == 'c128' else np.complex128,
                             order='F')
            plan.enqueue_host(other, 1)
    finally:
        for p in dev:
            plan.device_free(p)
        for p in host:
            plan.host_free(p)
        plan.close()


def test_process_targets_multi_equals_per_frame_calls():
    """Two plans (on the one GPU of the box: two host threads, two queues) share 7 frames;
    every frame's final targets equal the synchronous fsf:13 path's."""
    s = scenario('small')
    t = targets_for('small')
    frames = []
    for f in range(7):
        frames.append((t, 10 + f))
        t = C.evolve_targets(t, s['cfg'])
    plans = [Plan(s['cfg'], s['cfar'], s['clus'], s['pre_p'], frames_per_launch=2) for _ in range(2)]
    try:
        got = process_targets_multi(plans, frames)
        ref = [plans[0].process_targets(tt, frame_idx=fi)['final_targets'] for tt, fi in frames]
        assert any(len(r) for r in ref)
        assert got == ref
        with pytest.raises(Exception):   # one host thread per plan
            process_targets_multi([plans[0], plans[0]], frames)
    finally:
        for p in plans:
            p.close()


def test_results_rows_equal_results():
    """rsp_results_rows packs what rsp_results_get returns: frame by frame, one NaN row for a
    frame without targets (the payload rsp.dist.gather_rows moves)."""
    s = scenario('small')
    t = targets_for('small')
    plan = Plan(s['cfg'], s['cfar'], s['clus'], s['pre_p'], frames_per_launch=2)
    d = plan.device_alloc(plan.cube_bytes)
    e = plan.device_alloc(plan.cube_bytes)
    try:
        plan.synthesize_device(d, t, frame_idx=1)
        plan.synthesize_device(e, [], frame_idx=2)   # noise only: no targets
        plan.enqueue_many([d if k % 2 == 0 else e for k in range(5)], range(10, 15))   # rsp_enqueue_device_n
        plan.drain()
        rows = plan.results_rows(clear=False)
        res = plan.results(clear=True)
        want = []
        for r in res:
            for x in r['final_targets']:
                want.append((r['frame_idx'], x['Range'], x['Velocity'], x['Angle'], x['Power']))
            if not r['final_targets']:
                want.append((r['frame_idx'],) + (np.nan,) * 4)
        np.testing.assert_array_equal(rows, np.asarray(want, np.float64).reshape(-1, 5))
        assert len(plan.results_rows()) == 0
    finally:
        plan.device_free(d)
        plan.device_free(e)
        plan.close()


@pytest.mark.parametrize('prec', ['c128', 'c64'])
def test_queue_rdm_equals_sync_rdm(prec):
    """rsp_enqueue_device_rdm: the queue writes each requested frame's complex RD map (rdm_13beam,
    fsf:131-136) into the caller's device buffer.  It must equal the synchronous rsp_process_cube
    map of the same cube exactly, frames that request no map must leave their buffers untouched,
    and the final targets must be the queue's without maps."""
    s = scenario('x2')
    t = targets_for('x2')
    plan = Plan(s['cfg'], s['cfar'], s['clus'], s['pre_p'], frames_per_launch=2, precision=prec)
    sz = plan.sizes
    esz = np.dtype(plan.cdtype).itemsize
    cubes = [plan.device_alloc(plan.cube_bytes) for _ in range(2)]
    maps = [plan.device_alloc(sz.rdm_elems * esz) for _ in range(3)]
    try:
        for i, c in enumerate(cubes):
            plan.synthesize_device(c, t, frame_idx=i + 1)
            t = C.evolve_targets(t, s['cfg'])
        sentinel = np.full(sz.rdm_elems, 7.0 + 3.0j, plan.cdtype)
        plan.device_upload(maps[2], sentinel)
        plan.sync()
        seq = [0, 1, 0, 1, 0]
        plan.enqueue_many([cubes[k] for k in seq], range(30, 35))
        plan.drain()
        ref = plan.results()
        # frames 30 and 31 with maps, then three without (map 2 must stay the sentinel)
        plan.enqueue_many([cubes[0], cubes[1]], [30, 31], rdms=[maps[0], maps[1]])
        plan.enqueue_many([cubes[k] for k in seq[2:]], range(32, 35))
        plan.drain()
        got = plan.results()
        _same(got, ref)
        for k in range(2):
            host = plan.device_download(cubes[k], plan.cube_bytes // esz, plan.cdtype)
            host = host.reshape(plan.P, plan.N, sz.C, order='F')
            want = plan.process_cube(host, frame_idx=30 + k, want_rdm=True)['rdm']
            q = plan.rdm_from_device(maps[k])
            assert q.shape == want.shape
            np.testing.assert_array_equal(q.astype(np.complex128), want)
        np.testing.assert_array_equal(plan.device_download(maps[2], sz.rdm_elems, plan.cdtype), sentinel)
    finally:
        for p in cubes + maps:
            plan.device_free(p)
        plan.close()
