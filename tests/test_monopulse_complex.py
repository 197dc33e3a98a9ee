"""S9 with the complex monopulse ratio (RSP_PLAN_MONOPULSE_COMPLEX, Plan(monopulse='complex')).

fun_process_single_frame's S9 takes the angle from the amplitude ratio (|S_A| - |S_B|) /
(|S_A| + |S_B| + eps) (fsf:280-290).  The Monte-Carlo script main_plot_snr_vs_angle_error.m keeps
an inline copy of S9 that uses the complex ratio real((S_A - S_B) / (S_A + S_B + eps)) of the
complex RD map instead (:455-462, "v7.6 uses the complex ratio").  With the plan option the device
runs that estimator: K2 writes every frame's complex map (the caller's, or plan-owned) and K3's S9
reads S_A, S_B from it.

Checked against oracle.chain.process_cube(..., monopulse='complex') on the same cubes: the
detection list is the amplitude run's (the CFAR does not depend on the estimator), every
detection's Range / Velocity equal the amplitude run's and its Angle the oracle's complex-ratio
angle (complex double: 1e-9); the final targets likewise; the throughput queue equals the
synchronous path.  The script's own SNR sweep with this estimator is in tests/test_montecarlo.py.
"""
import numpy as np
import pytest

from oracle import chain
from rsp.plan import Plan

from _scen import scenario, targets_for, noisy_cube, device_cube

pytestmark = pytest.mark.gpu


def _frame(name):
    s = scenario(name)
    tg = targets_for(name)
    if name == 'reference':
        p = Plan(s['cfg'], s['cfar'], s['clus'], s['pre_p'])
        cube = device_cube(p, tg, frame_idx=1)
        p.close()
    else:
        cube = noisy_cube(s, tg, dtype=np.complex128)
    return s, cube


@pytest.mark.parametrize('name', ['small', 'x2', 'reference'])
def test_complex_ratio_matches_oracle(name):
    s, cube = _frame(name)
    fin_o, st = chain.process_cube(cube, s['cfg'], s['cfar'], s['clus'], s['pre_o'], keep=True, monopulse='complex')
    pa = Plan(s['cfg'], s['cfar'], s['clus'], s['pre_p'])
    pc = Plan(s['cfg'], s['cfar'], s['clus'], s['pre_p'], monopulse='complex')
    try:
        amp = pa.process_cube(cube, frame_idx=1)
        cpx = pc.process_cube(cube, frame_idx=1)
    finally:
        pa.close()
        pc.close()
    keys = [(d['v_idx'], d['r_idx'], d['pair_idx']) for d in cpx['detections']]
    assert keys == [(d['v_idx'], d['r_idx'], d['pair_idx']) for d in amp['detections']]
    assert keys == [(int(v), int(r), int(p)) for v, r, p, _ in st['dets']]
    moved = 0
    for d, da, e in zip(cpx['detections'], amp['detections'], st['par']):
        assert d['Range'] == da['Range'] and d['Velocity'] == da['Velocity']
        assert d['Angle'] == pytest.approx(e['Angle'], abs=1e-9)
        moved += d['Angle'] != da['Angle']
    assert moved > 0, 'the complex ratio changed no angle'
    assert len(cpx['final_targets']) == len(fin_o)
    for a, b in zip(cpx['final_targets'], fin_o):
        for f in ('Range', 'Velocity', 'Angle', 'Power'):
            assert a[f] == pytest.approx(b[f], rel=1e-9, abs=1e-9), f


def test_complex_ratio_queue_equals_sync():
    """The throughput queue (no caller maps: the plan's own per-lane maps) == the synchronous path."""
    s, cube = _frame('x2')
    ps = Plan(s['cfg'], s['cfar'], s['clus'], s['pre_p'], monopulse='complex')
    pq = Plan(s['cfg'], s['cfar'], s['clus'], s['pre_p'], frames_per_launch=4, monopulse='complex')
    try:
        want = ps.process_cube(cube, frame_idx=1)['final_targets']
        d = pq.device_alloc(pq.cube_bytes)
        pq.upload_cube(d, cube)
        pq.enqueue_many([d] * 6, list(range(1, 7)))
        pq.drain()
        res = pq.results()
        pq.device_free(d)
    finally:
        ps.close()
        pq.close()
    assert len(res) == 6
    for r in res:
        tg = r['final_targets']
        assert len(tg) == len(want), r['frame_idx']
        for a, b in zip(tg, want):
            for f in ('Range', 'Velocity', 'Angle', 'Power'):
                assert a[f] == b[f], (r['frame_idx'], f)


def test_complex_ratio_c64():
    """Complex single: the complex-ratio angle of every detection the oracle also has (same
    complex64-rounded cube) within the c64 tolerance of tests/test_gpu_parity.py (1e-3 deg)."""
    s, cube = _frame('x2')
    cube = cube.astype(np.complex64)
    _, st = chain.process_cube(cube.astype(np.complex128), s['cfg'], s['cfar'], s['clus'], s['pre_o'], keep=True,
                               monopulse='complex')
    p = Plan(s['cfg'], s['cfar'], s['clus'], s['pre_p'], precision='c64', monopulse='complex')
    try:
        got = p.process_cube(cube, frame_idx=1)['detections']
    finally:
        p.close()
    want = {(int(d[0]), int(d[1]), int(d[2])): e for d, e in zip(st['dets'], st['par'])}
    n = 0
    for d in got:
        e = want.get((d['v_idx'], d['r_idx'], d['pair_idx']))
        if e is None:
            continue
        n += 1
        assert d['Angle'] == pytest.approx(e['Angle'], abs=1e-3)
    assert n > 0.95 * len(want)
