"""Golden fixtures (tests/golden/, made by tests/golden/make_golden.py).

CPU: the oracle still reproduces every stored vector (so the checker cannot drift).
GPU: the device path -- S4 synthesis + Philox noise on the device, then S5..S11 through
the C-ABI (rsp_process_targets), complex double -- matches the stored vectors with the
complex-double tolerances of tests/test_gpu_parity.py: cube probes to 1e-10 relative,
RDM probes to 1e-12 * max|RDM|, the identical detection list (v, r, pair in order, S to
1e-12 relative), final targets to 1e-9.
"""
import glob
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
FILES = sorted(glob.glob(os.path.join(HERE, 'golden', 'golden_*.npz')))


def _load(fn):
    z = np.load(fn, allow_pickle=False)
    return {k: z[k] for k in z.files}


def _targets(g):
    return [dict(Range=r, Velocity=v, ElevationAngle=a, SNR_dB=s) for r, v, a, s in g['targets']]


def test_fixtures_present():
    assert len(FILES) >= 4


@pytest.mark.parametrize('fn', FILES, ids=[os.path.basename(f) for f in FILES])
def test_oracle_reproduces_golden(fn):
    from oracle import chain
    from _scen import scenario
    g = _load(fn)
    s = scenario(str(g['name']))
    tg = _targets(g)
    f = int(g['frame_idx'])
    cube = chain.synthesize_echo(tg, s['cfg'], s['pre_o']) + chain.philox_noise(s['cfg'], f, int(g['seed']))
    np.testing.assert_allclose(cube.ravel(order='F')[g['cube_idx']], g['cube_val'], rtol=1e-12, atol=1e-12)
    fin, st = chain.process_cube(cube, s['cfg'], s['cfar'], s['clus'], s['pre_o'], keep=True)
    np.testing.assert_allclose(st['rdm'].ravel(order='F')[g['rdm_idx']], g['rdm_val'], rtol=1e-9,
                               atol=1e-9 * float(g['rdm_absmax']))
    dets = np.asarray(st['dets'], float).reshape(-1, 4)
    assert np.array_equal(dets[:, :3], g['dets'][:, :3])
    np.testing.assert_allclose(dets[:, 3], g['dets'][:, 3], rtol=1e-9)
    fin_a = np.asarray([[t['Range'], t['Velocity'], t['Angle'], t['Power']] for t in fin]).reshape(-1, 4)
    np.testing.assert_allclose(fin_a, g['final'], rtol=1e-9, atol=1e-9)


@pytest.mark.gpu
@pytest.mark.parametrize('fn', FILES, ids=[os.path.basename(f) for f in FILES])
def test_device_matches_golden(fn):
    from rsp.plan import Plan
    from _scen import scenario
    g = _load(fn)
    s = scenario(str(g['name']))
    tg = _targets(g)
    f, seed = int(g['frame_idx']), int(g['seed'])
    plan = Plan(s['cfg'], s['cfar'], s['clus'], s['pre_p'])
    try:
        d = plan.device_alloc(plan.cube_bytes)
        plan.synthesize_device(d, tg, f, seed=seed)
        plan.sync()
        cube = plan.device_download(d, plan.sizes.cube_elems, plan.cdtype)
        plan.device_free(d)
        scale = np.abs(g['cube_val']).max()
        assert np.abs(cube[g['cube_idx']] - g['cube_val']).max() <= 1e-10 * scale

        out = plan.process_targets(tg, frame_idx=f, seed=seed, want_rdm=True)
    finally:
        plan.close()
    rdm = out['rdm'].ravel(order='F')[g['rdm_idx']]
    assert np.abs(rdm - g['rdm_val']).max() <= 1e-12 * float(g['rdm_absmax'])
    got = np.asarray([[x['v_idx'], x['r_idx'], x['pair_idx'], x['amp']] for x in out['detections']],
                     float).reshape(-1, 4)
    assert np.array_equal(got[:, :3], g['dets'][:, :3])
    np.testing.assert_allclose(got[:, 3], g['dets'][:, 3], rtol=1e-12)
    fin = np.asarray([[t['Range'], t['Velocity'], t['Angle'], t['Power']] for t in out['final_targets']],
                     float).reshape(-1, 4)
    np.testing.assert_allclose(fin, g['final'], rtol=1e-9, atol=1e-9)
