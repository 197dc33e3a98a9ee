"""GPU parity: librsp (HIP, gfx950) vs the CPU oracle on identical inputs.

Configurations: small (P=64), x2 (BASELINE #2, P=128), p256 (P=256), x4 (BASELINE #4:
32C x 16B x 8192N x 256P, two MFMA row blocks, 5-block long segment, 32-cell K3 tiles) and
reference (the v8 frame 16C x 13B x 5819N x 332P: the factored 4 x 83 slow-time DFT K1, B=13
in BMAX=16), each
through the complex-double plan (the default, MATLAB's arithmetic) and through the
complex-single plan (the reference frame's device-synthesised cube rounded to complex64).

Tolerances, complex double (c128) vs the complex128 oracle:
  * RDM / CFAR maps: max |delta| <= 1e-12 * max |oracle| (the device CFAR map is the one K3
    thresholds, fsf:184-187).
  * CFAR detections: the identical (v, r, pair) set, in the identical fsf find() order.
  * S9 of every detection: amp rel 1e-12, Range / Velocity / Angle abs 1e-9.
  * final targets: identical count, every field rel/abs 1e-9.
Complex single (c64) vs the oracle on the same (complex64-rounded) cube:
  * maps: max |delta| <= 2e-5 * max |oracle| and relative L2 <= 1e-5.
  * CFAR decisions identical except cells whose oracle margin |S - T*noise| / (T*noise) is
    below 1e-4 (a fp32 rounding can legitimately flip those).
  * S9 estimates of matched detections: amp rel 1e-4, Angle 1e-3 deg; Range / Velocity
    equal to 1e-6 unless the spline argmax moved by one sample (<= deltaR/8, deltaV/4),
    which is allowed for at most 2% of detections.
  * final targets: against the oracle when the raw sets agree, else against the oracle's
    clustering (S10/S11) of the device's own detections.
"""
import numpy as np
import pytest

from oracle import chain
from rsp.plan import Plan

from _scen import scenario, targets_for, noisy_cube, device_cube, SEED

pytestmark = pytest.mark.gpu

MAP_TOL = {'c128': 1e-12, 'c64': 2e-5}
MARGIN = 1e-4
LARGE = ('x4', 'reference')   # inputs synthesised on the device (numpy synthesis takes ~30 s)
CASES = [('small', 'c128'), ('small', 'c64'), ('x2', 'c128'), ('x2', 'c64'), ('p256', 'c128'), ('p256', 'c64'),
         ('x4', 'c128'), ('x4', 'c64'), ('reference', 'c128'), ('reference', 'c64')]

_cube_cache = {}


def _input_cube(name, s, tg):
    """The noisy complex128 cube of frame 1 (cached per config; one config at a time)."""
    if name not in _cube_cache:
        _cube_cache.clear()
        if name in LARGE:
            p = Plan(s['cfg'], s['cfar'], s['clus'], s['pre_p'])
            _cube_cache[name] = device_cube(p, tg, frame_idx=1)
            p.close()
        else:
            _cube_cache[name] = noisy_cube(s, tg, dtype=np.complex128)
    return _cube_cache[name]


@pytest.fixture(scope='module', params=CASES, ids=['%s-%s' % c for c in CASES])
def case(request):
    name, prec = request.param
    s = scenario(name)
    tg = targets_for(name)
    cube = _input_cube(name, s, tg)
    if prec == 'c64':
        cube = cube.astype(np.complex64)
    fin, st = chain.process_cube(cube.astype(np.complex128), s['cfg'], s['cfar'], s['clus'], s['pre_o'], keep=True)
    st = {k: st[k] for k in ('rdm', 'S_all', 'dets', 'par')}
    plan = Plan(s['cfg'], s['cfar'], s['clus'], s['pre_p'], precision=prec)
    gpu = plan.process_cube(cube, frame_idx=1, want_rdm=True, want_cfar=True)
    # the same frame with the complex map kept on chip (K2's magnitude-only store path, as the
    # throughput queue runs it)
    gpu_mag = plan.process_cube(cube, frame_idx=1, want_rdm=False, want_cfar=True)
    plan.close()
    yield dict(name=name, prec=prec, s=s, tg=tg, fin=fin, st=st, gpu=gpu, gpu_mag=gpu_mag)


def _map_close(a, b, tol):
    scale = np.abs(b).max()
    err = np.abs(a - b).max()
    assert err <= tol * scale, 'max err %.3g vs scale %.3g (tol %g)' % (err, scale, tol)
    if tol > 1e-9:
        rl2 = np.linalg.norm((a - b).ravel()) / np.linalg.norm(b.ravel())
        assert rl2 <= 1e-5, 'rel L2 %.3g' % rl2


def test_rdm_parity(case):
    _map_close(case['gpu']['rdm'], case['st']['rdm'], MAP_TOL[case['prec']])


def test_cfar_map_parity(case):
    """rdm_for_cfar_all as produced on the device (K3's S tile), not recomputed on the host."""
    _map_close(case['gpu']['cfar_maps'], case['st']['S_all'], MAP_TOL[case['prec']])


def test_cfar_map_without_rdm(case):
    """K2 without the complex RD map stores the same magnitudes: the CFAR maps and the detection
    list are bit-identical to the run that also writes the RDM."""
    a, b = case['gpu_mag'], case['gpu']
    assert np.array_equal(a['cfar_maps'], b['cfar_maps']), 'max diff %g' % np.abs(a['cfar_maps'] - b['cfar_maps']).max()
    assert [(d['v_idx'], d['r_idx'], d['pair_idx']) for d in a['detections']] == \
        [(d['v_idx'], d['r_idx'], d['pair_idx']) for d in b['detections']]


def _keys(dets):
    return [(int(d[0]), int(d[1]), int(d[2])) for d in dets]


def test_detection_sets(case):
    o = set(_keys(case['st']['dets']))
    g = {(d['v_idx'], d['r_idx'], d['pair_idx']) for d in case['gpu']['detections']}
    assert len(o) > 0
    if case['prec'] == 'c128':
        assert o == g, 'CFAR decisions differ: oracle-only %r, device-only %r' % (sorted(o - g)[:8], sorted(g - o)[:8])
        return
    mg = chain.cfar_margin(case['st']['rdm'], case['s']['cfar'])
    for (v, r, p) in o ^ g:
        assert mg[v - 1, r - 1, p - 1] < MARGIN, 'CFAR decision differs at (v=%d r=%d pair=%d)' % (v, r, p)


def test_detection_order_and_estimates(case):
    pre = case['s']['pre_o']
    od = {k: (d, e) for k, d, e in zip(_keys(case['st']['dets']), case['st']['dets'], case['st']['par'])}
    gd = case['gpu']['detections']
    keys = [(d['v_idx'], d['r_idx'], d['pair_idx']) for d in gd]
    assert keys == sorted(keys, key=lambda k: (k[2], k[1], k[0])), 'not in fsf find() order'
    if case['prec'] == 'c128':
        assert keys == _keys(case['st']['dets'])
        for d in gd:
            raw, est = od[(d['v_idx'], d['r_idx'], d['pair_idx'])]
            assert d['amp'] == pytest.approx(raw[3], rel=1e-12)
            for f in ('Range', 'Velocity', 'Angle'):
                assert d[f] == pytest.approx(est[f], abs=1e-9), f
        return
    moved = 0
    n = 0
    for d in gd:
        k = (d['v_idx'], d['r_idx'], d['pair_idx'])
        if k not in od:
            continue
        n += 1
        raw, est = od[k]
        assert d['amp'] == pytest.approx(raw[3], rel=1e-4)
        assert d['Angle'] == pytest.approx(est['Angle'], abs=1e-3)
        dr, dv = abs(d['Range'] - est['Range']), abs(d['Velocity'] - est['Velocity'])
        if dr > 1e-6 * max(1.0, abs(est['Range'])) or dv > 1e-6:
            assert dr <= pre['deltaR'] / 8 + 1e-6 and dv <= pre['deltaV'] / 4 + 1e-9
            moved += 1
    assert n > 0
    assert moved <= max(1, 0.02 * n)


def test_final_targets(case):
    fg = case['gpu']['final_targets']
    if case['prec'] == 'c128':
        fo = case['fin']
        assert len(fo) == len(fg)
        for a, b in zip(fo, fg):
            for f in ('Range', 'Velocity', 'Angle', 'Power'):
                assert b[f] == pytest.approx(a[f], rel=1e-9, abs=1e-9), f
        return
    o = set(_keys(case['st']['dets']))
    g = {(d['v_idx'], d['r_idx'], d['pair_idx']) for d in case['gpu']['detections']}
    pre = case['s']['pre_o']
    if o == g:
        fo = case['fin']
        tol = dict(Range=pre['deltaR'] / 8, Velocity=pre['deltaV'] / 4, Angle=2e-3)
    else:   # near-threshold cells flipped: the clustering of the device's own detections
        par = [dict(Range=d['Range'], Velocity=d['Velocity'], Angle=d['Angle'], Power=d['amp'])
               for d in case['gpu']['detections']]
        fo = chain.cluster_stage2(chain.cluster_stage1(par, case['s']['clus']), case['s']['clus'])
        tol = dict(Range=1e-9, Velocity=1e-9, Angle=1e-9)
    assert len(fo) == len(fg)
    for a, b in zip(fo, fg):
        for f, t in tol.items():
            assert b[f] == pytest.approx(a[f], abs=t), f
        assert b['Power'] == pytest.approx(a['Power'], rel=1e-4)


def test_targets_found(case):
    """Every simulated target is reported by the GPU chain near its true range."""
    fg = case['gpu']['final_targets']
    for t in case['tg']:
        if t['SNR_dB'] < -15:
            continue
        assert any(abs(f['Range'] - t['Range']) < 15 for f in fg), 'target at %g m missed' % t['Range']


def test_process_stage2_mtd_dropin_reference_gated():
    """process_stage2_mtd(iq_data, angle, config) -- the literal 3-argument call of
    debug_simulated_data_processing_v3.m:189 -- on the reference frame's DBF output gated like
    the v2 .mat frames ([332 x 3404 x 13], main_simulate_echoes_with_array_v2.m:256-267): the
    [332 x 3404 x 13] MTD and PC results (process_stage2_mtd.m:29-30) equal the oracle's S6 + S7
    of the same columns put back at their PRT positions, to 1e-12 of the map maximum."""
    import rsp
    s = scenario('reference')
    tg = targets_for('reference')
    iq = chain.dbf(_input_cube('reference', s, tg), s['pre_o']['DBF_coeffs_data_C'])
    cols = rsp.REFERENCE_GATE_COLS
    gated = np.concatenate([iq[:, a - 1:b, :] for a, b in cols], axis=1)
    assert gated.shape == (332, 3404, 13)
    mtd, pc = rsp.process_stage2_mtd(gated, np.zeros(332), s['cfg'])
    assert mtd.shape == pc.shape == (332, 3404, 13)
    full = np.zeros_like(iq)
    for a, b in cols:
        full[:, a - 1:b, :] = iq[:, a - 1:b, :]
    pc_o = chain.pulse_compress(full, s['pre_o'])
    _map_close(pc, pc_o, MAP_TOL['c128'])
    _map_close(mtd, chain.mtd(pc_o, s['pre_o']), MAP_TOL['c128'])
    # the caller's own config (debug_simulated_data_processing_v3.m:55-106: point_PRT = 3404 gated
    # samples, point_prt = [3404 228 723 2453], no gap_duration / Array, config.mtd.beam_num)
    # describes the same waveform and gating: identical results
    mtd3, pc3 = rsp.process_stage2_mtd(gated, np.zeros(332), rsp.debug_v3_config())
    np.testing.assert_array_equal(mtd3, mtd)
    np.testing.assert_array_equal(pc3, pc)
    # gate columns must be ascending and disjoint (v2:257-264)
    with pytest.raises(rsp.RspError):
        rsp.process_stage2_mtd(gated, np.zeros(332), s['cfg'], gate_cols=((83, 310), (300, 1022), (1023, 3475)))


@pytest.mark.parametrize('prec', ['c128', 'c64'])
def test_synthesis_path_matches_oracle_cube(prec):
    s = scenario('small')
    tg = targets_for('small')
    plan = Plan(s['cfg'], s['cfar'], s['clus'], s['pre_p'], precision=prec)
    try:
        dev = device_cube(plan, tg, frame_idx=3)
    finally:
        plan.close()
    ref = noisy_cube(s, tg, frame_idx=3, dtype=np.complex128)
    assert np.abs(dev - ref).max() <= (1e-10 if prec == 'c128' else 1e-5) * np.abs(ref).max()


@pytest.mark.gpu
def test_synthesis_with_the_target_cap_matches_oracle_cube():
    """The most targets one synthesis takes (64: they travel in the kernel arguments, 2 KiB) --
    spread over range, velocity and angle, some outside the fast-time window -- against the oracle
    cube; one more is refused before anything runs."""
    s = scenario('small')
    sc = s['cfg']['Sig_Config']
    rng = np.random.default_rng(64)
    rmax = sc['c'] * sc['point_PRT'] / sc['fs'] / 2 * 1.1   # a few delays past the window
    tg = [dict(Range=float(rng.uniform(50.0, rmax)), Velocity=float(rng.uniform(-30.0, 30.0)),
               ElevationAngle=float(rng.uniform(-40.0, 40.0)), SNR_dB=float(rng.uniform(-20.0, 20.0)))
          for _ in range(64)]
    import rsp
    plan = Plan(s['cfg'], s['cfar'], s['clus'], s['pre_p'])
    try:
        dev = device_cube(plan, tg, frame_idx=5)
        ptr = plan.device_alloc(plan.cube_bytes)
        try:
            with pytest.raises(rsp.RspError):
                plan.synthesize_device(ptr, tg + tg[:1], frame_idx=5)
        finally:
            plan.device_free(ptr)
    finally:
        plan.close()
    ref = noisy_cube(s, tg, frame_idx=5, dtype=np.complex128)
    assert np.abs(dev - ref).max() <= 1e-10 * np.abs(ref).max()


def test_process_targets_equals_cube_path():
    s = scenario('small')
    tg = targets_for('small')
    plan = Plan(s['cfg'], s['cfar'], s['clus'], s['pre_p'])
    a = plan.process_targets(tg, frame_idx=2, seed=SEED)
    b = plan.process_cube(noisy_cube(s, tg, frame_idx=2, dtype=np.complex128), frame_idx=2)
    plan.close()
    ka = [(d['v_idx'], d['r_idx'], d['pair_idx']) for d in a['detections']]
    kb = [(d['v_idx'], d['r_idx'], d['pair_idx']) for d in b['detections']]
    assert ka == kb
    assert len(a['final_targets']) == len(b['final_targets'])


@pytest.mark.parametrize('prec', ['c128', 'c64'])
def test_queue_matches_sync_path(prec):
    s = scenario('small')
    tg = targets_for('small')
    plan = Plan(s['cfg'], s['cfar'], s['clus'], s['pre_p'], frames_per_launch=3, precision=prec)
    ptrs = [plan.device_alloc(plan.cube_bytes) for _ in range(4)]
    try:
        for f, p in enumerate(ptrs):
            plan.synthesize_device(p, tg, frame_idx=f + 1)
        for rep in range(2):
            for f, p in enumerate(ptrs):
                plan.enqueue(p, f + 1 + 10 * rep)
        plan.drain()
        res = plan.results()
        assert [r['frame_idx'] for r in res] == [1, 2, 3, 4, 11, 12, 13, 14]
        for f in range(4):
            sync = plan.process_targets(tg, frame_idx=f + 1)
            for r in (res[f], res[f + 4]):
                assert len(r['final_targets']) == len(sync['final_targets'])
                for a, b in zip(r['final_targets'], sync['final_targets']):
                    assert a == b
    finally:
        for p in ptrs:
            plan.device_free(p)
        plan.close()


@pytest.mark.parametrize('prec', ['c128', 'c64'])
def test_stage2_parity(prec):
    s = scenario('small')
    tg = targets_for('small')
    cube = noisy_cube(s, tg, dtype=np.complex128)
    iq = chain.dbf(cube, s['pre_o']['DBF_coeffs_data_C'])
    if prec == 'c64':
        iq = iq.astype(np.complex64).astype(np.complex128)
    pc_o = chain.pulse_compress(iq, s['pre_o'])
    mtd_o = chain.mtd(pc_o, s['pre_o'])
    plan = Plan(s['cfg'], s['cfar'], s['clus'], s['pre_p'], precision=prec)
    mtd, pc = plan.process_stage2(iq)
    plan.close()
    _map_close(pc, pc_o, MAP_TOL[prec])
    _map_close(mtd, mtd_o, MAP_TOL[prec])


def test_profile_stages_reports_three_kernels():
    s = scenario('small')
    plan = Plan(s['cfg'], s['cfar'], s['clus'], s['pre_p'])
    ptr = plan.device_alloc(plan.cube_bytes)
    plan.synthesize_device(ptr, targets_for('small'), 1)
    st = plan.profile_stages([ptr], iters=3)
    plan.device_free(ptr)
    plan.close()
    assert [x['stage'] for x in st] == ['k1_dbf_mtd', 'k2_pc', 'k3_cfar']
    assert all(x['ms'] > 0 and x['bytes'] > 0 for x in st)
    # K3's stage bytes = the rows under test of every beam's magnitude map (k3_map_bytes), the
    # formula tests/test_bench_args.py checks against the PMC-measured traffic
    import bench
    sc = s['cfg']['Sig_Config']
    G = sum(sc['point_prt_segments'])
    assert st[2]['bytes'] == st[2]['frames'] * bench.k3_map_bytes(sc['prtNum'], G, sc['beam_num'], s['cfar'], 8)


@pytest.mark.parametrize('prec', ['c128', 'c64'])
@pytest.mark.parametrize('name', ['small', 'x2', 'p256', 'reference'])
def test_persistent_k1_bit_identical_to_tiled_k1(name, prec):
    """The persistent software-pipelined K1 (k1p_dbf_mtd for power-of-two P; k1q_dbf_mtd for the
    factored DFT of the reference frame's P = 332) and the one-tile-per-workgroup K1
    (RSP_PLAN_K1_TILED) do the same operations in the same order: identical RDM bits and
    detections, on the synchronous path and through the 8-frame queue."""
    s = scenario(name)
    tg = targets_for(name)
    cube = _input_cube(name, s, tg).astype(np.complex128 if prec == 'c128' else np.complex64)
    outs, queued = [], []
    for tiled in (False, True):
        plan = Plan(s['cfg'], s['cfar'], s['clus'], s['pre_p'], frames_per_launch=8, precision=prec, k1_tiled=tiled)
        outs.append(plan.process_cube(cube, frame_idx=1, want_rdm=True))
        ptrs = [plan.device_alloc(plan.cube_bytes) for _ in range(3)]
        try:
            for f, p in enumerate(ptrs):
                plan.synthesize_device(p, tg, frame_idx=f + 1)
            for i in range(10):
                plan.enqueue(ptrs[i % 3], i + 1)
            plan.drain()
            queued.append(plan.results())
        finally:
            for p in ptrs:
                plan.device_free(p)
            plan.close()
    assert np.array_equal(outs[1]['rdm'], outs[0]['rdm'])
    assert outs[1]['detections'] == outs[0]['detections']
    assert outs[1]['final_targets'] == outs[0]['final_targets']
    assert [r['frame_idx'] for r in queued[1]] == [r['frame_idx'] for r in queued[0]]
    assert [r['final_targets'] for r in queued[1]] == [r['final_targets'] for r in queued[0]]
