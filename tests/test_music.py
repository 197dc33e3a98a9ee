"""MUSIC DOA (MUSIC_1D.m:21-48, run_music_algorithm.m:22-69; SURVEY 8(f) rank 1, BASELINE #5).

CPU tests pin the oracle (oracle/music.py) by known answers the scripts themselves imply;
GPU tests compare librsp's MUSIC path with the complex128 oracle on identical snapshots, in
both plan precisions.

Complex double (the default, MATLAB's arithmetic: f64 MFMA covariance, Householder +
multisection + inverse iteration in double), tolerances written here:
  * synthesis: max |X_dev - X_oracle| <= 1e-12 * max |X_oracle| (fp64 on both sides);
  * covariance: max |R_dev - R| <= 1e-12 * max |R|;
  * eigenvalues: max |d_dev - d| <= 1e-11 * max d;
  * spectrum: |dB_dev - dB| <= 1e-7 dB wherever the oracle is above -60 dB;
  * peaks: the same M indices, in the same order, and the same findpeaks count -- exactly.
Complex single (precision 'c64': f32 MFMA covariance, one-wave fp32 eigensolver):
  * synthesis 1e-6, covariance 2e-6, eigenvalues 2e-5 (relative to the maximum), spectrum
    0.02 dB; peaks the same except that a peak whose oracle height is within 0.02 dB of another
    candidate may trade places with it.
Parity beyond the oracle is unpinned: the reference holds no MUSIC fixtures and MATLAB is absent.
"""
import numpy as np
import pytest

from oracle import music as mu

SEED = 20250101


# ---------------------------------------------------------------------------- CPU: oracle
def test_findpeaks_semantics():
    """MATLAB findpeaks: strict local maxima, first sample of a flat top, never the ends."""
    y = np.array([5, 1, 3, 3, 2, 4, 4, 4, 6, 0, 7, 7])
    assert list(mu.findpeaks(y)) == [2, 8]          # plateau 3,3 -> index 2; 6 at 8; ends excluded
    assert list(mu.findpeaks([1, 2, 2, 2])) == []   # plateau running into the end
    assert list(mu.findpeaks([0, 1, 0, 1, 0])) == [1, 3]
    assert list(mu.findpeaks([1, 1, 1])) == []


def test_noise_free_nulls_sit_on_the_sources():
    """With sources on the scan grid and no noise the noise subspace is orthogonal to the
    source steering vectors: the pseudo-spectrum peaks exactly at them (MUSIC_1D.m:37)."""
    scan = np.deg2rad(np.arange(-90, 91, 1.0))
    scene = {'angles_rad': np.deg2rad([-30.0, -10.0, 60.0]), 'complex_sources': 0, 'snr_db': 300.0,
             'snr_measured': 1}
    X = mu.synthesize(scene, 10, 1000, 0.5, 0, SEED)       # MUSIC_1D.m:10,18 (N = 10, K = 1000)
    r = mu.music_1d(X, 3, scan, 0.5)
    assert np.allclose(sorted(r['angles_deg']), [-30.0, -10.0, 60.0], atol=1e-9)
    assert np.abs(r['eig'][3:]).max() < 1e-12 * r['eig'][0]   # rank-M covariance


def test_eigenvalue_structure_matches_the_signal_model():
    """R -> S Rs S^H + sigma^2 I: the N - M noise eigenvalues cluster at the measured noise
    power (awgn 'measured', MUSIC_1D.m:24) within the Marchenko-Pastur band."""
    scene, scan, dl = mu.music_1d_scene()
    N, K = 64, 1024
    X = mu.synthesize(scene, N, K, dl, 3, SEED)
    r = mu.music_1d(X, 3, scan, dl)
    p_sig = 3.0                                                # three unit-variance real sources
    sigma2 = p_sig / 10.0
    lo, hi = sigma2 * (1 - np.sqrt(N / K)) ** 2, sigma2 * (1 + np.sqrt(N / K)) ** 2
    noise = r['eig'][3:]
    assert noise.min() > 0.8 * lo and noise.max() < 1.2 * hi
    assert r['eig'][2] > 20 * noise.max()
    assert np.all(np.abs(np.sort(r['angles_deg']) - np.array([-30.0, -10.0, 60.0])) < 1.0)


def test_run_music_resolves_the_close_pair():
    """run_music_algorithm.m:14-15: 2.0 and -1.5 deg are resolved on the 0.1 deg grid."""
    scene, scan, dl = mu.run_music_scene()
    X = mu.synthesize(scene, 16, 256, dl, 0, SEED)
    r = mu.music_1d(X, 2, scan, dl)
    assert sorted(np.round(r['angles_deg'], 1)) == [-1.5, 2.0]


def test_batch_oracle_equals_per_instance():
    scene, scan, dl = mu.music_1d_scene()
    Xs = np.stack([mu.synthesize(scene, 16, 128, dl, i, SEED) for i in range(4)])
    PdB, pk = mu.music_batch(Xs, 3, scan, dl)
    for i in range(4):
        r = mu.music_1d(Xs[i], 3, scan, dl)
        assert np.abs(PdB[i] - r['spectrum_db']).max() < 1e-9
        assert list(pk[i]) == list(r['peaks'])


def test_product_scenes_equal_oracle_scenes():
    """rsp.music's scene constants (used by bench.py) restate the same script lines as the oracle's."""
    from rsp import music as pm
    for a, b in ((pm.music_1d_scene(), mu.music_1d_scene()), (pm.run_music_scene(), mu.run_music_scene())):
        assert a[2] == b[2] and np.array_equal(a[1], b[1])
        for k in b[0]:
            assert np.array_equal(np.asarray(a[0][k]), np.asarray(b[0][k])), k


def test_music_bad_config_is_rejected():
    from rsp import _abi
    from rsp.music import MusicPlan
    with pytest.raises(_abi.RspError) as e:
        MusicPlan(65, 128, 3, np.linspace(-1, 1, 50))
    assert e.value.code == _abi.RSP_ERR_UNSUPPORTED
    with pytest.raises(_abi.RspError) as e:
        MusicPlan(16, 128, 16, np.linspace(-1, 1, 50))     # M must leave a noise subspace
    assert e.value.code == _abi.RSP_ERR_UNSUPPORTED


# ---------------------------------------------------------------------------- GPU: parity
CASES = {
    # BASELINE config #5: 64 channels x 1024 snapshots, MUSIC_1D.m scene
    'config5': (64, 1024, 3, mu.music_1d_scene),
    # the literal MUSIC_1D.m: N = 10 (not a multiple of 4: scalar-load covariance), K = 1000
    'music_1d': (10, 1000, 3, mu.music_1d_scene),
    # run_music_algorithm.m: 16 channels, 256 snapshots, 401-point degree grid
    'run_music': (16, 256, 2, mu.run_music_scene),
}


TOL = {'c128': dict(X=1e-12, R=1e-12, eig=1e-11, db=1e-7, swap=0.0),
       'c64': dict(X=1e-6, R=2e-6, eig=2e-5, db=0.02, swap=0.02)}
PARAMS = [(c, p) for c in sorted(CASES) for p in ('c128', 'c64')]


@pytest.fixture(scope='module', params=PARAMS, ids=['%s-%s' % cp for cp in PARAMS])
def music_case(request):
    from rsp.music import MusicPlan
    name, prec = request.param
    N, K, M, mk = CASES[name]
    scene, scan, dl = mk()
    n_inst = 8
    plan = MusicPlan(N, K, M, scan, dl, max_batch=n_inst, precision=prec)
    d_X = plan.device_alloc(n_inst)
    plan.synthesize_device(d_X, scene, n_inst, inst0=0, seed=SEED)
    X = plan.download(d_X, n_inst)
    out = plan.process_device(d_X, n_inst, want_cov=True)
    prof = plan.profile(d_X, n_inst, iters=2)
    ref = [mu.music_1d(X[i].astype(np.complex128), M, scan, dl) for i in range(n_inst)]
    yield dict(N=N, K=K, M=M, scene=scene, scan=scan, dl=dl, X=X, out=out, ref=ref, plan=plan, prof=prof,
               n=n_inst, tol=TOL[prec], prec=prec, name=name)
    plan.device_free(d_X)
    plan.close()


@pytest.mark.gpu
def test_music_synthesis_matches_oracle(music_case):
    c = music_case
    for i in range(c['n']):
        x = mu.synthesize(c['scene'], c['N'], c['K'], c['dl'], i, SEED)
        assert np.abs(c['X'][i] - x).max() <= c['tol']['X'] * np.abs(x).max()


@pytest.mark.gpu
def test_music_covariance_mfma(music_case):
    c = music_case
    for i in range(c['n']):
        R = c['ref'][i]['R']
        assert np.abs(c['out']['R'][i] - R).max() <= c['tol']['R'] * np.abs(R).max()


@pytest.mark.gpu
def test_music_eigenvalues(music_case):
    c = music_case
    assert c['prof']['eig_ms'] > 0.0
    for i in range(c['n']):
        d = c['ref'][i]['eig']
        assert np.abs(c['out']['eig'][i] - d).max() <= c['tol']['eig'] * d.max()


@pytest.mark.gpu
def test_music_spectrum_and_peaks(music_case):
    c = music_case
    for i in range(c['n']):
        ref = c['ref'][i]['spectrum_db']
        got = c['out']['spectrum_db'][i]
        live = ref > -60.0
        assert np.abs(got[live] - ref[live]).max() <= c['tol']['db']
        want = list(c['ref'][i]['peaks'])
        have = list(c['out']['peaks'][i])
        if c['prec'] == 'c128':
            assert have == want   # index work: exact
        elif have != want:   # complex single: only near-equal peak heights may trade places
            pk = mu.findpeaks(ref)
            hv = np.sort(ref[pk])[::-1]
            assert len(hv) > c['M'] and hv[c['M'] - 1] - hv[c['M']] <= c['tol']['swap'], (have, want)
        assert c['out']['n_peaks'][i] == c['ref'][i]['n_peaks']


@pytest.mark.gpu
def test_music_host_path_equals_device_path(music_case):
    """rsp_music_process (host complex128 X, MATLAB layout) == the device-resident path."""
    c = music_case
    o = c['plan'].process(c['X'][:3])
    assert np.array_equal(o['peaks'], c['out']['peaks'][:3])
    assert np.abs(o['spectrum_db'] - c['out']['spectrum_db'][:3]).max() == 0.0


@pytest.mark.gpu
def test_music_peaks_only_call_equals_full_call(music_case):
    """Without the eigenvalues requested (the bench's step), complex double finds only the M signal
    eigenvalues; the peaks and their count are those of the call that returns every output."""
    c = music_case
    n = c['n']
    peaks = np.zeros((n, c['M']), np.int32)
    npk = np.zeros(n, np.int32)
    d_X = c['plan'].device_alloc(n)
    try:
        c['plan'].synthesize_device(d_X, c['scene'], n, inst0=0, seed=SEED)
        c['plan'].peaks_device(d_X, n, peaks, npk)
    finally:
        c['plan'].device_free(d_X)
    assert np.array_equal(peaks, c['out']['peaks'])
    assert np.array_equal(npk, c['out']['n_peaks'])
    if c['prec'] == 'c128' and c['name'] in ('config5', 'music_1d'):
        # complex double answers these scenes through the block-power fast path (every instance
        # converges with the proven subspace bound); the full call above ran the full eigensolver
        assert c['plan'].fast_count() == n


@pytest.mark.gpu
def test_music_fast_path_falls_back_on_a_small_gap():
    """A covariance whose M-th and (M+1)-th eigenvalues are nearly equal: the block power
    iteration cannot prove convergence in its fixed steps, so every instance must take the full
    eigensolver -- and the peaks-only call still equals the full call."""
    from rsp.music import MusicPlan
    N, K, M = 16, 64, 2
    scan = np.linspace(-np.pi / 2, np.pi / 2, 50)
    rng = np.random.default_rng(7)
    mags = np.concatenate([[9.0, 1.0 + 1e-3, 1.0], rng.uniform(0.2, 0.5, N - 3)])   # lambda_2 ~ lambda_3
    Q, _ = np.linalg.qr(rng.standard_normal((N, N)) + 1j * rng.standard_normal((N, N)))
    X = np.zeros((2, N, K), np.complex128)
    for i in range(2):   # X X^H / K = Q diag(mags) Q^H exactly: X = Q sqrt(K mags) on N snapshots
        X[i, :, :N] = Q @ np.diag(np.sqrt(mags * K))
    plan = MusicPlan(N, K, M, scan, 0.5, max_batch=2)
    try:
        full = plan.process(X)
        assert plan.fast_count() == 0   # the full call (every eigenvalue requested)
        pk, npk = plan.peaks(X)
        assert plan.fast_count() == 0   # peaks-only: lambda_3 / lambda_2 ~ 1, no proof in 8 powers
        assert np.array_equal(pk, full['peaks']) and np.array_equal(npk, full['n_peaks'])
    finally:
        plan.close()
    ev = np.sort(full['eig'][0])[::-1][:3]
    assert np.abs(ev - [9.0, 1.001, 1.0]).max() <= 1e-12 * 9.0


@pytest.mark.gpu
def test_music_fast_path_taken_on_well_separated_signals():
    """The converse: a large gap (lambda_2 / lambda_3 = 100) converges in the fixed steps, so the
    peaks-only call takes the fast path for every instance and equals the full call."""
    from rsp.music import MusicPlan
    N, K, M = 16, 64, 2
    scan = np.linspace(-np.pi / 2, np.pi / 2, 50)
    rng = np.random.default_rng(8)
    mags = np.concatenate([[900.0, 100.0], rng.uniform(0.5, 1.0, N - 2)])
    Q, _ = np.linalg.qr(rng.standard_normal((N, N)) + 1j * rng.standard_normal((N, N)))
    X = np.zeros((2, N, K), np.complex128)
    for i in range(2):
        X[i, :, :N] = Q @ np.diag(np.sqrt(mags * K))
    plan = MusicPlan(N, K, M, scan, 0.5, max_batch=2)
    try:
        full = plan.process(X)
        pk, npk = plan.peaks(X)
        assert plan.fast_count() == 2
    finally:
        plan.close()
    assert np.array_equal(pk, full['peaks']) and np.array_equal(npk, full['n_peaks'])


@pytest.mark.gpu
def test_music_decoupled_covariance_eigenvalues():
    """A covariance whose tridiagonal form is decoupled (every off-diagonal exactly zero): X with
    one snapshot per channel gives R = diag(|a_n|^2 / K), and the Householder steps are all the
    identity.  The multisection Sturm count must then return the diagonal itself, sorted
    descending (MUSIC_1D.m:29-31), including repeated values; rows with e = 0 are the case where
    an exactly zero leading minor must not flip the count twice (dstebz's -pivmin rule)."""
    from rsp.music import MusicPlan
    N, K, M = 16, 64, 3
    scan = np.linspace(-np.pi / 2, np.pi / 2, 50)
    rng = np.random.default_rng(5)
    mags = np.concatenate([rng.uniform(0.5, 4.0, N - 4), [2.0, 2.0, 1.0, 1.0]])   # repeated eigenvalues
    X = np.zeros((2, N, K), np.complex128)
    for i in range(2):
        ph = np.exp(2j * np.pi * rng.random(N))
        X[i, np.arange(N), np.arange(N)] = np.sqrt(mags * K) * ph
    plan = MusicPlan(N, K, M, scan, 0.5, max_batch=2)
    try:
        o = plan.process(X)
    finally:
        plan.close()
    want = np.sort(mags)[::-1]
    for i in range(2):
        assert np.abs(o['eig'][i] - want).max() <= 1e-12 * want.max(), (o['eig'][i], want)


@pytest.mark.gpu
@pytest.mark.parametrize('scale', [1e-60, 1e40])
def test_music_scale_invariance(music_case, scale):
    """eig is scale-invariant: X scaled by 1e-60 (R by 1e-120) or 1e40 gives eigenvalues scaled by
    scale^2 (to the c128 tolerance) and the same spectrum, peaks and findpeaks count (ADVICE r4:
    the Sturm count's e^2 floor is relative to ||T||, not an absolute 2^-600)."""
    c = music_case
    if c['prec'] != 'c128':
        pytest.skip('complex single cannot hold R at 1e-120 / 1e80')
    o = c['plan'].process(c['X'][:2] * scale)
    for i in range(2):
        d = c['out']['eig'][i]
        assert np.abs(o['eig'][i] / scale ** 2 - d).max() <= c['tol']['eig'] * d.max()
        assert list(o['peaks'][i]) == list(c['out']['peaks'][i])
        assert o['n_peaks'][i] == c['out']['n_peaks'][i]
        live = c['out']['spectrum_db'][i] > -60.0
        assert np.abs(o['spectrum_db'][i][live] - c['out']['spectrum_db'][i][live]).max() <= 1e-6


@pytest.mark.gpu
@pytest.mark.parametrize('N,M', [(4, 2), (3, 2), (4, 3)])
def test_music_small_n_full_call_returns_every_eigenvalue(N, M):
    """with N <= 4 a call that reads the eigenvalues asks for neig = N <= 4, which
    must not select the peaks-only fast path (it writes no eigenvalue when it converges).  The
    output array starts at zero, so an unwritten eigenvalue fails the comparison with LAPACK's
    eigvalsh of the same covariance; the spectrum and peaks are the oracle's too."""
    from rsp.music import MusicPlan
    K, n = 64, 3
    scan = np.linspace(-np.pi / 2, np.pi / 2, 60)
    rng = np.random.default_rng(100 * N + M)
    X = rng.standard_normal((n, N, K)) + 1j * rng.standard_normal((n, N, K))
    X[:, :, :4] *= 5.0
    plan = MusicPlan(N, K, M, scan, 0.5, max_batch=n)
    try:
        o = plan.process(X)
        assert plan.fast_count() == 0
        pk, npk = plan.peaks(X)   # the peaks-only call may take the fast path; same answer
        sp = plan.process(X, want_eig=False)   # the spectrum call: fast path only under its dB bound
    finally:
        plan.close()
    for i in range(n):
        R = X[i] @ X[i].conj().T / K
        want = np.sort(np.linalg.eigvalsh(R))[::-1]
        assert np.abs(o['eig'][i] - want).max() <= 1e-11 * want.max(), (o['eig'][i], want)
        ref = mu.music_1d(X[i], M, scan, 0.5)
        live = ref['spectrum_db'] > -60.0
        assert np.abs(o['spectrum_db'][i][live] - ref['spectrum_db'][live]).max() <= 1e-7
        # the device pads the M peak slots with 0 when findpeaks finds fewer (N = 4, M = 3 here)
        have = [int(p) for p in o['peaks'][i] if p > 0]
        assert have == [int(p) for p in ref['peaks']] == [int(p) for p in pk[i] if p > 0]
        assert list(o['peaks'][i]) == list(pk[i])
        assert o['n_peaks'][i] == ref['n_peaks'] == npk[i]
        assert np.abs(sp['spectrum_db'][i][live] - ref['spectrum_db'][live]).max() <= 1e-7
        assert list(sp['peaks'][i]) == list(o['peaks'][i]) and sp['n_peaks'][i] == o['n_peaks'][i]


@pytest.mark.gpu
def test_music_spectrum_call_without_eigenvalues(music_case):
    """a call that reads spectrum_db but not the eigenvalues (rsp_mex('music')
    with two outputs) keeps the block-power subspace only where its proven 1e-12 subspace bound
    also bounds P_dB's error by 1e-8 dB (<= 8.69e-12 n / den_min), else runs the full
    eigensolver; either way its spectrum holds the oracle tolerance and its peaks are the full
    call's.  Complex double: config #5 (den_min ~ 0.4, bound ~1.5e-9 dB) takes the fast path for
    every instance; MUSIC_1D.m's N = 10 scene (den_min ~ 0.003, bound ~3e-8 dB) converges (the
    peaks-only call takes the fast path) but must fall back here."""
    c = music_case
    o = c['plan'].process(c['X'][:4], want_eig=False)
    assert 'eig' not in o
    if c['prec'] == 'c128' and c['name'] == 'config5':
        assert c['plan'].fast_count() == 4
    if c['prec'] == 'c128' and c['name'] == 'music_1d':
        assert c['plan'].fast_count() == 0
        c['plan'].peaks(c['X'][:4])
        assert c['plan'].fast_count() == 4   # so the fallback above was the spectrum bound's
    for i in range(4):
        ref = c['ref'][i]['spectrum_db']
        live = ref > -60.0
        assert np.abs(o['spectrum_db'][i][live] - ref[live]).max() <= c['tol']['db']
        if c['prec'] == 'c128':   # against the full path (eigenvalues read) of the same instance
            full = c['out']['spectrum_db'][i]
            assert np.abs(o['spectrum_db'][i][live] - full[live]).max() <= 1e-8
        assert list(o['peaks'][i]) == list(c['out']['peaks'][i])
        assert o['n_peaks'][i] == c['out']['n_peaks'][i]


@pytest.mark.gpu
def test_music_spectrum_device_form(music_case):
    """MusicPlan.spectrum_device (bench.py --want-spectrum's step) returns the host call's spectrum
    and peaks for device-resident snapshots."""
    c = music_case
    n = 4
    spec = np.zeros((n, len(c['scan'])), np.float64)
    pk = np.zeros((n, c['M']), np.int32)
    npk = np.zeros(n, np.int32)
    d_X = c['plan'].device_alloc(n)
    try:
        c['plan'].synthesize_device(d_X, c['scene'], n, inst0=0, seed=SEED)
        c['plan'].spectrum_device(d_X, n, spec, pk, npk)
    finally:
        c['plan'].device_free(d_X)
    o = c['plan'].process(c['X'][:n], want_eig=False)
    assert np.array_equal(spec, o['spectrum_db'])
    assert np.array_equal(pk, o['peaks']) and np.array_equal(npk, o['n_peaks'])


@pytest.mark.gpu
@pytest.mark.parametrize('scale', [1e-80, 1e-60, 1e40])
def test_music_peaks_only_scale_invariance(music_case, scale):
    """The peaks-only call (fast path) at scaled snapshots: ADVICE r5 (low) -- the fast path's
    ||A||_F^2 is summed from the scaled entries, so R ~ 1e-160 (X ~ 1e-80) no longer underflows the
    squares and the Davis-Kahan bound keeps its ||C|| term.  Peaks and counts are the unscaled ones."""
    c = music_case
    if c['prec'] != 'c128':
        pytest.skip('complex single cannot hold R at these scales')
    pk, npk = c['plan'].peaks(c['X'][:2] * scale)
    assert np.array_equal(pk, c['out']['peaks'][:2])
    assert np.array_equal(npk, c['out']['n_peaks'][:2])
    if c['name'] in ('config5', 'music_1d'):
        assert c['plan'].fast_count() == 2
