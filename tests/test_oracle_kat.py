"""CPU tests: pin the oracle against the known answers derivable from the reference.

The reference (MATLAB) holds no golden vectors and cannot run here; SURVEY.md section 4
lists the known-answer tests derivable from its own files (KAT-1..KAT-4).  These tests
pin the oracle (oracle/) and the product's host precompute against them, and pin the
vectorised oracle CFAR against a literal scalar restatement of fsf:192-213.
"""
import numpy as np
import pytest

from oracle import chain, precompute as op
from oracle.philox import philox4x32_10, unit_normal_complex
from rsp import config as C
from rsp.precompute import precompute as product_precompute

from _scen import scenario


@pytest.fixture(scope='module')
def ref():
    cfg, cfar, clus, W, ang, k = C.named_config('reference')
    return cfg, op.precompute(cfg, W, ang, k, C.V8_FIR)


def test_kat1_integer_geometry(ref):
    """v8:68,93-96,114-123 evaluate to exact integers at the reference config."""
    cfg, pre = ref
    sc = cfg['Sig_Config']
    assert sc['point_PRT'] == 5819
    tx = pre['tx_pulse']
    nz = np.flatnonzero(tx)
    assert nz[0] == 0 and list(nz[:4]) == [0, 1, 2, 3]            # rect 4 samples
    assert np.flatnonzero(tx[4:])[0] + 4 == 289                    # offset1
    assert np.flatnonzero(tx[489:])[0] + 489 == 1284               # offset2
    assert nz[-1] == 1284 + 700 - 1                                # tx span 1984 samples
    assert (pre['seg_start_narrow'], pre['seg_start_medium'], pre['seg_start_long']) == (5, 490, 1985)
    assert 5819 - 490 + 1 == 5330 and 5819 - 1985 + 1 == 3835
    assert (pre['N_fft_med'], pre['N_fft_long']) == (8192, 8192)
    assert pre['N_total_gate'] == 3404


def test_kat2_fir_group_delay(ref):
    """round(mean(grpdelay(fir))) of the symmetric 35-tap FIR = 17 (v8:104)."""
    _, pre = ref
    assert pre['fir_delay'] == 17
    assert pre['MF_narrow'].max() == 6.0


def test_kat3_beam_peaks():
    """plot_beam_patterns.m:20,38,52-85: |fliplr(W) a(theta)| peaks at beam_angles_deg (v8:144)."""
    W = C.load_reference_dbf()[:, ::-1]
    wl = C.C_LIGHT / 9500e6
    ang = np.arange(-900, 1001) / 10
    n = np.arange(1, 17)[:, None]
    sv = np.exp(1j * 2 * np.pi * 0.0138 * n * np.sin(np.deg2rad(ang))[None, :] / wl)
    peaks = ang[np.argmax(np.abs(W @ sv), axis=1)]
    assert np.allclose(peaks, C.V8_BEAM_ANGLES)


def test_kat3_kernel_convention_beam_peaks():
    """With the kernel's convention (x * W', phases exp(j c dphi), c = 0..15, fc 9.45 GHz)
    every reference beam peaks within 0.8 deg of its nominal angle (SURVEY KAT-3)."""
    W = C.load_reference_dbf()
    wl = C.C_LIGHT / 9450e6
    ang = np.arange(-900, 1001) / 10
    c = np.arange(16)[:, None]
    a = np.exp(1j * 2 * np.pi * 0.0138 * c * np.sin(np.deg2rad(ang))[None, :] / wl)
    peaks = ang[np.argmax(np.abs(np.conj(W) @ a), axis=1)]
    assert np.abs(peaks - np.asarray(C.V8_BEAM_ANGLES)).max() <= 0.8


@pytest.mark.parametrize('name', ['small', 'x2'])
def test_kat4_noiseless_peak_position(name):
    """Noiseless single target: |RDM| peaks at gate (1-based) = delay_samples for the
    medium/long segments and at the fftshifted Doppler bin nearest 2v/lambda (KAT-4)."""
    s = scenario(name)
    cfg, pre = s['cfg'], s['pre_o']
    sc = cfg['Sig_Config']
    # target inside the long-segment gates, on a beam's boresight
    G = pre['N_total_gate']
    g1, g2 = pre['N_gate_narrow'], pre['N_gate_medium']
    delay = (g1 + g2 + G) // 2
    rng = delay * sc['c'] / (2 * sc['fs'])
    v = 0.2 * sc['wavelength'] / (2 * sc['prt'])
    ang = float(pre['beam_angles_deg'][1])
    raw = chain.synthesize_echo([dict(Range=rng, Velocity=v, ElevationAngle=ang, SNR_dB=20.0)], cfg, pre)
    fin, st = chain.process_cube(raw, cfg, s['cfar'], s['clus'], pre, keep=True)
    A = np.abs(st['rdm'][:, :, 1])
    vi, ri = np.unravel_index(np.argmax(A), A.shape)
    assert ri + 1 == delay
    fd = 2 * v / sc['wavelength']
    P = sc['prtNum']
    k = int(np.round(fd * sc['prt'] * P)) % P
    assert vi == (k + P // 2) % P


def test_product_precompute_matches_oracle():
    for name in ['reference', 'x2', 'small', 'plumbing', 'x4']:
        cfg, cfar, clus, W, ang, k = C.named_config(name)
        a = product_precompute(cfg, W, ang, k, C.V8_FIR)
        b = op.precompute(cfg, W, ang, k, C.V8_FIR)
        assert set(a) == set(b)
        for key in a:
            np.testing.assert_allclose(np.asarray(a[key]), np.asarray(b[key]), rtol=1e-12, atol=1e-12,
                                       err_msg='%s.%s' % (name, key))


def test_philox_random123_kats():
    """Published Philox4x32-10 known-answer vectors (Random123)."""
    vecs = [((0, 0, 0, 0), (0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
            ((0xffffffff,) * 4, (0xffffffff, 0xffffffff), (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
            ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
             (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1))]
    for ctr, key, want in vecs:
        got = philox4x32_10(*[np.uint32(x) for x in ctr], *key)
        assert tuple(int(g) for g in got) == want


def test_noise_statistics():
    z = unit_normal_complex(1 << 18, frame_idx=7, seed=20250101)
    assert abs(z.real.mean()) < 0.01 and abs(z.imag.mean()) < 0.01
    assert abs(z.real.var() - 1) < 0.01 and abs(z.imag.var() - 1) < 0.01
    assert abs(np.mean(z.real * z.imag)) < 0.01
    z2 = unit_normal_complex(1 << 10, frame_idx=8, seed=20250101)
    assert not np.allclose(z[:1 << 10], z2)


def _cfar_scalar(S, cfar):
    """Literal restatement of the fsf:192-213 double loop (1-based -> 0-based)."""
    nV, nR = S.shape
    gR, gV, rR, rV, T = (cfar['guardCells_R'], cfar['guardCells_V'], cfar['refCells_R'],
                         cfar['refCells_V'], cfar['T_CFAR'])
    det = np.zeros_like(S, bool)
    for r in range(rR + gR, nR - rR - gR):
        for v in range(rV + gV, nV - rV - gV):
            nr = max(np.mean(S[v, r - gR - rR:r - gR]), np.mean(S[v, r + gR + 1:r + gR + rR + 1]))
            nv = max(np.mean(S[v - gV - rV:v - gV, r]), np.mean(S[v + gV + 1:v + gV + rV + 1, r]))
            det[v, r] = S[v, r] > T * max(nr, nv)
    return det


def test_cfar_vectorised_equals_scalar_loop():
    rng = np.random.default_rng(5)
    P, G, B = 48, 80, 3
    rdm = (rng.standard_normal((P, G, B)) + 1j * rng.standard_normal((P, G, B)))
    rdm[20, 40, :] *= 60
    rdm[30, 50, 1] *= 40
    cfar = C.default_cfar_params()
    dets, S_all = chain.goca_cfar(rdm, cfar)
    want = []
    for p in range(B - 1):
        m = _cfar_scalar(S_all[:, :, p], cfar)
        rr, vv = np.nonzero(m.T)
        want += [(v + 1, r + 1, p + 1) for r, v in zip(rr, vv)]
    assert [tuple(int(x) for x in d[:3]) for d in dets] == want
    assert len(want) >= 2


def test_spline_peak_symmetric_and_shifted():
    cells = np.arange(10, 15)
    y = np.array([1.0, 3.0, 5.0, 3.0, 1.0])
    assert chain._spline_peak(cells, y, 1 / 8) == 12.0
    y2 = np.array([1.0, 3.0, 5.0, 4.5, 1.0])           # peak pulled right of the centre cell
    assert 12.0 < chain._spline_peak(cells, y2, 1 / 8) <= 12.5


def test_cluster_stage1_chaining_and_weights():
    """BFS links transitively (fsf:313-336) and merges with power weights (fsf:341-351)."""
    cp = C.default_cluster_params()
    d = [dict(Range=1000.0, Velocity=5.0, Angle=1.0, Power=1.0),
         dict(Range=1025.0, Velocity=5.1, Angle=2.0, Power=3.0),
         dict(Range=1050.0, Velocity=5.2, Angle=3.0, Power=1.0),   # chained via the middle one
         dict(Range=1000.0, Velocity=9.0, Angle=1.0, Power=2.0)]   # separate in velocity
    out = chain.cluster_stage1(d, cp)
    assert len(out) == 2
    assert out[0]['Power'] == 5.0
    assert out[0]['Range'] == pytest.approx((1000 + 3 * 1025 + 1050) / 5)
    assert out[1]['Velocity'] == 9.0


def test_cluster_stage2_winner_take_all():
    """Stage 2 groups on (R, V) only and keeps the first max-Power member (fsf:393-406)."""
    cp = C.default_cluster_params()
    t = [dict(Range=1000.0, Velocity=5.0, Angle=1.0, Power=2.0),
         dict(Range=1010.0, Velocity=5.1, Angle=30.0, Power=7.0),
         dict(Range=1020.0, Velocity=5.2, Angle=-3.0, Power=7.0)]
    out = chain.cluster_stage2(t, cp)
    assert len(out) == 1 and out[0]['Angle'] == 30.0


def test_empty_paths():
    """Empty detection lists give empty outputs (fsf:229-231, 305-308, 358-361)."""
    cfg, cfar, clus, W, ang, k = C.named_config('plumbing')   # 1 beam -> no pairs (fsf:181)
    pre = op.precompute(cfg, W, ang, k, C.V8_FIR)
    raw = chain.synthesize_echo([], cfg, pre) + chain.philox_noise(cfg, 1, 1)
    fin, st = chain.process_cube(raw, cfg, cfar, clus, pre, keep=True)
    assert fin == [] and st['dets'].shape == (0, 4) and st['par'] == []


def test_k_calibration_literal_reproduces_negative_kat():
    """calibrate_all_monopulse_slopes.m:24-73 restated literally (fliplr'd CSV weights, complex
    w*a responses, real() of the complex ratio, 11-point polyfit) on the reference CSV gives the
    SURVEY section-4 negative KAT K = [-2.54, -2.33, ..., -21.49] -- not the LUT hard-coded at
    v8:138, which therefore stays input data."""
    from rsp import config as C
    k = C.calibrate_all_monopulse_slopes(C.load_reference_dbf(), C.V8_BEAM_ANGLES)
    assert k.shape == (12,)
    np.testing.assert_allclose(k[[0, 1, 5, 9, 11]], [-2.5448, -2.3314, -2.9340, -8.4438, -21.4863], atol=5e-4)
    assert np.all(k < 0)
    assert np.abs(k - np.asarray(C.V8_K_LUT)).max() > 1.0   # the hard-coded LUT is not reproducible


def test_k_calibration_amplitude_variant_inverts_the_kernel_ratio():
    """The amplitude variant (synthetic configs, BASELINE #4) is a different, named function: for
    the x4 Taylor-tapered beams, K is the slope d(angle)/d(ratio) of the amplitude ratio
    (|A|-|B|)/(|A|+|B|) of conj(W) a(theta) near the crossover (the ratio the amplitude monopulse
    of fsf:280-290 computes), so K times a ratio change recovers the angle change."""
    from rsp import config as C
    cfg, _, _, W, ang, k = C.named_config('x4')
    d, wl = cfg['Array']['element_spacing'], cfg['Sig_Config']['wavelength']
    k2 = C.calibrate_k_slopes_amplitude(W, ang, d, wl)
    np.testing.assert_array_equal(k, k2)
    n = np.arange(W.shape[1])
    def ratio(p, th):
        a = np.exp(1j * 2 * np.pi * d * n * np.sin(np.deg2rad(th)) / wl)
        A, B = abs(np.conj(W[p]) @ a), abs(np.conj(W[p + 1]) @ a)
        return (A - B) / (A + B)
    for p in (0, 7, 14):
        xo = 0.5 * (ang[p] + ang[p + 1])
        for off in (-0.05, 0.04):
            assert k[p] * (ratio(p, xo + off) - ratio(p, xo)) == pytest.approx(off, rel=0.05)
