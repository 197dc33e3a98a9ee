"""Host-side one-off precompute: the driver's "%% 3" section.

Mirrors ``main_simulate_echoes_with_array_v8.m:79-155`` (identical in
``_v8_1:101-169``, ``_v8_2:117-190``, ``_v8_3:121-189``) and returns the
``precomputed_data`` struct as a dict with the reference's field names.  This is
caller-side setup in float64 (as in MATLAB); the plan uploads what it needs.
"""
import numpy as np


def _mround(x):
    return float(np.sign(x) * np.floor(abs(x) + 0.5))


def _nextpow2(n):
    return int(np.ceil(np.log2(n)))


def _grpdelay_mean(b, npts=512):
    """mean(grpdelay(b, 1)) with MATLAB's default 512 points on [0, pi)."""
    b = np.asarray(b, float)
    w = np.pi * np.arange(npts) / npts
    n = np.arange(len(b))
    e = np.exp(-1j * np.outer(w, n))
    num = e @ (n * b)
    den = e @ b
    ok = np.abs(den) > 1e-12 * np.abs(den).max()
    return float(np.mean(np.real(num[ok] / den[ok])))


def precompute(config, dbf_coeffs, beam_angles_deg, k_slopes_LUT, fir_coeffs):
    sc = config['Sig_Config']
    fs, c, P, N = sc['fs'], sc['c'], sc['prtNum'], sc['point_PRT']
    tau1, tau2, tau3 = sc['tao']
    gap1, gap2 = sc['gap_duration'][:2]
    segs = [int(s) for s in sc['point_prt_segments']]
    G = sum(segs)
    out = {}
    # 3.1 waveform: rect + down-chirp + up-chirp (v8:80-98)
    n1, n2, n3 = (int(_mround(t * fs)) for t in (tau1, tau2, tau3))
    t2 = np.linspace(-tau2 / 2, tau2 / 2, n2)
    t3 = np.linspace(-tau3 / 2, tau3 / 2, n3)
    p2 = np.exp(2j * np.pi * 0.5 * (-sc['B'] / tau2) * t2 ** 2)
    p3 = np.exp(2j * np.pi * 0.5 * (sc['B'] / tau3) * t3 ** 2)
    tx = np.zeros(N, np.complex128)
    o1 = int(_mround((tau1 + gap1) * fs))
    o2 = o1 + int(_mround((tau2 + gap2) * fs))
    tx[:n1] = 1
    tx[o1:o1 + n2] = p2
    tx[o2:o2 + n3] = p3
    out['tx_pulse'] = tx
    out['P_signal_unscaled'] = float(np.mean(np.abs(tx[tx != 0]) ** 2))
    # 3.2 matched filters (v8:101-109)
    fir = np.asarray(fir_coeffs, float)
    fir = 6.0 * fir / fir.max()
    out['MF_narrow'] = fir
    out['fir_delay'] = int(_mround(_grpdelay_mean(fir)))
    out['MF_medium_win'] = np.conj(p2 * np.kaiser(n2, 4.5))[::-1].copy()
    out['MF_long_win'] = np.conj(p3 * np.kaiser(n3, 4.5))[::-1].copy()
    # 3.3 FFT'd filters (v8:112-123); segment starts are 1-based like MATLAB
    ssm = n1 + gap1 * fs + n2 + 1
    ssl = n1 + gap1 * fs + n2 + gap2 * fs + n3 + 1
    if not (float(ssm).is_integer() and float(ssl).is_integer()):
        raise ValueError('segment starts are not integers: %r %r' % (ssm, ssl))
    ssm, ssl = int(ssm), int(ssl)
    out['N_fft_med'] = 2 ** _nextpow2(N - ssm + 1 + n2 - 1)
    out['N_fft_long'] = 2 ** _nextpow2(N - ssl + 1 + n3 - 1)
    out['MF_medium_fft'] = np.fft.fft(out['MF_medium_win'], out['N_fft_med'])
    out['MF_long_fft'] = np.fft.fft(out['MF_long_win'], out['N_fft_long'])
    # 3.4 stitching (v8:126-132)
    out['N_gate_narrow'], out['N_gate_medium'], out['N_gate_long'] = segs
    out['N_total_gate'] = G
    out['seg_start_narrow'] = n1 + 1
    out['seg_start_medium'] = ssm
    out['seg_start_long'] = ssl
    # 3.5-3.6 MTD window and axes (v8:135-145)
    out['MTD_win'] = np.kaiser(P, 4.5)
    v_max = sc['wavelength'] / (2 * sc['prt'])
    out['velocity_axis'] = np.linspace(-v_max / 2, v_max / 2, P)
    out['range_axis'] = np.arange(G) * (c / (2 * fs))
    out['deltaR'] = c / fs / 2
    out['deltaV'] = v_max / P
    out['beam_angles_deg'] = np.asarray(beam_angles_deg, float)
    out['k_slopes_LUT'] = np.asarray(k_slopes_LUT, float)
    # 3.7 DBF weights (v8:148-150), complex B x C
    out['DBF_coeffs_data_C'] = np.asarray(dbf_coeffs, np.complex128)
    return out
