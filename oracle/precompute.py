"""Oracle restatement of the v8 precompute -- TEST INFRASTRUCTURE ONLY.

Follows ``main_simulate_echoes_with_array_v8.m:79-155`` (section "%% 3"),
parameterised by the config dict (same field names as the MATLAB structs
``config.Sig_Config`` / ``config.Array``).  MATLAB semantics made explicit:
``round`` = half away from zero, ``kaiser`` = I0 window, ``grpdelay`` =
mean group delay over 512 points, ``fft(x, n)`` zero-pads to n.
"""
import numpy as np
import scipy.signal as ss


def mround(x):
    """MATLAB round(): half away from zero."""
    return np.sign(x) * np.floor(np.abs(x) + 0.5)


def nextpow2(n):
    """MATLAB nextpow2 for positive integers."""
    return int(np.ceil(np.log2(n))) if n > 0 else 0


def precompute(config, dbf_coeffs, beam_angles_deg, k_slopes_LUT, fir_coeffs):
    sc = config['Sig_Config']
    fs, c, P = sc['fs'], sc['c'], sc['prtNum']
    N = sc['point_PRT']
    wl = sc['wavelength']
    tau1, tau2, tau3 = sc['tao']
    gap1, gap2 = sc['gap_duration'][0], sc['gap_duration'][1]
    segs = sc['point_prt_segments']
    G = int(sum(segs))
    ts = 1.0 / fs
    pre = {}
    # --- 3.1 waveform (v8:80-98)
    k2 = -sc['B'] / tau2
    k3 = sc['B'] / tau3
    ns1 = int(mround(tau1 * fs)); ns2 = int(mround(tau2 * fs)); ns3 = int(mround(tau3 * fs))
    t2 = np.linspace(-tau2 / 2, tau2 / 2, ns2)
    t3 = np.linspace(-tau3 / 2, tau3 / 2, ns3)
    pulse2 = np.exp(1j * 2 * np.pi * (0.5 * k2 * t2 ** 2))
    pulse3 = np.exp(1j * 2 * np.pi * (0.5 * k3 * t3 ** 2))
    tx = np.zeros(N, complex)
    tx[:ns1] = 1.0
    off1 = int(mround((tau1 + gap1) * fs))
    tx[off1:off1 + ns2] = pulse2
    off2 = off1 + int(mround((tau2 + gap2) * fs))
    tx[off2:off2 + ns3] = pulse3
    pre['tx_pulse'] = tx
    pre['P_signal_unscaled'] = float(np.mean(np.abs(tx[tx != 0]) ** 2))
    # --- 3.2 matched filters (v8:101-109)
    fir = np.asarray(fir_coeffs, float)
    fir = 6 * fir / np.max(fir)
    pre['MF_narrow'] = fir
    _, gd = ss.group_delay((fir, [1.0]), w=512)
    pre['fir_delay'] = int(mround(np.mean(gd)))
    pre['MF_medium_win'] = np.conj(pulse2 * np.kaiser(ns2, 4.5))[::-1]
    pre['MF_long_win'] = np.conj(pulse3 * np.kaiser(ns3, 4.5))[::-1]
    # --- 3.3 frequency-domain filters (v8:112-123)
    gap1n = gap1 * fs
    gap2n = gap2 * fs
    ssm = ns1 + gap1n + ns2 + 1
    ssl = ns1 + gap1n + ns2 + gap2n + ns3 + 1
    assert float(ssm).is_integer() and float(ssl).is_integer(), 'non-integer segment start'
    ssm, ssl = int(ssm), int(ssl)
    Ls_m = N - ssm + 1
    Ls_l = N - ssl + 1
    pre['N_fft_med'] = 2 ** nextpow2(Ls_m + ns2 - 1)
    pre['N_fft_long'] = 2 ** nextpow2(Ls_l + ns3 - 1)
    pre['MF_medium_fft'] = np.fft.fft(pre['MF_medium_win'], pre['N_fft_med'])
    pre['MF_long_fft'] = np.fft.fft(pre['MF_long_win'], pre['N_fft_long'])
    # --- 3.4 stitching (v8:126-132)
    pre['N_gate_narrow'], pre['N_gate_medium'], pre['N_gate_long'] = (int(s) for s in segs)
    pre['N_total_gate'] = G
    pre['seg_start_narrow'] = ns1 + 1
    pre['seg_start_medium'] = ssm
    pre['seg_start_long'] = ssl
    # --- 3.5 MTD window (v8:135)
    pre['MTD_win'] = np.kaiser(P, 4.5)
    # --- 3.6 axes (v8:138-145)
    v_max = wl / (2 * sc['prt'])
    pre['velocity_axis'] = np.linspace(-v_max / 2, v_max / 2, P)
    pre['range_axis'] = np.arange(G) * (c / (2 * fs))
    pre['deltaR'] = c * ts / 2
    pre['deltaV'] = v_max / P
    pre['beam_angles_deg'] = np.asarray(beam_angles_deg, float)
    pre['k_slopes_LUT'] = np.asarray(k_slopes_LUT, float)
    # --- 3.7 DBF weights (v8:148-150), already complex B x C
    pre['DBF_coeffs_data_C'] = np.asarray(dbf_coeffs, complex)
    return pre
