"""Amplitude known-answer test: the RDM peak VALUE of a noiseless target, in closed form.

SURVEY KAT-4 pins only where a noiseless target lands.  Its value follows from the reference's
own definitions, independently of any restatement:

  * echo (fsf:51-73): x[m, n, c] = A exp(j 2 pi fd prt m) tx[n - ds] exp(j c dphi), with
    A = sqrt(10^(SNR/10) P_noise_floor / P_signal_unscaled) (fsf:61-63, P_noise_floor = 1), ds the
    delay in samples, dphi = 2 pi d sin(theta) / lambda (fsf:163-169);
  * DBF (fsf:93-97): beam b scales it by g_b = sum_c conj(W[b, c]) exp(j c dphi);
  * pulse compression (fsf:115-120): the medium / long matched filter is fliplr(conj(chirp .*
    kaiser(L, 4.5))) (v8:106-109); at the gate where the segment's chirp aligns the filter sees that
    chirp alone (the rectangular pulse ends and the other chirp starts outside its L-sample window),
    so the output is A g_b exp(...) sum_q kaiser[q] |chirp[q]|^2 = A g_b exp(...) sum kaiser;
    that gate is ds - 1 (0-based), KAT-4's position;
  * MTD (fsf:131-136): for a Doppler exactly on bin k0 (fd prt P = k0) the window-then-FFT gives
    sum(MTD_win) at the fftshifted bin (k0 + P/2) mod P.

So |RDM[v*, ds - 1, b]| = A |g_b| sum(kaiser_seg) sum(MTD_win) for every beam b.  Checked for a
target in the medium and one in the long segment at BASELINE config #2 (x2) and at the
reference frame, to 1e-11 relative (measured 4e-15 to 5e-14 in the oracle): in the oracle (CPU) and on the device (GPU, complex double).
"""
import numpy as np
import pytest

from oracle import chain
from _scen import scenario

REL = 1e-11


def _kat_target(s, seg):
    """A target on an exact sample delay and an exact Doppler bin, in segment seg."""
    sc = s['cfg']['Sig_Config']
    pre = s['pre_o']
    g1, g2, G = pre['N_gate_narrow'], pre['N_gate_medium'], pre['N_total_gate']
    ds = g1 + g2 // 2 if seg == 'medium' else g1 + g2 + (G - g1 - g2) // 3
    P = sc['prtNum']
    k0 = P // 8 + 3
    R = ds * sc['c'] / (2 * sc['fs'])
    v = k0 * sc['wavelength'] / (2 * sc['prt'] * P)
    return dict(Range=R, Velocity=v, ElevationAngle=10.0, SNR_dB=20.0), ds, k0


def _closed_form(s, t, seg):
    sc = s['cfg']['Sig_Config']
    pre = s['pre_o']
    C = sc['channel_num']
    A = np.sqrt(10 ** (t['SNR_dB'] / 10) * 1.0 / pre['P_signal_unscaled'])
    dphi = 2 * np.pi * s['cfg']['Array']['element_spacing'] * np.sin(np.deg2rad(t['ElevationAngle'])) / sc['wavelength']
    g = np.conj(pre['DBF_coeffs_data_C']) @ np.exp(1j * np.arange(C) * dphi)           # g_b, every beam
    n = round(sc['tao'][1 if seg == 'medium' else 2] * sc['fs'])
    return A * np.abs(g) * np.kaiser(n, 4.5).sum() * np.sum(pre['MTD_win'])


def _peak(rdm, ds, k0, P):
    return np.abs(rdm[(k0 + P // 2) % P, ds - 1, :])


CASES = [('x2', 'medium'), ('x2', 'long'), ('reference', 'medium'), ('reference', 'long')]


@pytest.mark.parametrize('name,seg', CASES)
def test_oracle_rdm_peak_value(name, seg):
    s = scenario(name)
    t, ds, k0 = _kat_target(s, seg)
    cube = chain.synthesize_echo([t], s['cfg'], s['pre_o'])
    pre = s['pre_o']
    rdm = chain.mtd(chain.pulse_compress(chain.dbf(cube, pre['DBF_coeffs_data_C']), pre), pre)
    P = s['cfg']['Sig_Config']['prtNum']
    want = _closed_form(s, t, seg)
    got = _peak(rdm, ds, k0, P)
    np.testing.assert_allclose(got, want, rtol=REL)
    # and it is the map's maximum of the beam that looks at the target (KAT-4's position)
    b = int(np.argmax(want))
    assert np.unravel_index(np.argmax(np.abs(rdm[:, :, b])), rdm.shape[:2]) == ((k0 + P // 2) % P, ds - 1)


@pytest.mark.gpu
@pytest.mark.parametrize('name,seg', CASES)
def test_device_rdm_peak_value(name, seg):
    from rsp.plan import Plan
    s = scenario(name)
    t, ds, k0 = _kat_target(s, seg)
    cube = chain.synthesize_echo([t], s['cfg'], s['pre_o'])   # the noiseless input (S4 without S4.1)
    plan = Plan(s['cfg'], s['cfar'], s['clus'], s['pre_p'])
    try:
        rdm = plan.process_cube(cube, frame_idx=1, want_rdm=True)['rdm']
    finally:
        plan.close()
    P = s['cfg']['Sig_Config']['prtNum']
    np.testing.assert_allclose(_peak(rdm, ds, k0, P), _closed_form(s, t, seg), rtol=REL)
