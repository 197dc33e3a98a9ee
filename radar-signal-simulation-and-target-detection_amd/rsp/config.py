"""Configuration structs mirroring the reference drivers.

The reference builds MATLAB structs literally in each driver script
(``main_simulate_echoes_with_array_v8.m:28-70``):  ``config.Sig_Config.*``,
``config.Array.*``, ``cfar_params``, ``cluster_params`` and a ``targets`` struct
array.  Here they are plain dicts with the same field names, so host code reads
like the reference.  ``make_config`` derives ``wavelength`` and ``point_PRT``
exactly as v8:66-69 does.

Named configurations:
  * ``'reference'``  - the v8 reference frame: 16C x 13B x 5819 x 332.
  * ``'plumbing'``   - BASELINE config #1: 8C x 1B x 1024 x 32 (scaled waveform).
  * ``'x2'``         - BASELINE config #2: 16C x 8B x 4096 x 128 (the bench workload).
  * ``'x4'``         - BASELINE config #4: 32C x 16B x 8192 x 256 (synthetic weights).
  * ``'small'``      - a 16C x 4B x 3072 x 64 frame for fast parity tests.
"""
import os
import numpy as np

DATA_DIR = os.path.join(os.path.dirname(__file__), 'data')

# v8:101 -- 35-tap narrow-pulse FIR (integer taps, normalised later by 6/max).
V8_FIR = [794, 1403, 2143, 2672, 2591, 1711, -58, -2351, -4592, -5855, -5338, -2389, 3005,
          10341, 18410, 25779, 30907, 32768, 30907, 25779, 18410, 10341, 3005, -2389, -5338,
          -5855, -4592, -2351, -58, 1711, 2591, 2672, 2143, 1403, 794]
# v8:138 -- measured monopulse slope LUT for the 12 adjacent beam pairs (opaque data).
V8_K_LUT = [-4.6391, -4.6888, -4.7578, -4.7891, -4.7214, -4.7513, -5.2343, -5.4529, -5.7323,
            -6.1685, -7.0256, -8.7612]
# v8:144 -- beam pointing angles of the 13 CSV beams.
V8_BEAM_ANGLES = [-16, -9.6, -3.2, 3.2, 9.6, 16, 22.6, 29.2, 36.1, 43.3, 51, 59.6, 70.3]

C_LIGHT = 2.99792458e8


def load_reference_dbf():
    """13 x 16 complex DBF weights of the reference CSV (v8:148-150), via the repo data file."""
    return np.load(os.path.join(DATA_DIR, 'dbf_coef_13x16.npy'))


def make_config(*, prtNum, point_PRT=None, prt=None, channel_num, beam_num,
                tao=(0.16e-6, 8e-6, 28e-6), gap_duration=(11.4e-6, 31.8e-6, 153.4e-6),
                point_prt_segments=(228, 723, 2453), fs=25e6, fc=9450e6, B=20e6,
                element_spacing=0.0138):
    """Build ``config`` like v8:54-69.  Give either ``prt`` (seconds) or ``point_PRT``."""
    if prt is None:
        prt = point_PRT / fs
    sc = dict(c=C_LIGHT, fs=fs, fc=fc, prtNum=int(prtNum), prt=prt, B=B, tao=list(tao),
              gap_duration=list(gap_duration), point_prt_segments=[int(s) for s in point_prt_segments],
              channel_num=int(channel_num), beam_num=int(beam_num))
    sc['wavelength'] = sc['c'] / sc['fc']
    sc['point_PRT'] = int(np.floor(prt * fs + 0.5))
    return {'Sig_Config': sc, 'Array': {'element_spacing': element_spacing}}


def debug_v3_config():
    """The ``config`` of debug_simulated_data_processing_v3.m:55-106 (the caller of the 3-argument
    process_stage2_mtd at :189), the fields the stage-2 path reads: a Sig_Config with
    point_PRT = 3404 (the gated sample count of the v2 .mat frames), point_prt = [3404 228 723
    2453], no gap_duration, no point_prt_segments and no Array, plus config.mtd.beam_num = 13."""
    sc = dict(c=C_LIGHT, fs=25e6, fc=9450e6, prtNum=332, point_PRT=3404, channel_num=16, beam_num=13,
              prt=232.76e-6, B=20e6, tao=[0.16e-6, 8e-6, 28e-6], point_prt=[3404, 228, 723, 2453])
    sc['prf'] = 1 / sc['prt']
    sc['wavelength'] = sc['c'] / sc['fc']
    sc['deltaR'] = sc['c'] / (2 * sc['fs'])
    mtd = dict(win_size=4, prtNum=sc['prtNum'], beam_num=sc['beam_num'], fs=sc['fs'], fc=sc['fc'], prt=sc['prt'],
               B=sc['B'], tao=list(sc['tao']), point_prt=list(sc['point_prt']))
    return {'Sig_Config': sc, 'mtd': mtd}


def stage2_config(config):
    """A v8-style ``config`` (make_config) for the stage-2 path from any caller's config.

    process_stage2_mtd.m:1 is called from debug_simulated_data_processing_v3.m:189, whose config
    (debug_v3_config) differs from the v8 drivers': point_PRT is the gated count 3404, the segment
    gate counts are point_prt(2:4), and there is no gap_duration or Array.  The full PRT is
    round(prt fs) (v8:68), B is config.mtd.beam_num when present (process_stage2_mtd.m:15),
    the segment gate counts come from point_prt_segments or else point_prt(2:4), and the pulse
    gaps from gap_duration or else the reference waveform's (v8:61: 11.4 / 31.8 / 153.4 us).
    Array.element_spacing is not used by stage 2 (kept when given)."""
    sc = config['Sig_Config']
    fs = float(sc['fs'])
    prt = float(sc['prt']) if 'prt' in sc else float(sc['point_PRT']) / fs
    if 'point_prt_segments' in sc:
        segs = [int(x) for x in sc['point_prt_segments']]
    elif 'point_prt' in sc and len(sc['point_prt']) >= 4:
        segs = [int(x) for x in list(sc['point_prt'])[1:4]]
    else:
        raise KeyError('config.Sig_Config needs point_prt_segments or point_prt = [total narrow medium long]')
    B = int(config.get('mtd', {}).get('beam_num', sc['beam_num']))
    d = config.get('Array', {}).get('element_spacing', 0.0138)
    out = make_config(prtNum=int(sc['prtNum']), prt=prt, channel_num=int(sc.get('channel_num', B)), beam_num=B,
                      tao=tuple(sc['tao']), gap_duration=tuple(sc.get('gap_duration', (11.4e-6, 31.8e-6, 153.4e-6))),
                      point_prt_segments=segs, fs=fs, fc=float(sc['fc']), B=float(sc['B']), element_spacing=d)
    if 'c' in sc:   # the caller's c, as matlab/process_stage2_mtd.m (s.c = sc.c; s.wavelength = s.c / s.fc)
        o = out['Sig_Config']
        o['c'] = float(sc['c'])
        o['wavelength'] = o['c'] / o['fc']
    return out


def default_cfar_params():
    """v8:45-47."""
    return dict(refCells_V=5, guardCells_V=10, refCells_R=5, guardCells_R=10, T_CFAR=8.0, method='GOCA')


def default_cluster_params():
    """v8:49-51."""
    return dict(max_range_sep=30.0, max_vel_sep=0.4, max_angle_sep=5.0)


def steering_weights(angles_deg, C, d, wl, taper=None):
    """Synthetic DBF weights: W[b, c] = t_c exp(j 2 pi d c sin(theta_b) / wl) / sum(t).

    With the kernel's convention y = x * W' (fsf:95) and channel phases
    exp(j c dphi) (fsf:163-169), beam b peaks at theta_b.
    """
    t = np.ones(C) if taper is None else np.asarray(taper, float)
    n = np.arange(C)
    W = np.exp(1j * 2 * np.pi * d * np.outer(np.sin(np.deg2rad(angles_deg)), n) / wl)
    return W * t[None, :] / t.sum()


def calibrate_all_monopulse_slopes(dbf_coeffs_C, beam_angles_deg, fc=9450e6, d=0.0138, c=C_LIGHT):
    """Literal restatement of calibrate_all_monopulse_slopes.m:24-73.

    ``dbf_coeffs_C`` is the B x C complex DBF table as read from the CSV (:24-25); the script
    flips its channel order (:26, ``fliplr``).  For each adjacent pair (:35-72): 501 angles over
    +-|dtheta| around the crossover (:44-47), steering vectors exp(j 2 pi d n sind(theta)/lambda),
    n = 0..C-1 (:50-53), complex responses w * a (no conjugate, :56-57), the complex ratio
    (A-B)/(A+B) (:58), and the slope p(1) of polyfit(real(ratio), angle - crossover, 1) over the
    11 points around the crossover (:63-72).  Returns k_slopes_LUT (1 x B-1).

    On the reference CSV this does NOT give the LUT hard-coded in v8:138 (SURVEY section 4,
    negative KAT: about -2.54 ... -21.49), which is why the reference configs take the LUT as
    input data."""
    W = np.fliplr(np.asarray(dbf_coeffs_C, complex))                          # :26
    B, C = W.shape
    wl = c / fc                                                               # :17
    n = np.arange(C)[:, None]                                                 # :50
    k = np.zeros(B - 1)
    for p in range(B - 1):                                                    # :35
        xo = (beam_angles_deg[p] + beam_angles_deg[p + 1]) / 2                # :44
        wdt = abs(beam_angles_deg[p] - beam_angles_deg[p + 1])                # :46
        ang = np.linspace(xo - wdt, xo + wdt, 501)                            # :47
        sv = np.exp(1j * 2 * np.pi * d * n * np.sin(np.deg2rad(ang))[None, :] / wl)   # :53
        rA, rB = W[p] @ sv, W[p + 1] @ sv                                     # :56-57
        ratio = (rA - rB) / (rA + rB)                                         # :58
        ci = int(np.argmin(np.abs(ang - xo)))                                 # :63
        sl = slice(ci - 5, ci + 6)                                            # :64-68
        k[p] = np.polyfit(np.real(ratio[sl]), ang[sl] - xo, 1)[0]             # :71-72
    return k


def calibrate_k_slopes_amplitude(W, beam_angles_deg, d, wl):
    """NOT the reference's calibration: the amplitude variant used for synthetic-weight configs
    (BASELINE #4).  Same scan and fit as calibrate_all_monopulse_slopes.m:35-73, but with the
    kernel's own beam outputs -- y = x * W' (fsf:95), i.e. responses conj(W) a(theta) -- and the
    amplitude ratio (|A|-|B|)/(|A|+|B|) that the amplitude monopulse of fsf:280-290 forms, so that
    K * ratio maps the kernel's ratio back to the angle offset for these weights."""
    B, C = W.shape
    n = np.arange(C)[:, None]
    k = np.zeros(B - 1)
    for p in range(B - 1):
        a0, a1 = beam_angles_deg[p], beam_angles_deg[p + 1]
        xo = (a0 + a1) / 2
        wdt = abs(a0 - a1)
        ang = np.linspace(xo - wdt, xo + wdt, 501)
        sv = np.exp(1j * 2 * np.pi * d * n * np.sin(np.deg2rad(ang))[None, :] / wl)
        rA = np.abs(np.conj(W[p]) @ sv)
        rB = np.abs(np.conj(W[p + 1]) @ sv)
        ratio = (rA - rB) / (rA + rB)
        ci = int(np.argmin(np.abs(ang - xo)))
        sl = slice(ci - 5, ci + 6)
        k[p] = np.polyfit(ratio[sl], ang[sl] - xo, 1)[0]
    return k


def named_config(name):
    """Return (config, cfar_params, cluster_params, dbf_W, beam_angles, k_lut)."""
    cfar, clus = default_cfar_params(), default_cluster_params()
    if name == 'reference':
        cfg = make_config(prtNum=332, prt=232.76e-6, channel_num=16, beam_num=13)
        W = load_reference_dbf()
        return cfg, cfar, clus, W, list(V8_BEAM_ANGLES), list(V8_K_LUT)
    if name == 'x2':
        cfg = make_config(prtNum=128, point_PRT=4096, channel_num=16, beam_num=8,
                          point_prt_segments=(228, 723, 1860))
        W = load_reference_dbf()[:8]
        return cfg, cfar, clus, W, list(V8_BEAM_ANGLES[:8]), list(V8_K_LUT[:7])
    if name == 'p256':   # test config: P = 256 with 8 beams (persistent K1 at NT = 4, LGP = 8)
        cfg = make_config(prtNum=256, point_PRT=3072, channel_num=16, beam_num=8,
                          point_prt_segments=(228, 723, 836))
        W = load_reference_dbf()[:8]
        return cfg, cfar, clus, W, list(V8_BEAM_ANGLES[:8]), list(V8_K_LUT[:7])
    if name == 'small':
        cfg = make_config(prtNum=64, point_PRT=3072, channel_num=16, beam_num=4,
                          point_prt_segments=(228, 723, 836))
        W = load_reference_dbf()[4:8]
        return cfg, cfar, clus, W, list(V8_BEAM_ANGLES[4:8]), list(V8_K_LUT[4:7])
    if name == 'plumbing':
        cfg = make_config(prtNum=32, point_PRT=1024, channel_num=8, beam_num=1,
                          tao=(0.16e-6, 2e-6, 6e-6), gap_duration=(2.84e-6, 8e-6, 12e-6),
                          point_prt_segments=(64, 192, 256))
        sc = cfg['Sig_Config']
        W = steering_weights([10.0], 8, cfg['Array']['element_spacing'], sc['wavelength'])
        return cfg, cfar, clus, W, [10.0], []
    if name == 'x4':
        import scipy.signal.windows as sw
        cfg = make_config(prtNum=256, point_PRT=8192, channel_num=32, beam_num=16,
                          point_prt_segments=(228, 723, 5956))
        sc = cfg['Sig_Config']
        d, wl = cfg['Array']['element_spacing'], sc['wavelength']
        s = np.linspace(np.sin(np.deg2rad(-48.6)), np.sin(np.deg2rad(48.6)), 16)
        ang = np.rad2deg(np.arcsin(s))
        W = steering_weights(ang, 32, d, wl, taper=sw.taylor(32, nbar=4, sll=30, norm=False))
        k = calibrate_k_slopes_amplitude(W, ang, d, wl)
        return cfg, cfar, clus, W, list(ang), list(k)
    raise KeyError(name)


def v8_2_targets():
    """The five targets of main_simulate_echoes_with_array_v8_2.m:28-51."""
    return [dict(Range=3000.0, Velocity=15.0, ElevationAngle=10.0, SNR_dB=-10.0),
            dict(Range=5000.0, Velocity=20.0, ElevationAngle=5.0, SNR_dB=1.0),
            dict(Range=6500.0, Velocity=10.0, ElevationAngle=15.0, SNR_dB=-20.0),
            dict(Range=8000.0, Velocity=5.0, ElevationAngle=20.0, SNR_dB=5.0),
            dict(Range=10000.0, Velocity=8.0, ElevationAngle=8.0, SNR_dB=15.0)]


def evolve_targets(targets, config):
    """v8:170-173: Range -= Velocity * T_frame (T_frame = prtNum * prt)."""
    sc = config['Sig_Config']
    T = sc['prtNum'] * sc['prt']
    return [dict(t, Range=t['Range'] - t['Velocity'] * T) for t in targets]
