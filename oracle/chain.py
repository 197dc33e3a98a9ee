"""Oracle restatement of fun_process_single_frame.m -- TEST INFRASTRUCTURE ONLY.

Every function cites the MATLAB lines it restates.  Arrays keep MATLAB index
order: the echo cube is ``raw[m, n, c]`` ([P x N x C]), beams ``iq[m, n, b]``,
range-Doppler maps ``rdm[v, r, b]``; all indices below are 0-based unless a
comment says "1-based".  Arithmetic is float64 / complex128 like MATLAB.
"""
import numpy as np
import scipy.fft as sfft
import scipy.signal as ss
from scipy.interpolate import CubicSpline

from .philox import unit_normal_complex
from .precompute import mround

EPS = np.finfo(float).eps   # MATLAB eps


def calculate_phase_shifts(angle_deg, d, wl, C):
    """fun_process_single_frame.m:163-169 (channel indices 0:15, generalised to 0:C-1)."""
    dphi = 2 * np.pi * d * np.sin(np.deg2rad(angle_deg)) / wl
    return np.rad2deg(np.arange(C) * dphi)


def synthesize_echo(targets, config, pre):
    """S4, fun_process_single_frame.m:45-78 -> noiseless raw_iq_data[m, n, c]."""
    sc = config['Sig_Config']
    P, N, C = sc['prtNum'], sc['point_PRT'], sc['channel_num']
    ts = 1.0 / sc['fs']
    tx = pre['tx_pulse']
    raw = np.zeros((P, N, C), complex)
    m = np.arange(P)
    for t in targets:
        delay = 2 * t['Range'] / sc['c']
        ds = int(mround(delay / ts))
        fd = 2 * t['Velocity'] / sc['wavelength']
        dop = np.exp(1j * 2 * np.pi * fd * m * sc['prt'])                     # fsf:58 ((m-1) 1-based)
        amp = np.sqrt(10 ** (t['SNR_dB'] / 10) * 1.0 / pre['P_signal_unscaled'])  # fsf:61-63
        base = np.zeros(N, complex)
        if 0 < ds < N:                                                       # fsf:66-69
            ln = min(len(tx), N - ds)
            base[ds:ds + ln] = tx[:ln]
        ph = np.exp(1j * np.deg2rad(calculate_phase_shifts(
            t['ElevationAngle'], config['Array']['element_spacing'], sc['wavelength'], C)))
        raw += (amp * dop)[:, None, None] * base[None, :, None] * ph[None, None, :]
    return raw


def philox_noise(config, frame_idx, seed, p_noise=1.0):
    """S4.1 noise (fsf:80-88) from the documented Philox generator, shaped [P, N, C]."""
    sc = config['Sig_Config']
    P, N, C = sc['prtNum'], sc['point_PRT'], sc['channel_num']
    z = unit_normal_complex(P * N * C, frame_idx, seed) * np.sqrt(p_noise / 2)
    # linear index = m + P*(n + N*c)  (MATLAB column-major [P x N x C])
    return z.reshape(C, N, P).transpose(2, 1, 0)


def dbf(raw, W):
    """S5, fsf:90-97: per pulse [N x C] * W' (conjugate transpose) -> [P, N, B]."""
    return raw @ np.conj(W).T


def pulse_compress(iq, pre):
    """S6, fsf:99-127 -> pc[P, G, B]."""
    P, N, B = iq.shape
    g1, g2, G = pre['N_gate_narrow'], pre['N_gate_medium'], pre['N_total_gate']
    out = np.zeros((P, G, B), complex)
    for b in range(B):
        bd = iq[:, :, b]
        sn = bd[:, pre['seg_start_narrow'] - 1:]
        sm = bd[:, pre['seg_start_medium'] - 1:]
        sl = bd[:, pre['seg_start_long'] - 1:]
        pn = ss.lfilter(pre['MF_narrow'], 1.0, sn, axis=1)                 # fsf:111
        pn = np.roll(pn, -pre['fir_delay'], axis=1)                         # fsf:112
        pm = sfft.ifft(sfft.fft(sm, pre['N_fft_med'], axis=1) * pre['MF_medium_fft'],
                       pre['N_fft_med'], axis=1)                 # fsf:115-116
        pl = sfft.ifft(sfft.fft(sl, pre['N_fft_long'], axis=1) * pre['MF_long_fft'],
                       pre['N_fft_long'], axis=1)                # fsf:119-120
        out[:, :, b] = np.concatenate([pn[:, :g1], pm[:, g1:g1 + g2], pl[:, g1 + g2:G]], axis=1)
    return out


def mtd(pc, pre):
    """S7, fsf:129-136: fftshift(fft(pc .* MTD_win, [], 1), 1)."""
    w = pre['MTD_win'][:, None, None]
    return sfft.fftshift(sfft.fft(pc * w, axis=0), axes=0)


def goca_cfar(rdm, cfar):
    """S8, fun_run_goca_cfar_8 (fsf:172-223), vectorised over CUTs.

    Returns (all_raw_detections [n x 4] with 1-based v, r, pair and the S value,
    rdm_for_cfar_all [P, G, B-1]).  Detection order = pair, then MATLAB find()
    column-major order (r outer, v inner).
    """
    P, G, B = rdm.shape
    T = cfar['T_CFAR']
    gR, gV, rR, rV = cfar['guardCells_R'], cfar['guardCells_V'], cfar['refCells_R'], cfar['refCells_V']
    A = np.abs(rdm)
    S_all = A[:, :, :-1] + A[:, :, 1:]                                       # fsf:184-187
    dets = []
    r0, r1 = rR + gR, G - rR - gR          # 0-based CUT range [r0, r1)  (fsf:192)
    v0, v1 = rV + gV, P - rV - gV          # (fsf:193)
    for p in range(B - 1):
        S = S_all[:, :, p]
        if r1 <= r0 or v1 <= v0:
            continue
        rs = np.arange(r0, r1)
        vs = np.arange(v0, v1)
        # mean() = sum / n, summed left to right like the slice order
        lead_r = sum(S[v0:v1, rs - gR - rR + k] for k in range(rR)) / rR      # fsf:197
        trail_r = sum(S[v0:v1, rs + gR + 1 + k] for k in range(rR)) / rR      # fsf:198
        lead_v = sum(S[vs - gV - rV + k, r0:r1] for k in range(rV)) / rV      # fsf:202
        trail_v = sum(S[vs + gV + 1 + k, r0:r1] for k in range(rV)) / rV      # fsf:203
        noise = np.maximum(np.maximum(lead_r, trail_r), np.maximum(lead_v, trail_v))
        hit = S[v0:v1, r0:r1] > T * noise                                     # fsf:209 strict >
        rr, vv = np.nonzero(hit.T)                                            # find(): column-major
        for ri, vi in zip(rr, vv):
            v, r = vi + v0, ri + r0
            dets.append((v + 1, r + 1, p + 1, S[v, r]))                        # fsf:220 (1-based)
    arr = np.array(dets, float).reshape(-1, 4)
    return arr, S_all


def cfar_margin(rdm, cfar):
    """Relative distance |S - T*noise| / (T*noise) of every CUT (for tolerance bands in tests)."""
    P, G, B = rdm.shape
    T = cfar['T_CFAR']
    gR, gV, rR, rV = cfar['guardCells_R'], cfar['guardCells_V'], cfar['refCells_R'], cfar['refCells_V']
    A = np.abs(rdm)
    S_all = A[:, :, :-1] + A[:, :, 1:]
    r0, r1 = rR + gR, G - rR - gR
    v0, v1 = rV + gV, P - rV - gV
    out = np.full((P, G, B - 1), np.inf)
    if r1 <= r0 or v1 <= v0:
        return out
    rs = np.arange(r0, r1); vs = np.arange(v0, v1)
    for p in range(B - 1):
        S = S_all[:, :, p]
        lead_r = sum(S[v0:v1, rs - gR - rR + k] for k in range(rR)) / rR
        trail_r = sum(S[v0:v1, rs + gR + 1 + k] for k in range(rR)) / rR
        lead_v = sum(S[vs - gV - rV + k, r0:r1] for k in range(rV)) / rV
        trail_v = sum(S[vs + gV + 1 + k, r0:r1] for k in range(rV)) / rV
        thr = T * np.maximum(np.maximum(lead_r, trail_r), np.maximum(lead_v, trail_v))
        out[v0:v1, r0:r1, p] = np.abs(S[v0:v1, r0:r1] - thr) / thr
    return out


def _spline_peak(cells, data, step):
    """interp1(cells-cells(1), data, q-cells(1), 'spline') + first argmax (fsf:257-260)."""
    x = cells - cells[0]
    nq = int(round((cells[-1] - cells[0]) / step)) + 1
    q = cells[0] + np.arange(nq) * step
    if len(cells) == 3:
        # MATLAB spline with 3 points (not-a-knot) is the interpolating parabola
        coef = np.polyfit(x, data, 2)
        val = np.polyval(coef, q - cells[0])
    else:
        val = CubicSpline(x, data, bc_type='not-a-knot')(q - cells[0])
    return q[int(np.argmax(val))]


def parameter_estimation(dets, S_all, rdm, pre, monopulse='amplitude'):
    """S9, fun_parameter_estimation_9 (fsf:226-299).  monopulse='complex': the angle from
    real((S_A - S_B) / (S_A + S_B + eps)) of the complex map, as the inline S9 of
    main_plot_snr_vs_angle_error.m:455-462 does, instead of fsf:282-290's amplitude ratio."""
    out = []
    if dets.shape[0] == 0:
        return out
    P, G = rdm.shape[0], rdm.shape[1]
    extra, rI, vI = 2, 8, 4                                                 # fsf:237
    for v1b, r1b, p1b, power in dets:
        v, r, p = int(v1b), int(r1b), int(p1b)                              # 1-based
        S = S_all[:, :, p - 1]
        rc = np.arange(r - extra, r + extra + 1)
        rc = rc[(rc >= 1) & (rc <= G)]
        rmax = r if len(rc) < 3 else _spline_peak(rc, S[v - 1, rc - 1], 1.0 / rI)
        est_r = pre['range_axis'][r - 1] + (rmax - r) * pre['deltaR']       # fsf:262
        vc = np.arange(v - extra, v + extra + 1)
        vc = vc[(vc >= 1) & (vc <= P)]
        vmax = v if len(vc) < 3 else _spline_peak(vc, S[vc - 1, r - 1], 1.0 / vI)
        est_v = pre['velocity_axis'][v - 1] + (vmax - v) * pre['deltaV']    # fsf:278
        if monopulse == 'complex':                                          # mpsae:455-458
            SA, SB = rdm[v - 1, r - 1, p - 1], rdm[v - 1, r - 1, p]
            ratio = ((SA - SB) / (SA + SB + EPS)).real
        else:
            SA = abs(rdm[v - 1, r - 1, p - 1])                              # fsf:282-283
            SB = abs(rdm[v - 1, r - 1, p])
            ratio = (SA - SB) / (SA + SB + EPS)
        ang = (pre['beam_angles_deg'][p - 1] + pre['beam_angles_deg'][p]) / 2 \
            + pre['k_slopes_LUT'][p - 1] * ratio                             # fsf:285-290
        out.append({'Range': est_r, 'Velocity': est_v, 'Angle': ang, 'Power': power,
                    'PairIndex': p})
    return out


def _bfs_labels(items, close):
    """The BFS labelling loop shared by fsf:310-336 and fsf:363-389."""
    n = len(items)
    ids = [0] * n
    cur = 0
    for i in range(n):
        if ids[i] == 0:
            cur += 1
            queue = [i]
            while queue:
                ci = queue.pop(0)
                if ids[ci] == 0:
                    ids[ci] = cur
                    for j in range(n):
                        if ids[j] == 0 and close(items[ci], items[j]):
                            queue.append(j)
    return ids, cur


def cluster_stage1(dets, cp):
    """S10, fun_cluster_stage1_10 (fsf:302-352): (R,V,A) BFS + power-weighted mean."""
    if not dets:
        return []
    close = lambda a, b: (abs(a['Range'] - b['Range']) <= cp['max_range_sep'] and
                          abs(a['Velocity'] - b['Velocity']) <= cp['max_vel_sep'] and
                          abs(a['Angle'] - b['Angle']) <= cp['max_angle_sep'])
    ids, n = _bfs_labels(dets, close)
    out = []
    for k in range(1, n + 1):
        mem = [d for d, i in zip(dets, ids) if i == k]
        pw = np.array([d['Power'] for d in mem])
        tp = pw.sum()
        out.append({'Range': np.sum(np.array([d['Range'] for d in mem]) * pw) / tp,
                    'Velocity': np.sum(np.array([d['Velocity'] for d in mem]) * pw) / tp,
                    'Angle': np.sum(np.array([d['Angle'] for d in mem]) * pw) / tp,
                    'Power': tp})
    return out


def cluster_stage2(tg, cp):
    """S11, fun_cluster_stage2_11 (fsf:355-407): (R,V) BFS + winner-take-all."""
    if not tg:
        return []
    close = lambda a, b: (abs(a['Range'] - b['Range']) <= cp['max_range_sep'] and
                          abs(a['Velocity'] - b['Velocity']) <= cp['max_vel_sep'])
    ids, n = _bfs_labels(tg, close)
    out = []
    for k in range(1, n + 1):
        mem = [d for d, i in zip(tg, ids) if i == k]
        w = mem[int(np.argmax([d['Power'] for d in mem]))]
        out.append({'Range': w['Range'], 'Velocity': w['Velocity'], 'Angle': w['Angle'],
                    'Power': w['Power']})
    return out


def process_cube(raw_noisy, config, cfar, cluster, pre, keep=False, monopulse='amplitude'):
    """S5..S11 of fsf on a given noisy cube raw[m, n, c]; returns final targets (+ stages)."""
    iq = dbf(raw_noisy, pre['DBF_coeffs_data_C'])
    pc = pulse_compress(iq, pre)
    rdm = mtd(pc, pre)
    dets, S_all = goca_cfar(rdm, cfar)
    par = parameter_estimation(dets, S_all, rdm, pre, monopulse)
    st1 = cluster_stage1(par, cluster)
    fin = cluster_stage2(st1, cluster)
    if keep:
        return fin, dict(iq=iq, pc=pc, rdm=rdm, dets=dets, S_all=S_all, par=par, st1=st1)
    return fin


def fun_process_single_frame(targets, config, cfar, cluster, pre, frame_idx, seed=20250101):
    """fsf:13 signature: synthesis (S4) + Philox noise (S4.1) + S5..S11."""
    raw = synthesize_echo(targets, config, pre) + philox_noise(config, frame_idx, seed)
    return process_cube(raw, config, cfar, cluster, pre)
