"""MUSIC direction finding, restated -- TEST INFRASTRUCTURE ONLY (oracle side).

Restates the two MUSIC scripts of the reference (BASELINE config #5):

* ``MUSIC_1D.m:21-48``            -- real source signals ``Alpha = randn(M, K)``,
  ``awgn(X, SNR, 'measured')``, scan ``linspace(-pi/2, pi/2, 200)``, findpeaks + top M;
* ``run_music_algorithm.m:22-69`` -- complex unit-power sources with amplitudes, fixed
  noise power ``1/10^(SNR/10)``, ``1 / (a' En En' a)`` over a degree grid.

Both share the arithmetic of ``MUSIC_1D.m:28-41``: R = X X^H / K, ``eig`` (Hermitian:
ascending real eigenvalues), stable descending sort, noise subspace = eigenvectors
M+1..N, P(phi) = 1 / sum_j |q_j^H a(phi)|^2, P_dB = 10 log10(P / max P).

MATLAB ``randn`` (and ``awgn``'s internal ``randn``) cannot be reproduced, so the synthetic
snapshots use the documented Philox4x32-10 / Box-Muller stream of ``oracle/philox.py`` with
MUSIC stream tags: source samples draw linear index m + M*k (tag ``TAG_SRC``), noise draws
c + N*k (tag ``TAG_NOISE``), counter word 2 = instance index.  The device synthesis kernel
(``csrc/rsp_music.hip: k_music_synth``) draws the same numbers.

Parity: the reference holds no MUSIC fixtures and MATLAB is absent, so the restatement is
pinned by known answers derivable from the scripts themselves (noise-free subspace nulls at
the source angles, the eigenvalue structure of a rank-M + sigma^2 I covariance, findpeaks
semantics) -- tests/test_music.py.  Beyond those: parity unpinned.
"""
import numpy as np

from .philox import unit_normal_complex

TAG_SRC = 0x4D555341     # 'MUSA'
TAG_NOISE = 0x4D55534E   # 'MUSN'


def steering(n_ch, d_over_lambda, ang_rad):
    """a(phi) = exp(1j k z sin(phi)), z = (0:N-1) d (MUSIC_1D.m:12,21,36; run_music_algorithm.m:27,64)."""
    z = np.arange(n_ch, dtype=np.float64)[:, None]
    return np.exp(1j * 2.0 * np.pi * d_over_lambda * z * np.sin(np.asarray(ang_rad, np.float64))[None, :])


def synthesize(scene, n_ch, K, d_over_lambda, inst, seed):
    """One snapshot matrix X1 [N x K] (MUSIC_1D.m:21-24 / run_music_algorithm.m:27-39).

    scene: angles_rad, amplitudes, complex_sources (0: Alpha = randn(M,K), MUSIC_1D.m:22;
    1: (randn + 1j randn)/sqrt(2) * amplitude, run_music_algorithm.m:30-32), snr_db,
    snr_measured (1: awgn(X, SNR, 'measured'), MUSIC_1D.m:24; 0: noise power 10^(-SNR/10),
    run_music_algorithm.m:35-36).
    """
    ang = np.asarray(scene['angles_rad'], np.float64)
    M = len(ang)
    amp = np.asarray(scene.get('amplitudes', np.ones(M)), np.float64)
    S = steering(n_ch, d_over_lambda, ang)                                      # [N x M]
    z = unit_normal_complex(M * K, inst, seed, tag=TAG_SRC).reshape(K, M).T     # index m + M k
    if scene.get('complex_sources', 0):
        alpha = z / np.sqrt(2.0) * amp[:, None]
    else:
        alpha = z.real * amp[:, None]
    X = S @ alpha
    if scene.get('snr_measured', 1):
        p_sig = np.sum(np.abs(X) ** 2) / X.size                                 # awgn 'measured'
        p_noise = p_sig / 10.0 ** (scene['snr_db'] / 10.0)
    else:
        p_noise = 1.0 / 10.0 ** (scene['snr_db'] / 10.0)
    n = unit_normal_complex(n_ch * K, inst, seed, tag=TAG_NOISE).reshape(K, n_ch).T
    return X + np.sqrt(p_noise / 2.0) * n


def findpeaks(y):
    """Indices (0-based) of MATLAB ``findpeaks(y)`` with no options: local maxima strictly above
    both neighbours; a flat-topped peak reports its first sample; the end samples never qualify
    (the series is bookended by NaN).  Restates the documented behaviour used at MUSIC_1D.m:43."""
    y = np.asarray(y, np.float64)
    n = len(y)
    if n < 3:
        return np.zeros(0, np.int64)
    keep = np.concatenate([[True], y[1:] != y[:-1]])     # first of every run of equal values
    idx = np.nonzero(keep)[0]
    v = y[idx]
    out = []
    for t in range(1, len(idx) - 1):
        if v[t] > v[t - 1] and v[t] > v[t + 1]:
            out.append(idx[t])
    return np.asarray(out, np.int64)


def music_1d(X, M, scan_rad, d_over_lambda):
    """MUSIC_1D.m:28-48 on one snapshot matrix X [N x K] (complex128, like MATLAB)."""
    N, K = X.shape
    R = X @ X.conj().T / K                                   # :28
    R = 0.5 * (R + R.conj().T)                               # herk output is exactly Hermitian
    w, V = np.linalg.eigh(R)                                 # :29 (ascending)
    order = np.argsort(-w, kind='stable')                    # :30-31 sort 'descend'
    Q = V[:, order]                                          # :32
    Qn = Q[:, M:]                                            # :33
    S1 = steering(N, d_over_lambda, scan_rad)                # :35-36
    denom = np.sum(np.abs(Qn.conj().T @ S1) ** 2, axis=0)    # :37
    P = np.abs(1.0 / denom)                                  # :37,39
    PdB = 10.0 * np.log10(P / P.max())                       # :40-41
    pk = findpeaks(PdB)                                      # :43
    srt = np.argsort(-PdB[pk], kind='stable')                # :44-45
    top = pk[srt][:M]                                        # :46-47
    scan = np.asarray(scan_rad, np.float64)
    return {'R': R, 'eig': w[order], 'denom': denom, 'spectrum_db': PdB, 'peaks': top + 1,
            'n_peaks': len(pk), 'angles_deg': scan[top] * 180.0 / np.pi}


def music_batch(Xs, M, scan_rad, d_over_lambda):
    """Vectorised MUSIC_1D.m:28-41 over a stack Xs [I x N x K] (the CPU baseline); findpeaks
    per instance."""
    I, N, K = Xs.shape
    R = np.einsum('ink,imk->inm', Xs, Xs.conj()) / K
    w, V = np.linalg.eigh(R)
    order = np.argsort(-w, axis=1, kind='stable')
    Qn = np.take_along_axis(V, order[:, None, :], axis=2)[:, :, M:]
    S1 = steering(N, d_over_lambda, scan_rad)
    denom = np.sum(np.abs(np.einsum('inj,ns->ijs', Qn.conj(), S1)) ** 2, axis=1)
    P = 1.0 / denom
    PdB = 10.0 * np.log10(P / P.max(axis=1, keepdims=True))
    peaks = []
    for i in range(I):
        pk = findpeaks(PdB[i])
        peaks.append(pk[np.argsort(-PdB[i][pk], kind='stable')][:M] + 1)
    return PdB, peaks


def music_1d_scene():
    """The MUSIC_1D.m:5-35 setup generalised to BASELINE config #5 (64 channels, 1024
    snapshots): d = lambda/2, sources (-10, -30, 60) deg, SNR 10 dB 'measured', 200-point scan."""
    return ({'angles_rad': np.deg2rad([-10.0, -30.0, 60.0]), 'amplitudes': np.ones(3), 'complex_sources': 0,
             'snr_db': 10.0, 'snr_measured': 1},
            np.linspace(-np.pi / 2, np.pi / 2, 200), 0.5)


def run_music_scene():
    """run_music_algorithm.m:7-20,60: 16 channels at 13.8 mm, fc 9.45 GHz, sources 2.0 / -1.5 deg
    with amplitudes 1 / 0.7, 256 snapshots, SNR 15 dB, scan -20:0.1:20 deg."""
    wl = 2.99792458e8 / 9450e6
    scan = np.deg2rad(np.round(np.arange(-200, 201) * 0.1, 10))
    return ({'angles_rad': np.deg2rad([2.0, -1.5]), 'amplitudes': np.array([1.0, 0.7]), 'complex_sources': 1,
             'snr_db': 15.0, 'snr_measured': 0},
            scan, 0.0138 / wl)
