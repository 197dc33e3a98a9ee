"""MUSIC direction finding on the device (MUSIC_1D.m:21-48, run_music_algorithm.m:22-69).

``MusicPlan`` binds the ``rsp_music_*`` C-ABI (include/rsp.h): the scripts' parameters
(N channels, K snapshots, M sources, element spacing / wavelength, scan grid phi_list) make the
plan; ``process`` runs a batch of snapshot matrices X [N x K] through

  R = X X^H / K -> eig, sort descend -> Q_n -> P(phi) = 1/sum|Q_n^H a(phi)|^2 -> P_dB -> findpeaks

and returns what the scripts compute: ``P_MUSIC_dB``, the sorted eigenvalues ``EVA``, the M
peak indices / angles ``phi_e`` (MUSIC_1D.m:48).  ``MUSIC_1D(X, ...)`` is the one-instance
form of MUSIC_1D.m.  ``precision``: 'c128' (complex double, MATLAB's arithmetic; default) or
'c64' (complex single).  All compute runs in librsp.so; there is no CPU path.
"""
import ctypes as ct

import numpy as np

from . import _abi


class MusicPlan:
    def __init__(self, channel_num, num_snapshots, num_sources, scan_rad, d_over_lambda=0.5, max_batch=1,
                 device=0, precision='c128'):
        if precision not in ('c128', 'c64'):
            raise ValueError("precision must be 'c128' or 'c64'")
        self._lib = _abi.lib()
        self.precision = precision
        self.cdtype = np.complex128 if precision == 'c128' else np.complex64   # device snapshots
        self.scan_rad = np.ascontiguousarray(scan_rad, np.float64)
        self.N, self.K, self.M, self.S = int(channel_num), int(num_snapshots), int(num_sources), len(self.scan_rad)
        self.max_batch = int(max_batch)
        cfg = _abi.MusicConfig(self.N, self.K, self.M, self.S, float(d_over_lambda),
                               self.scan_rad.ctypes.data_as(_abi._dp), self.max_batch,
                               _abi.RSP_C128 if precision == 'c128' else _abi.RSP_C64)
        h = ct.c_void_p()
        _abi.check(self._lib.rsp_music_create(ct.byref(cfg), int(device), ct.byref(h)))
        self._h = h

    def close(self):
        if getattr(self, '_h', None):
            self._lib.rsp_music_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- outputs -------------------------------------------------------------------------
    def _out(self, n, want_cov, want_eig=True):
        o = {'spectrum_db': np.zeros((n, self.S), np.float64), 'peaks': np.zeros((n, self.M), np.int32),
             'n_peaks': np.zeros(n, np.int32)}
        if want_eig:
            o['eig'] = np.zeros((n, self.N), np.float64)
        if want_cov:
            o['R'] = np.zeros((n, self.N, self.N, 2), np.float64)   # per instance: [b][a] = R(a, b)
        st = _abi.MusicOut(o['spectrum_db'].ctypes.data_as(_abi._dp),
                           o['eig'].ctypes.data_as(_abi._dp) if want_eig else None,
                           o['peaks'].ctypes.data_as(ct.POINTER(ct.c_int32)),
                           o['n_peaks'].ctypes.data_as(ct.POINTER(ct.c_int32)),
                           o['R'].ctypes.data_as(_abi._dp) if want_cov else None)
        return o, st

    def _finish(self, o):
        if 'R' in o:
            r = o.pop('R')
            o['R'] = np.ascontiguousarray(np.transpose(r[..., 0] + 1j * r[..., 1], (0, 2, 1)))
        pk = o['peaks']
        o['angles_deg'] = np.where(pk > 0, self.scan_rad[np.maximum(pk - 1, 0)] * 180.0 / np.pi, np.nan)
        return o

    def process(self, X, want_cov=False, want_eig=True):
        """X: complex [n, N, K] (or [N, K]) host snapshots -> dict of per-instance outputs.
        ``want_eig=False``: the eigenvalues are not read (no 'eig' key), so complex double finds
        only the M signal eigenvalues (the spectrum is still the full eigensolver's)."""
        X = np.asarray(X)
        if X.ndim == 2:
            X = X[None]
        n = X.shape[0]
        if X.shape[1:] != (self.N, self.K):
            raise ValueError('X must be [n, %d, %d], got %s' % (self.N, self.K, X.shape))
        # MATLAB column-major N x K per instance == C-order [n][K][N]
        if X.dtype == np.complex64:
            buf, dt = np.ascontiguousarray(np.transpose(X, (0, 2, 1))), _abi.RSP_C64
        else:
            buf, dt = np.ascontiguousarray(np.transpose(X.astype(np.complex128), (0, 2, 1))), _abi.RSP_C128
        o, st = self._out(n, want_cov, want_eig)
        _abi.check(self._lib.rsp_music_process(self._h, buf.ctypes.data, dt, n, ct.byref(st)))
        return self._finish(o)

    def peaks(self, X):
        """rsp_music_process on host snapshots with only the peaks requested (the eigenvalues not
        read): (peak indices [n, M] 1-based, findpeaks counts [n])."""
        X = np.asarray(X)
        if X.ndim == 2:
            X = X[None]
        n = X.shape[0]
        buf = np.ascontiguousarray(np.transpose(X.astype(np.complex128 if self.cdtype == np.complex128 else np.complex64),
                                                (0, 2, 1)))
        pk = np.zeros((n, self.M), np.int32)
        npk = np.zeros(n, np.int32)
        st = _abi.MusicOut(None, None, pk.ctypes.data_as(ct.POINTER(ct.c_int32)),
                           npk.ctypes.data_as(ct.POINTER(ct.c_int32)), None)
        dt = _abi.RSP_C128 if buf.dtype == np.complex128 else _abi.RSP_C64
        _abi.check(self._lib.rsp_music_process(self._h, buf.ctypes.data, dt, n, ct.byref(st)))
        return pk, npk

    # ---- device-resident path (bench) ------------------------------------------------------
    def device_alloc(self, n_inst):
        p = ct.c_void_p()
        _abi.check(self._lib.rsp_music_device_alloc(self._h, n_inst * self.N * self.K * np.dtype(self.cdtype).itemsize,
                                                    ct.byref(p)))
        return p.value

    def device_free(self, p):
        _abi.check(self._lib.rsp_music_device_free(self._h, ct.c_void_p(p)))

    def download(self, d_X, n_inst):
        h = np.zeros((n_inst, self.K, self.N), self.cdtype)
        _abi.check(self._lib.rsp_music_device_download(self._h, h.ctypes.data, ct.c_void_p(d_X), h.nbytes))
        return np.ascontiguousarray(np.transpose(h, (0, 2, 1)))

    def synthesize_device(self, d_X, scene, n_inst, inst0=0, seed=20250101):
        ang = list(scene['angles_rad'])
        amp = list(scene.get('amplitudes', [1.0] * len(ang)))
        sc = _abi.MusicScene(len(ang), int(scene.get('complex_sources', 0)), int(scene.get('snr_measured', 1)), 0,
                             float(scene['snr_db']), (ct.c_double * 8)(*ang), (ct.c_double * 8)(*amp))
        _abi.check(self._lib.rsp_music_synthesize_device(self._h, ct.byref(sc), n_inst, inst0, ct.c_uint64(seed),
                                                         ct.c_void_p(d_X)))

    def process_device(self, d_X, n_inst, fetch=True, want_cov=False):
        if not fetch:
            _abi.check(self._lib.rsp_music_process_device(self._h, ct.c_void_p(d_X), n_inst, None))
            return None
        o, st = self._out(n_inst, want_cov)
        _abi.check(self._lib.rsp_music_process_device(self._h, ct.c_void_p(d_X), n_inst, ct.byref(st)))
        return self._finish(o)

    def peaks_device(self, d_X, n_inst, peaks, n_peaks):
        """Device run returning only the peak indices (into caller arrays): the bench's step."""
        st = _abi.MusicOut(None, None, peaks.ctypes.data_as(ct.POINTER(ct.c_int32)),
                           n_peaks.ctypes.data_as(ct.POINTER(ct.c_int32)), None)
        _abi.check(self._lib.rsp_music_process_device(self._h, ct.c_void_p(d_X), n_inst, ct.byref(st)))

    def eig_device(self, d_X, n_inst, eig, peaks, n_peaks):
        """Device run returning all N eigenvalues (descending, MUSIC_1D.m:29-33) and the peak indices
        into caller arrays: the form of the 3-output rsp_mex('music') / music_1d_calllib.m call,
        which always runs the full eigensolver (bench.py --want-eig)."""
        st = _abi.MusicOut(None, eig.ctypes.data_as(_abi._dp), peaks.ctypes.data_as(ct.POINTER(ct.c_int32)),
                           n_peaks.ctypes.data_as(ct.POINTER(ct.c_int32)), None)
        _abi.check(self._lib.rsp_music_process_device(self._h, ct.c_void_p(d_X), n_inst, ct.byref(st)))

    def spectrum_device(self, d_X, n_inst, spec, peaks, n_peaks):
        """Device run returning the pseudo-spectrum P_dB ([n_inst, n_scan], MUSIC_1D.m:41) and the peak
        indices into caller arrays, without the eigenvalues: the form of the 2-output rsp_mex('music')
        call and of MUSIC_1D.m's plot (bench.py --want-spectrum)."""
        st = _abi.MusicOut(spec.ctypes.data_as(_abi._dp), None, peaks.ctypes.data_as(ct.POINTER(ct.c_int32)),
                           n_peaks.ctypes.data_as(ct.POINTER(ct.c_int32)), None)
        _abi.check(self._lib.rsp_music_process_device(self._h, ct.c_void_p(d_X), n_inst, ct.byref(st)))

    def fast_count(self):
        """Instances of the last call answered by the block-power fast path (rsp_music_fast_count)."""
        n = ct.c_int32()
        _abi.check(self._lib.rsp_music_fast_count(self._h, ct.byref(n)))
        return n.value

    def profile(self, d_X, n_inst, iters=20, what='peaks'):
        """HIP-event times of the two stages for the form of call ``what``: 'peaks' (the bench's
        step), 'spectrum' (spectrum_db read) or 'eigenvalues' (all N eigenvalues read)."""
        forms = {'peaks': _abi.RSP_MUSIC_PEAKS, 'spectrum': _abi.RSP_MUSIC_SPECTRUM,
                 'eigenvalues': _abi.RSP_MUSIC_EIGENVALUES}
        ms = (ct.c_float * 2)()
        _abi.check(self._lib.rsp_music_profile_ex(self._h, ct.c_void_p(d_X), n_inst, iters, forms[what], ms))
        return {'cov_ms': ms[0], 'eig_ms': ms[1]}


def music_1d_scene():
    """MUSIC_1D.m:5-35 scene at BASELINE config #5 (64 channels, 1024 snapshots): d = lambda/2,
    real sources at (-10, -30, 60) deg, awgn 10 dB 'measured', 200-point scan over +-90 deg.
    Returns (scene dict for MusicPlan.synthesize_device, scan grid [rad], d/lambda)."""
    return ({'angles_rad': np.deg2rad([-10.0, -30.0, 60.0]), 'amplitudes': np.ones(3), 'complex_sources': 0,
             'snr_db': 10.0, 'snr_measured': 1},
            np.linspace(-np.pi / 2, np.pi / 2, 200), 0.5)


def run_music_scene():
    """run_music_algorithm.m:7-20,60: 16 channels at 13.8 mm, fc 9.45 GHz, complex sources at
    2.0 / -1.5 deg with amplitudes 1 / 0.7, SNR 15 dB (fixed noise power), scan -20:0.1:20 deg."""
    wl = 2.99792458e8 / 9450e6
    return ({'angles_rad': np.deg2rad([2.0, -1.5]), 'amplitudes': np.array([1.0, 0.7]), 'complex_sources': 1,
             'snr_db': 15.0, 'snr_measured': 0},
            np.deg2rad(np.round(np.arange(-200, 201) * 0.1, 10)), 0.0138 / wl)


def MUSIC_1D(X1, M, phi_list=None, d_over_lambda=0.5, device=0, precision='c128'):
    """MUSIC_1D.m:26-48 on one snapshot matrix X1 [N x K]: returns (phi_e [deg], P_MUSIC_dB, EVA)."""
    X1 = np.asarray(X1)
    if phi_list is None:
        phi_list = np.linspace(-np.pi / 2, np.pi / 2, 200)   # MUSIC_1D.m:35
    plan = MusicPlan(X1.shape[0], X1.shape[1], M, phi_list, d_over_lambda, max_batch=1, device=device,
                     precision=precision)
    try:
        o = plan.process(X1)
    finally:
        plan.close()
    return o['angles_deg'][0], o['spectrum_db'][0], o['eig'][0]
