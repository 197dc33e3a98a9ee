"""Host-side plan object over the C-ABI (include/rsp.h).

Arrays use MATLAB index order (the reference's), stored column-major so they are
passed to the library exactly as a MEX gateway would pass mxArray data:
echo cube ``[P, N, C]``, range-Doppler maps ``[P, G, B]``, CFAR maps
``[P, G, B-1]``.
"""
import ctypes as ct
import numpy as np

from . import _abi
from ._abi import check, lib


def _dptr(a):
    return a.ctypes.data_as(ct.POINTER(ct.c_double))


def _det_dict(d):
    return {'v_idx': d.v_idx, 'r_idx': d.r_idx, 'pair_idx': d.pair_idx, 'amp': d.amp,
            'Range': d.Range, 'Velocity': d.Velocity, 'Angle': d.Angle}


def _tgt_dict(t):
    return {'Range': t.Range, 'Velocity': t.Velocity, 'Angle': t.Angle, 'Power': t.Power}


class Plan:
    """One device plan = the reference's per-frame kernel bound to fixed config/precompute.

    Parameters mirror ``fun_process_single_frame(targets, config, cfar_params,
    cluster_params, precomputed_data, frame_idx)`` (fun_process_single_frame.m:13).
    ``precision``: 'c128' (complex double, MATLAB's arithmetic; default) or 'c64'.
    ``k1_tiled``: force the one-tile-per-workgroup K1 (parity tests compare it with the
    persistent K1 the plan otherwise picks).
    ``monopulse``: 'amplitude' (fsf:282-290, the default) or 'complex' -- S9's angle from
    real((S_A - S_B) / (S_A + S_B + eps)) of the complex map, the estimator of the inline S9 in
    main_plot_snr_vs_angle_error.m:455-462 (RSP_PLAN_MONOPULSE_COMPLEX).
    """

    def __init__(self, config, cfar_params, cluster_params, precomputed_data, device=0, frames_per_launch=1,
                 precision='c128', k1_tiled=False, monopulse='amplitude'):
        sc = config['Sig_Config']
        pre = precomputed_data
        self.config = config
        self._keep = []

        def arr(x, cplx=False):
            a = np.ascontiguousarray(np.asarray(x, np.complex128 if cplx else np.float64))
            if cplx:
                a = a.view(np.float64)
            self._keep.append(a)
            return _dptr(a)

        self.cfg = _abi.SigConfig(c=sc['c'], fs=sc['fs'], fc=sc['fc'], prt=sc['prt'], wavelength=sc['wavelength'],
                                  element_spacing=config['Array']['element_spacing'], prtNum=sc['prtNum'],
                                  point_PRT=sc['point_PRT'], channel_num=sc['channel_num'], beam_num=sc['beam_num'])
        self.cfar = _abi.CfarParams(refCells_V=cfar_params['refCells_V'], guardCells_V=cfar_params['guardCells_V'],
                                    refCells_R=cfar_params['refCells_R'], guardCells_R=cfar_params['guardCells_R'],
                                    T_CFAR=cfar_params['T_CFAR'])
        self.cluster = _abi.ClusterParams(max_range_sep=cluster_params['max_range_sep'],
                                          max_vel_sep=cluster_params['max_vel_sep'],
                                          max_angle_sep=cluster_params['max_angle_sep'])
        W = np.asarray(pre['DBF_coeffs_data_C'], np.complex128)
        Wcm = np.asfortranarray(W).ravel(order='F')      # B x C column-major (MATLAB)
        klut = np.asarray(pre['k_slopes_LUT'], float)
        self.pre = _abi.Precomputed(
            tx_pulse=arr(pre['tx_pulse'], True) if 'tx_pulse' in pre else None,
            P_signal_unscaled=pre.get('P_signal_unscaled', 0.0),
            DBF_coeffs_data_C=arr(Wcm, True), MF_narrow=arr(pre['MF_narrow']), n_MF_narrow=len(pre['MF_narrow']),
            fir_delay=int(pre['fir_delay']), MF_medium_fft=arr(pre['MF_medium_fft'], True),
            N_fft_med=int(pre['N_fft_med']), MF_long_fft=arr(pre['MF_long_fft'], True),
            N_fft_long=int(pre['N_fft_long']), N_gate_narrow=int(pre['N_gate_narrow']),
            N_gate_medium=int(pre['N_gate_medium']), N_gate_long=int(pre['N_gate_long']),
            N_total_gate=int(pre['N_total_gate']), seg_start_narrow=int(pre['seg_start_narrow']),
            seg_start_medium=int(pre['seg_start_medium']), seg_start_long=int(pre['seg_start_long']),
            MTD_win=arr(pre['MTD_win']), range_axis=arr(pre['range_axis']), velocity_axis=arr(pre['velocity_axis']),
            deltaR=float(pre['deltaR']), deltaV=float(pre['deltaV']), beam_angles_deg=arr(pre['beam_angles_deg']),
            k_slopes_LUT=arr(klut if klut.size else np.zeros(1)))
        if precision not in ('c128', 'c64'):
            raise ValueError("precision must be 'c128' or 'c64'")
        opt = _abi.PlanOptions()
        check(lib().rsp_plan_options_default(ct.byref(opt)))
        opt.device, opt.frames_per_launch = int(device), int(frames_per_launch)
        opt.precision = _abi.RSP_C128 if precision == 'c128' else _abi.RSP_C64
        if monopulse not in ('amplitude', 'complex'):
            raise ValueError("monopulse must be 'amplitude' (fsf:282-290) or 'complex' "
                             "(main_plot_snr_vs_angle_error.m:455-462), got %r" % (monopulse,))
        opt.flags = (_abi.RSP_PLAN_K1_TILED if k1_tiled else 0) | \
            (_abi.RSP_PLAN_MONOPULSE_COMPLEX if monopulse == 'complex' else 0)
        h = ct.c_void_p()
        check(lib().rsp_plan_create_ex(ct.byref(self.cfg), ct.byref(self.cfar), ct.byref(self.cluster),
                                       ct.byref(self.pre), ct.byref(opt), ct.byref(h)))
        self.h = h
        s = _abi.Sizes()
        check(lib().rsp_query_sizes(self.h, ct.byref(s)))
        self.sizes = s
        self.P, self.N, self.C, self.B, self.G = s.P, s.N, s.C, s.B, s.G
        self.precision = precision
        self.frames_per_launch = int(frames_per_launch)   # F: frames per kernel launch (1..RSP_MAX_F)
        self.cdtype = np.complex128 if precision == 'c128' else np.complex64   # device cube / map element
        self.cube_bytes = s.cube_elems * s.elem_bytes

    def close(self):
        if getattr(self, 'h', None):
            lib().rsp_plan_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- synchronous frame paths ---------------------------------------------------------
    def _frame_out(self, want_rdm, want_cfar):
        o = _abi.FrameOut()
        bufs = {}
        if want_rdm:
            bufs['rdm'] = np.empty((self.P, self.G, self.B), np.complex128, order='F')
            o.rdm = bufs['rdm'].ctypes.data_as(ct.POINTER(ct.c_double))
        if want_cfar and self.B > 1:
            bufs['cfar'] = np.empty((self.P, self.G, self.B - 1), np.float64, order='F')
            o.cfar_maps = _dptr(bufs['cfar'])
        # detections and final targets have no fixed count: read after the frame (rsp_last_*)
        o.dets, o.dets_cap, o.targets, o.targets_cap = None, 0, None, 0
        return o, bufs, None, None

    def last_detections(self):
        """Every detection of the last synchronous frame (rsp_last_detections; no capacity limit)."""
        n = ct.c_int32()
        check(lib().rsp_last_detections(self.h, None, 0, ct.byref(n)))
        dets = (_abi.Detection * max(n.value, 1))()
        check(lib().rsp_last_detections(self.h, dets, n.value, ct.byref(n)))
        return [_det_dict(dets[i]) for i in range(n.value)]

    def last_targets(self):
        """The final targets of the last synchronous frame (rsp_last_targets)."""
        n = ct.c_int32()
        check(lib().rsp_last_targets(self.h, None, 0, ct.byref(n)))
        tg = (_abi.Target * max(n.value, 1))()
        check(lib().rsp_last_targets(self.h, tg, n.value, ct.byref(n)))
        return [_tgt_dict(tg[i]) for i in range(n.value)]

    def _collect(self, o, bufs, dets, tg):
        res = {'final_targets': self.last_targets(), 'detections': self.last_detections()}
        assert len(res['detections']) == o.n_dets and len(res['final_targets']) == o.n_targets
        if 'rdm' in bufs:
            res['rdm'] = bufs['rdm']
        if 'cfar' in bufs:
            res['cfar_maps'] = bufs['cfar']
        return res

    def process_cube(self, cube, frame_idx=1, want_rdm=False, want_cfar=False):
        """S5..S11 on a noisy echo cube ``cube[m, n, c]`` (MATLAB [P x N x C]).  ``cfar_maps``
        (want_cfar) is rdm_for_cfar_all as the device's K3 thresholds it (fsf:184-187)."""
        cube = np.asarray(cube)
        if cube.shape != (self.P, self.N, self.C):
            raise ValueError('cube shape %r != (P, N, C) = %r' % (cube.shape, (self.P, self.N, self.C)))
        if cube.dtype == np.complex64:
            a, dt = np.asfortranarray(cube), _abi.RSP_C64
        else:
            a, dt = np.asfortranarray(cube, np.complex128), _abi.RSP_C128
        o, bufs, dets, tg = self._frame_out(want_rdm, want_cfar)
        check(lib().rsp_process_cube(self.h, a.ctypes.data_as(ct.c_void_p), dt, _abi.RSP_LAYOUT_PNC,
                                     int(frame_idx), ct.byref(o)))
        return self._collect(o, bufs, dets, tg)

    def process_targets(self, targets, frame_idx=1, seed=20250101, p_noise=1.0, want_rdm=False, want_cfar=False):
        """fsf:13 path: device S4 synthesis + S4.1 Philox noise + S5..S11."""
        tin = self._targets_in(targets)
        o, bufs, dets, tg = self._frame_out(want_rdm, want_cfar)
        check(lib().rsp_process_targets(self.h, tin, len(targets), int(frame_idx), int(seed), float(p_noise),
                                        ct.byref(o)))
        return self._collect(o, bufs, dets, tg)

    @staticmethod
    def _targets_in(targets):
        arr = (_abi.TargetIn * max(len(targets), 1))()
        for i, t in enumerate(targets):
            arr[i] = _abi.TargetIn(t['Range'], t['Velocity'], t['ElevationAngle'], t['SNR_dB'])
        return arr

    def process_stage2(self, iq_beams, gate_cols=None):
        """process_stage2_mtd backing: beams ``iq[m, n, b]`` -> (MTD [P,G,B], PC [P,G,B]).
        ``gate_cols``: ((first, last), ...) 1-based PRT columns of the segments of a gated
        input (rsp_process_stage2_gated); None: ``n`` is the full PRT."""
        iq = np.asarray(iq_beams)
        if iq.dtype == np.complex64:
            a, dt = np.asfortranarray(iq), _abi.RSP_C64
        else:
            a, dt = np.asfortranarray(iq, np.complex128), _abi.RSP_C128
        mtd = np.empty((self.P, self.G, self.B), np.complex128, order='F')
        pc = np.empty((self.P, self.G, self.B), np.complex128, order='F')
        mo, po = mtd.ctypes.data_as(ct.POINTER(ct.c_double)), pc.ctypes.data_as(ct.POINTER(ct.c_double))
        if gate_cols is None:
            if iq.shape != (self.P, self.N, self.B):
                raise ValueError('iq shape %r != (P, N, B) = %r' % (iq.shape, (self.P, self.N, self.B)))
            check(lib().rsp_process_stage2(self.h, a.ctypes.data_as(ct.c_void_p), dt, mo, po))
        else:
            cols = (ct.c_int32 * 6)(*[int(x) for fl in gate_cols for x in fl])
            if iq.shape[0] != self.P or iq.shape[2] != self.B:
                raise ValueError('iq shape %r: expected (P, n, B) with P=%d B=%d' % (iq.shape, self.P, self.B))
            check(lib().rsp_process_stage2_gated(self.h, a.ctypes.data_as(ct.c_void_p), dt, iq.shape[1], cols, mo, po))
        return mtd, pc

    # ---- device-resident queue -------------------------------------------------------------
    def device_alloc(self, nbytes):
        p = ct.c_void_p()
        check(lib().rsp_device_alloc(self.h, int(nbytes), ct.byref(p)))
        return p.value

    def device_free(self, ptr):
        check(lib().rsp_device_free(self.h, ct.c_void_p(ptr)))

    def device_upload(self, ptr, host):
        host = np.ascontiguousarray(host)
        check(lib().rsp_device_upload(self.h, ct.c_void_p(ptr), host.ctypes.data_as(ct.c_void_p), host.nbytes))

    def device_download(self, ptr, count, dtype):
        out = np.empty(int(count), dtype)
        check(lib().rsp_device_download(self.h, out.ctypes.data_as(ct.c_void_p), ct.c_void_p(ptr), out.nbytes))
        return out

    def upload_cube(self, ptr, cube):
        """Upload a [P, N, C] cube column-major, in the plan's precision, to device pointer ``ptr``."""
        a = np.asfortranarray(np.asarray(cube).astype(self.cdtype))
        check(lib().rsp_device_upload(self.h, ct.c_void_p(ptr), a.ctypes.data_as(ct.c_void_p), a.nbytes))

    def synthesize_device(self, ptr, targets, frame_idx, seed=20250101, p_noise=1.0):
        tin = self._targets_in(targets)
        check(lib().rsp_synthesize_device(self.h, tin, len(targets), int(frame_idx), int(seed), float(p_noise),
                                          ct.c_void_p(ptr)))

    def profile_synthesis(self, ptr, targets, iters=20):
        """rsp_profile_synthesis: device ms of one S4 + S4.1 synthesis into ``ptr`` (HIP events
        over ``iters`` launches) and the cube bytes it writes."""
        tin = self._targets_in(targets)
        ms, by = ct.c_float(), ct.c_int64()
        check(lib().rsp_profile_synthesis(self.h, tin, len(targets), int(iters), ct.c_void_p(ptr), ct.byref(ms),
                                          ct.byref(by)))
        return {'stage': 'k_synth', 'ms': float(ms.value), 'bytes': int(by.value), 'frames': 1}

    def enqueue(self, ptr, frame_idx):
        check(lib().rsp_enqueue_device(self.h, ct.c_void_p(ptr), int(frame_idx)))

    def enqueue_many(self, ptrs, frame_ids, rdms=None):
        """rsp_enqueue_device_n: device cubes ptrs[i] as frames frame_ids[i], one C call.  With
        ``rdms`` (device pointers, one per frame, rdm_elems complex elements each) every frame's
        complex RD map is written there (rsp_enqueue_device_rdm_n), complete after drain()."""
        n = len(ptrs)
        arr = (ct.c_void_p * max(n, 1))(*ptrs)
        ids = (ct.c_int32 * max(n, 1))(*[int(f) for f in frame_ids])
        if rdms is None:
            check(lib().rsp_enqueue_device_n(self.h, arr, ids, n))
        else:
            if len(rdms) != n:
                raise ValueError('one RD map per frame')
            ra = (ct.c_void_p * max(n, 1))(*rdms)
            check(lib().rsp_enqueue_device_rdm_n(self.h, arr, ids, ra, n))

    def rdm_from_device(self, ptr):
        """A device RD map ([B][P][G], plan precision, as rsp_enqueue_device_rdm writes it) as the
        MATLAB-shaped [P, G, B] complex array of rdm_13beam (fsf:135)."""
        sz = self.sizes
        m = self.device_download(ptr, sz.rdm_elems, self.cdtype).reshape(sz.B, sz.P, sz.G)
        return np.transpose(m, (1, 2, 0))

    def host_alloc(self, nbytes):
        """Pinned host memory (rsp_host_alloc); returns the address."""
        p = ct.c_void_p()
        check(lib().rsp_host_alloc(self.h, int(nbytes), ct.byref(p)))
        return p.value

    def host_free(self, ptr):
        check(lib().rsp_host_free(self.h, ct.c_void_p(ptr)))

    def host_cube(self, ptr):
        """A numpy [P, N, C] view (column-major, plan precision) of host memory at ``ptr``."""
        P, N, C = self.P, self.N, self.sizes.C
        buf = (ct.c_char * (P * N * C * np.dtype(self.cdtype).itemsize)).from_address(ptr)
        return np.ndarray((P, N, C), self.cdtype, buffer=buf, order='F')

    def enqueue_host(self, ptr_or_cube, frame_idx):
        """rsp_enqueue_host: a host cube (address, or a Fortran-ordered array in the plan's
        precision) that must stay unchanged until drain()."""
        if isinstance(ptr_or_cube, np.ndarray):
            a = ptr_or_cube
            if a.dtype != np.dtype(self.cdtype) or not a.flags.f_contiguous:
                raise ValueError('enqueue_host needs a Fortran-ordered %s cube' % np.dtype(self.cdtype))
            ptr = a.ctypes.data
        else:
            ptr = ptr_or_cube
        dt = _abi.RSP_C128 if np.dtype(self.cdtype) == np.complex128 else _abi.RSP_C64
        check(lib().rsp_enqueue_host(self.h, ct.c_void_p(ptr), dt, int(frame_idx)))

    def drain(self):
        check(lib().rsp_drain(self.h))

    def sync(self):
        check(lib().rsp_device_sync(self.h))

    def results(self, clear=True):
        nf, nt = ct.c_int32(), ct.c_int64()
        check(lib().rsp_results_count(self.h, ct.byref(nf), ct.byref(nt)))
        out = []
        cap = 4096
        buf = (_abi.Target * cap)()
        for i in range(nf.value):
            fi, n, nd = ct.c_int32(), ct.c_int32(), ct.c_int32()
            check(lib().rsp_results_get(self.h, i, ct.byref(fi), None, 0, ct.byref(n), ct.byref(nd)))
            if n.value > cap:
                cap = n.value
                buf = (_abi.Target * cap)()
            check(lib().rsp_results_get(self.h, i, ct.byref(fi), buf, cap, ct.byref(n), ct.byref(nd)))
            out.append({'frame_idx': fi.value, 'n_dets': nd.value,
                        'final_targets': [_tgt_dict(buf[j]) for j in range(n.value)]})
        if clear:
            check(lib().rsp_results_clear(self.h))
        return out

    def results_rows(self, clear=True):
        """The queued results as an [n, 5] float64 array (frame_idx, Range, Velocity, Angle,
        Power; one NaN row per frame without targets) in one C call (rsp_results_rows)."""
        n = ct.c_int64()
        check(lib().rsp_results_rows(self.h, None, 0, ct.byref(n)))
        rows = np.empty((max(n.value, 1), 5), np.float64)
        check(lib().rsp_results_rows(self.h, rows.ctypes.data_as(ct.POINTER(ct.c_double)), n.value, ct.byref(n)))
        if clear:
            check(lib().rsp_results_clear(self.h))
        return rows[:n.value]

    def set_stage_timing(self, on=True):
        """Live HIP-event timing of K1/K2/K3 of every queued batch (resets the sums)."""
        check(lib().rsp_set_stage_timing(self.h, 1 if on else 0))

    def stage_times(self):
        """Sums of the live stage timing: [{'stage', 'ms_total', 'launches', 'frames'}]."""
        n = self.sizes.n_stages
        ms = (ct.c_double * n)()
        nl, nf = ct.c_int64(), ct.c_int64()
        check(lib().rsp_stage_times(self.h, ms, n, ct.byref(nl), ct.byref(nf)))
        return [{'stage': lib().rsp_stage_name(i).decode(), 'ms_total': ms[i], 'launches': nl.value,
                 'frames': nf.value} for i in range(n)]

    def profile_stages(self, d_cubes, iters=20, d_rdms=None):
        """Per-stage HIP-event timing; d_cubes = device pointer or list of pointers (batched).
        d_rdms: K2 also writes each frame's complex RD map there (rsp_profile_stages_rdm)."""
        if not isinstance(d_cubes, (list, tuple)):
            d_cubes = [d_cubes]
        n = self.sizes.n_stages
        ms = (ct.c_float * n)()
        by = (ct.c_int64 * n)()
        arr = (ct.c_void_p * len(d_cubes))(*d_cubes)
        nf = ct.c_int32()
        if d_rdms:   # the C call reads min(len(d_cubes), F) maps: a shorter list would be read past its end
            need = min(len(d_cubes), self.frames_per_launch)
            if len(d_rdms) < need or any(r is None or not int(r) for r in d_rdms[:need]):
                raise ValueError('d_rdms needs %d non-null device maps (one per frame of the batch)' % need)
        ra = (ct.c_void_p * len(d_rdms))(*d_rdms) if d_rdms else None
        check(lib().rsp_profile_stages_rdm(self.h, arr, len(d_cubes), ra, int(iters), ms, by, n, ct.byref(nf)))
        return [{'stage': lib().rsp_stage_name(i).decode(), 'ms': ms[i], 'bytes': by[i], 'frames': nf.value}
                for i in range(n)]


def process_targets_multi(plans, frames, seed=20250101, p_noise=1.0, cap=1024):
    """rsp_process_targets_multi: frames = [(targets, frame_idx), ...] split over ``plans`` (one
    host thread each, typically one plan per device); returns the final targets of every frame,
    in order."""
    n = len(frames)
    tins = [Plan._targets_in(t) for t, _ in frames]
    tptr = (ct.POINTER(_abi.TargetIn) * max(n, 1))(*[ct.cast(t, ct.POINTER(_abi.TargetIn)) for t in tins])
    nt = (ct.c_int32 * max(n, 1))(*[len(t) for t, _ in frames])
    fi = (ct.c_int32 * max(n, 1))(*[int(f) for _, f in frames])
    out = (_abi.Target * (max(n, 1) * cap))()
    nout = (ct.c_int32 * max(n, 1))()
    ph = (ct.c_void_p * len(plans))(*[p.h for p in plans])
    check(lib().rsp_process_targets_multi(ph, len(plans), tptr, nt, fi, n, int(seed), float(p_noise), out, cap, nout))
    return [[_tgt_dict(out[j * cap + i]) for i in range(nout[j])] for j in range(n)]
