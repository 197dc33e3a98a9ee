"""ctypes binding of include/rsp.h (librsp.so).

This is the Python equivalent of the MEX / ``loadlibrary`` shim the MATLAB
reference would bind.  The library is built in-tree by
``csrc/Makefile`` into ``rsp/librsp.so``; importing this module does not touch
the GPU.  There is no CPU fallback: if the library is missing, ``lib()`` raises.
"""
import ctypes as ct
import os

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'librsp.so')
_INTREE = LIB_PATH

RSP_OK, RSP_ERR_INVALID, RSP_ERR_UNSUPPORTED, RSP_ERR_DEVICE, RSP_ERR_NOMEM, RSP_ERR_OVERFLOW = 0, -1, -2, -3, -4, -5
RSP_C64, RSP_C128 = 1, 2
RSP_LAYOUT_PNC = 0

_dp = ct.POINTER(ct.c_double)


class SigConfig(ct.Structure):
    _fields_ = [('c', ct.c_double), ('fs', ct.c_double), ('fc', ct.c_double), ('prt', ct.c_double),
                ('wavelength', ct.c_double), ('element_spacing', ct.c_double),
                ('prtNum', ct.c_int32), ('point_PRT', ct.c_int32), ('channel_num', ct.c_int32),
                ('beam_num', ct.c_int32)]


class CfarParams(ct.Structure):
    _fields_ = [('refCells_V', ct.c_int32), ('guardCells_V', ct.c_int32), ('refCells_R', ct.c_int32),
                ('guardCells_R', ct.c_int32), ('T_CFAR', ct.c_double)]


class ClusterParams(ct.Structure):
    _fields_ = [('max_range_sep', ct.c_double), ('max_vel_sep', ct.c_double), ('max_angle_sep', ct.c_double)]


class Precomputed(ct.Structure):
    _fields_ = [('tx_pulse', _dp), ('P_signal_unscaled', ct.c_double), ('DBF_coeffs_data_C', _dp),
                ('MF_narrow', _dp), ('n_MF_narrow', ct.c_int32), ('fir_delay', ct.c_int32),
                ('MF_medium_fft', _dp), ('N_fft_med', ct.c_int32), ('MF_long_fft', _dp), ('N_fft_long', ct.c_int32),
                ('N_gate_narrow', ct.c_int32), ('N_gate_medium', ct.c_int32), ('N_gate_long', ct.c_int32),
                ('N_total_gate', ct.c_int32), ('seg_start_narrow', ct.c_int32), ('seg_start_medium', ct.c_int32),
                ('seg_start_long', ct.c_int32), ('MTD_win', _dp), ('range_axis', _dp), ('velocity_axis', _dp),
                ('deltaR', ct.c_double), ('deltaV', ct.c_double), ('beam_angles_deg', _dp), ('k_slopes_LUT', _dp)]


class TargetIn(ct.Structure):
    _fields_ = [('Range', ct.c_double), ('Velocity', ct.c_double), ('ElevationAngle', ct.c_double),
                ('SNR_dB', ct.c_double)]


class Target(ct.Structure):
    _fields_ = [('Range', ct.c_double), ('Velocity', ct.c_double), ('Angle', ct.c_double), ('Power', ct.c_double)]


class Detection(ct.Structure):
    _fields_ = [('v_idx', ct.c_int32), ('r_idx', ct.c_int32), ('pair_idx', ct.c_int32), ('reserved', ct.c_int32),
                ('amp', ct.c_double), ('Range', ct.c_double), ('Velocity', ct.c_double), ('Angle', ct.c_double)]


class FrameOut(ct.Structure):
    _fields_ = [('rdm', _dp), ('cfar_maps', _dp), ('dets', ct.POINTER(Detection)), ('dets_cap', ct.c_int32),
                ('n_dets', ct.c_int32), ('targets', ct.POINTER(Target)), ('targets_cap', ct.c_int32),
                ('n_targets', ct.c_int32)]


class Sizes(ct.Structure):
    _fields_ = [('cube_elems', ct.c_int64), ('rdm_elems', ct.c_int64), ('cfar_map_elems', ct.c_int64),
                ('P', ct.c_int32), ('N', ct.c_int32), ('C', ct.c_int32), ('B', ct.c_int32), ('G', ct.c_int32),
                ('used_samples', ct.c_int32), ('max_detections', ct.c_int32), ('n_stages', ct.c_int32),
                ('precision', ct.c_int32), ('elem_bytes', ct.c_int32)]


RSP_PLAN_K1_TILED = 1
RSP_PLAN_MONOPULSE_COMPLEX = 2


class PlanOptions(ct.Structure):
    _fields_ = [('device', ct.c_int32), ('frames_per_launch', ct.c_int32), ('precision', ct.c_int32),
                ('flags', ct.c_int32)]


RSP_MUSIC_PEAKS, RSP_MUSIC_SPECTRUM, RSP_MUSIC_EIGENVALUES = 0, 1, 2   # rsp_music_profile_ex

RSP_MAT_CHAR, RSP_MAT_DOUBLE, RSP_MAT_SINGLE = 4, 6, 7
RSP_MAT_OUT_F64, RSP_MAT_OUT_F32, RSP_MAT_OUT_CHAR = 1, 2, 3
RSP_MAT_MAXDIMS = 8


class MatVar(ct.Structure):
    _fields_ = [('name', ct.c_char * 64), ('cls', ct.c_int32), ('is_complex', ct.c_int32), ('ndims', ct.c_int32),
                ('reserved', ct.c_int32), ('dims', ct.c_int64 * RSP_MAT_MAXDIMS), ('numel', ct.c_int64)]


class MatWVar(ct.Structure):
    _fields_ = [('name', ct.c_char_p), ('cls', ct.c_int32), ('is_complex', ct.c_int32), ('ndims', ct.c_int32),
                ('dims', ct.POINTER(ct.c_int64)), ('data', ct.c_void_p)]


class TrackPoint(ct.Structure):
    _fields_ = [('Range', ct.c_double), ('Velocity', ct.c_double), ('Angle', ct.c_double), ('Power', ct.c_double),
                ('iAntAngle', ct.c_double), ('iFrame', ct.c_int32), ('reserved', ct.c_int32)]


class InterFrameParams(ct.Structure):
    _fields_ = [('Gate_R', ct.c_double), ('Gate_V', ct.c_double), ('Gate_Az', ct.c_double), ('Gate_El', ct.c_double),
                ('Max_Frame_Gap', ct.c_int32), ('reserved', ct.c_int32)]


class Track(ct.Structure):
    _fields_ = [('Range', ct.c_double), ('Velocity', ct.c_double), ('Angle', ct.c_double), ('Azimuth', ct.c_double),
                ('Power', ct.c_double), ('FirstFrame', ct.c_int32), ('LastFrame', ct.c_int32),
                ('NumPoints', ct.c_int32), ('reserved', ct.c_int32)]


class MusicConfig(ct.Structure):
    _fields_ = [('channel_num', ct.c_int32), ('num_snapshots', ct.c_int32), ('num_sources', ct.c_int32),
                ('n_scan', ct.c_int32), ('d_over_lambda', ct.c_double), ('scan_rad', _dp), ('max_batch', ct.c_int32),
                ('precision', ct.c_int32)]


class MusicScene(ct.Structure):
    _fields_ = [('n_src', ct.c_int32), ('complex_sources', ct.c_int32), ('snr_measured', ct.c_int32),
                ('reserved', ct.c_int32), ('snr_db', ct.c_double), ('angles_rad', ct.c_double * 8),
                ('amplitudes', ct.c_double * 8)]


class MusicOut(ct.Structure):
    _fields_ = [('spectrum_db', _dp), ('eigenvalues', _dp),
                ('peak_idx', ct.POINTER(ct.c_int32)), ('n_peaks', ct.POINTER(ct.c_int32)), ('covariance', _dp)]


_P = ct.c_void_p
PROTOTYPES = {
    'rsp_abi_version': (ct.c_int32, []),
    'rsp_last_error': (ct.c_char_p, []),
    'rsp_plan_create': (ct.c_int32, [ct.POINTER(SigConfig), ct.POINTER(CfarParams), ct.POINTER(ClusterParams),
                                     ct.POINTER(Precomputed), ct.c_int32, ct.c_int32, ct.POINTER(_P)]),
    'rsp_plan_create_ex': (ct.c_int32, [ct.POINTER(SigConfig), ct.POINTER(CfarParams), ct.POINTER(ClusterParams),
                                        ct.POINTER(Precomputed), ct.POINTER(PlanOptions), ct.POINTER(_P)]),
    'rsp_plan_options_default': (ct.c_int32, [ct.POINTER(PlanOptions)]),
    'rsp_plan_destroy': (ct.c_int32, [_P]),
    'rsp_query_sizes': (ct.c_int32, [_P, ct.POINTER(Sizes)]),
    'rsp_process_cube': (ct.c_int32, [_P, _P, ct.c_int32, ct.c_int32, ct.c_int32, ct.POINTER(FrameOut)]),
    'rsp_process_targets': (ct.c_int32, [_P, ct.POINTER(TargetIn), ct.c_int32, ct.c_int32, ct.c_uint64,
                                         ct.c_double, ct.POINTER(FrameOut)]),
    'rsp_synthesize_device': (ct.c_int32, [_P, ct.POINTER(TargetIn), ct.c_int32, ct.c_int32, ct.c_uint64,
                                           ct.c_double, _P]),
    'rsp_profile_synthesis': (ct.c_int32, [_P, ct.POINTER(TargetIn), ct.c_int32, ct.c_int32, _P,
                                           ct.POINTER(ct.c_float), ct.POINTER(ct.c_int64)]),
    'rsp_enqueue_device': (ct.c_int32, [_P, _P, ct.c_int32]),
    'rsp_enqueue_device_n': (ct.c_int32, [_P, ct.POINTER(_P), ct.POINTER(ct.c_int32), ct.c_int32]),
    'rsp_enqueue_device_rdm': (ct.c_int32, [_P, _P, ct.c_int32, _P]),
    'rsp_enqueue_device_rdm_n': (ct.c_int32, [_P, ct.POINTER(_P), ct.POINTER(ct.c_int32), ct.POINTER(_P), ct.c_int32]),
    'rsp_enqueue_host': (ct.c_int32, [_P, _P, ct.c_int32, ct.c_int32]),
    'rsp_host_alloc': (ct.c_int32, [_P, ct.c_int64, ct.POINTER(_P)]),
    'rsp_host_free': (ct.c_int32, [_P, _P]),
    'rsp_process_targets_multi': (ct.c_int32, [ct.POINTER(_P), ct.c_int32, ct.POINTER(ct.POINTER(TargetIn)),
                                               ct.POINTER(ct.c_int32), ct.POINTER(ct.c_int32), ct.c_int32, ct.c_uint64,
                                               ct.c_double, ct.POINTER(Target), ct.c_int32, ct.POINTER(ct.c_int32)]),
    'rsp_drain': (ct.c_int32, [_P]),
    'rsp_last_detections': (ct.c_int32, [_P, ct.POINTER(Detection), ct.c_int32, ct.POINTER(ct.c_int32)]),
    'rsp_last_targets': (ct.c_int32, [_P, ct.POINTER(Target), ct.c_int32, ct.POINTER(ct.c_int32)]),
    'rsp_results_count': (ct.c_int32, [_P, ct.POINTER(ct.c_int32), ct.POINTER(ct.c_int64)]),
    'rsp_results_get': (ct.c_int32, [_P, ct.c_int32, ct.POINTER(ct.c_int32), ct.POINTER(Target), ct.c_int32,
                                     ct.POINTER(ct.c_int32), ct.POINTER(ct.c_int32)]),
    'rsp_results_clear': (ct.c_int32, [_P]),
    'rsp_results_rows': (ct.c_int32, [_P, _dp, ct.c_int64, ct.POINTER(ct.c_int64)]),
    'rsp_process_stage2': (ct.c_int32, [_P, _P, ct.c_int32, _dp, _dp]),
    'rsp_process_stage2_gated': (ct.c_int32, [_P, _P, ct.c_int32, ct.c_int32, ct.POINTER(ct.c_int32), _dp, _dp]),
    'rsp_profile_stages': (ct.c_int32, [_P, ct.POINTER(_P), ct.c_int32, ct.c_int32, ct.POINTER(ct.c_float),
                                        ct.POINTER(ct.c_int64), ct.c_int32, ct.POINTER(ct.c_int32)]),
    'rsp_profile_stages_rdm': (ct.c_int32, [_P, ct.POINTER(_P), ct.c_int32, ct.POINTER(_P), ct.c_int32,
                                            ct.POINTER(ct.c_float), ct.POINTER(ct.c_int64), ct.c_int32,
                                            ct.POINTER(ct.c_int32)]),
    'rsp_stage_name': (ct.c_char_p, [ct.c_int32]),
    'rsp_hbm_copy_probe': (ct.c_int32, [ct.c_int32, ct.c_int64, ct.c_int32, ct.POINTER(ct.c_double)]),
    'rsp_set_stage_timing': (ct.c_int32, [_P, ct.c_int32]),
    'rsp_stage_times': (ct.c_int32, [_P, ct.POINTER(ct.c_double), ct.c_int32, ct.POINTER(ct.c_int64),
                                     ct.POINTER(ct.c_int64)]),
    'rsp_cluster_detections': (ct.c_int32, [ct.POINTER(Detection), ct.c_int32, ct.POINTER(ClusterParams),
                                            ct.POINTER(Target), ct.c_int32, ct.POINTER(ct.c_int32)]),
    'rsp_device_alloc': (ct.c_int32, [_P, ct.c_int64, ct.POINTER(_P)]),
    'rsp_device_free': (ct.c_int32, [_P, _P]),
    'rsp_device_upload': (ct.c_int32, [_P, _P, _P, ct.c_int64]),
    'rsp_device_download': (ct.c_int32, [_P, _P, _P, ct.c_int64]),
    'rsp_device_sync': (ct.c_int32, [_P]),
    'rsp_mat_list': (ct.c_int32, [ct.c_char_p, ct.POINTER(MatVar), ct.c_int32, ct.POINTER(ct.c_int32)]),
    'rsp_mat_read': (ct.c_int32, [ct.c_char_p, ct.c_char_p, ct.c_int32, _P, ct.c_int64]),
    'rsp_mat_write': (ct.c_int32, [ct.c_char_p, ct.POINTER(MatWVar), ct.c_int32, ct.c_int32]),
    'rsp_mat_load_frame': (ct.c_int32, [ct.c_char_p, ct.c_int32, _P, ct.c_int64, ct.POINTER(ct.c_int32), _dp,
                                        ct.c_int32, ct.POINTER(ct.c_int32)]),
    'rsp_mat_save_frame': (ct.c_int32, [ct.c_char_p, _dp, ct.c_int32, ct.c_int32, ct.c_int32, _dp, ct.c_int32,
                                        ct.c_int32, ct.c_int32]),
    'rsp_inter_frame_cluster': (ct.c_int32, [ct.POINTER(TrackPoint), ct.c_int32, ct.POINTER(InterFrameParams),
                                             ct.POINTER(Track), ct.c_int32, ct.POINTER(ct.c_int32)]),
    'rsp_music_create': (ct.c_int32, [ct.POINTER(MusicConfig), ct.c_int32, ct.POINTER(_P)]),
    'rsp_music_destroy': (ct.c_int32, [_P]),
    'rsp_music_process': (ct.c_int32, [_P, _P, ct.c_int32, ct.c_int32, ct.POINTER(MusicOut)]),
    'rsp_music_process_device': (ct.c_int32, [_P, _P, ct.c_int32, ct.POINTER(MusicOut)]),
    'rsp_music_synthesize_device': (ct.c_int32, [_P, ct.POINTER(MusicScene), ct.c_int32, ct.c_int32, ct.c_uint64, _P]),
    'rsp_music_profile': (ct.c_int32, [_P, _P, ct.c_int32, ct.c_int32, ct.POINTER(ct.c_float)]),
    'rsp_music_profile_ex': (ct.c_int32, [_P, _P, ct.c_int32, ct.c_int32, ct.c_int32, ct.POINTER(ct.c_float)]),
    'rsp_music_fast_count': (ct.c_int32, [_P, ct.POINTER(ct.c_int32)]),
    'rsp_music_device_alloc': (ct.c_int32, [_P, ct.c_int64, ct.POINTER(_P)]),
    'rsp_music_device_free': (ct.c_int32, [_P, _P]),
    'rsp_music_device_download': (ct.c_int32, [_P, _P, _P, ct.c_int64]),
}

_lib = None


class RspError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__('rsp error %d: %s' % (code, msg))
        self.code = code


def lib():
    """Load librsp.so (raises if it was not built: there is no fallback path)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError('librsp.so not found at %s -- build it with __graft_entry__.build() '
                               'or `make -C csrc`' % LIB_PATH)
        h = ct.CDLL(LIB_PATH)
        for name, (res, args) in PROTOTYPES.items():
            if LIB_PATH != _INTREE and not hasattr(h, name):
                continue   # an A/B timing variant built from an older revision (tools/ab/): bind what it has
            fn = getattr(h, name)
            fn.restype = res
            fn.argtypes = args
        _lib = h
    return _lib


def check(rc):
    if rc != RSP_OK:
        raise RspError(rc, lib().rsp_last_error().decode(errors='replace'))
    return rc
