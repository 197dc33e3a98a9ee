"""MAT-file I/O of the reference's frames, through librsp's native
Level-5 reader/writer (csrc/rsp_mat.cpp; no scipy, no MATLAB).

Mirrors the MATLAB calls of the reference:

* ``save(output_filename, 'raw_iq_data_noise_sample', 'servo_angle')``
  (main_simulate_echoes_with_array_v2.m:285; v1 saves ``raw_iq_data``,
  main_simulate_echoes_with_array.m:229)  ->  :func:`save_frame` / :func:`save`
* ``sim_data = load(sim_data_path); raw_iq_data = sim_data.raw_iq_data_noise_sample;
  angle = sim_data.servo_angle;`` (debug_simulated_data_processing_v3.m:20-22)
  ->  :func:`load_frame` / :func:`load`
* ``whos -file``  ->  :func:`whos`

Arrays are numpy arrays with MATLAB's shape in Fortran order (``cube[m, n, c]`` is
MATLAB's ``raw_iq_data(m+1, n+1, c+1)``).  Host-only: no GPU is touched.
"""
import ctypes as ct

import numpy as np

from . import _abi
from ._abi import lib, check

_CLASS_DTYPE = {_abi.RSP_MAT_DOUBLE: np.float64, _abi.RSP_MAT_SINGLE: np.float32}


def _b(path):
    return str(path).encode()


def whos(path):
    """List the variables of a MAT file: [{'name', 'class', 'complex', 'size'}] (``whos -file``)."""
    n = ct.c_int32()
    check(lib().rsp_mat_list(_b(path), None, 0, ct.byref(n)))
    arr = (_abi.MatVar * max(n.value, 1))()
    check(lib().rsp_mat_list(_b(path), arr, n.value, ct.byref(n)))
    out = []
    for v in arr[:n.value]:
        out.append({'name': v.name.decode(), 'class': int(v.cls), 'complex': bool(v.is_complex),
                    'size': tuple(int(d) for d in v.dims[:v.ndims])})
    return out


def load(path, *names):
    """``S = load(path, names...)`` as a dict of numpy arrays (numeric -> float64 / complex128 in
    MATLAB shape, char -> str).  Variables of other classes (cell, struct, sparse) raise."""
    info = {v['name']: v for v in whos(path)}
    names = names or tuple(info)
    out = {}
    for nm in names:
        if nm not in info:
            raise KeyError('%s has no variable %r' % (path, nm))
        v = info[nm]
        if v['class'] == _abi.RSP_MAT_CHAR:
            cap = 4 * int(np.prod(v['size'])) + 1
            buf = ct.create_string_buffer(cap)
            check(lib().rsp_mat_read(_b(path), nm.encode(), _abi.RSP_MAT_OUT_CHAR, ct.cast(buf, ct.c_void_p), cap))
            out[nm] = buf.value.decode()
            continue
        a = np.empty(v['size'], np.complex128 if v['complex'] else np.float64, order='F')
        check(lib().rsp_mat_read(_b(path), nm.encode(), _abi.RSP_MAT_OUT_F64, a.ctypes.data_as(ct.c_void_p),
                                 a.size * (2 if v['complex'] else 1)))
        out[nm] = a
    return out


def save(path, compress=True, **variables):
    """``save(path, names...)``: numeric arrays as double (or single for float32 /
    complex64 input), str as char rows.  1-D arrays are saved as 1 x n rows like MATLAB
    row vectors; scalars as 1 x 1."""
    keep, wv = [], (_abi.MatWVar * max(len(variables), 1))()
    for i, (nm, val) in enumerate(variables.items()):
        if isinstance(val, str):
            data = np.frombuffer(val.encode('latin-1'), np.uint8)
            dims, cls, cplx = (1, data.size), _abi.RSP_MAT_CHAR, 0
        else:
            a = np.asarray(val)
            if a.ndim < 2:
                a = a.reshape(1, -1)
            single = a.dtype in (np.float32, np.complex64)
            cplx = int(np.iscomplexobj(a))
            dt = (np.complex64 if single else np.complex128) if cplx else (np.float32 if single else np.float64)
            data = np.asfortranarray(a, dt)
            dims, cls = a.shape, (_abi.RSP_MAT_SINGLE if single else _abi.RSP_MAT_DOUBLE)
        d = (ct.c_int64 * len(dims))(*dims)
        keep += [data, d]
        wv[i] = _abi.MatWVar(nm.encode(), cls, cplx, len(dims), d, data.ctypes.data_as(ct.c_void_p))
    check(lib().rsp_mat_write(_b(path), wv, len(variables), 1 if compress else 0))


def load_frame(path, dtype=np.complex128):
    """Frame loader of debug_simulated_data_processing_v3.m:20-22: returns ``(raw_iq_data,
    servo_angle)``, the cube [P x N x C] (``raw_iq_data_noise_sample``, else ``raw_iq_data``)
    and the servo angles (None if the file has none).  One pass over the file; complex64
    output halves host memory for the device path."""
    c64 = np.dtype(dtype) == np.complex64
    dims = (ct.c_int32 * 3)()
    na = ct.c_int32()
    check(lib().rsp_mat_load_frame(_b(path), _abi.RSP_C64 if c64 else _abi.RSP_C128, None, 0, dims, None, 0,
                                   ct.byref(na)))
    cube = np.empty(tuple(dims), np.complex64 if c64 else np.complex128, order='F')
    ang = np.empty(max(na.value, 1), np.float64)
    check(lib().rsp_mat_load_frame(_b(path), _abi.RSP_C64 if c64 else _abi.RSP_C128,
                                   cube.ctypes.data_as(ct.c_void_p), cube.size, dims,
                                   ang.ctypes.data_as(ct.POINTER(ct.c_double)), ang.size, ct.byref(na)))
    return cube, (ang[:na.value] if na.value else None)


def save_frame(path, cube, servo_angle=None, generation=2, compress=True):
    """``save(frame_sim_array_%d.mat, ...)`` of main_simulate_echoes_with_array_v2.m:285
    (generation 2: ``raw_iq_data_noise_sample``) or main_simulate_echoes_with_array.m:229
    (generation 1: ``raw_iq_data``)."""
    a = np.asfortranarray(cube, np.complex128)
    if a.ndim != 3:
        raise ValueError('cube must be [P x N x C]')
    P, N, C = a.shape
    ang = None if servo_angle is None else np.ascontiguousarray(servo_angle, np.float64).ravel()
    check(lib().rsp_mat_save_frame(_b(path), a.ctypes.data_as(ct.POINTER(ct.c_double)), P, N, C,
                                   None if ang is None else ang.ctypes.data_as(ct.POINTER(ct.c_double)),
                                   0 if ang is None else ang.size, int(generation), 1 if compress else 0))
