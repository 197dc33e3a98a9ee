"""MAT-file frame I/O: librsp's native Level-5 reader/writer
(csrc/rsp_mat.cpp) through rsp.matio.

CPU (no GPU): the two MATLAB-written files the reference holds (tests/golden/ref_mat/, R2025
PCWIN64, compressed, UTF-16 char data) decode to the values scipy.io.loadmat gives; files
written by scipy (compressed and plain, every numeric class, complex, N-D, char, empty) read
back exactly; files written by librsp load exactly in scipy; a hand-built big-endian file
reads; frame save/load of both generations' variable names
(main_simulate_echoes_with_array.m:229 `raw_iq_data`, _v2.m:285 `raw_iq_data_noise_sample`
+ `servo_angle`) round-trips bit-exactly; malformed inputs return status codes.
GPU: a frame saved to .mat and loaded back drives rsp_process_cube to the same result as
the in-memory cube, and the stage-2 flow of debug_simulated_data_processing_v3.m
(load -> per-pulse DBF -> process_stage2_mtd) matches the oracle.
"""
import json
import os
import struct

import numpy as np
import pytest
import scipy.io as sio

from rsp import matio
from rsp._abi import RspError

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.path.join(HERE, 'golden', 'ref_mat')


@pytest.mark.parametrize('fn', ['FIR.mat', 'file.mat'])
def test_reads_matlab_written_reference_files(fn):
    exp = json.load(open(os.path.join(REF, 'expected.json'), encoding='utf-8'))[fn]
    path = os.path.join(REF, fn)
    listed = {v['name']: v for v in matio.whos(path)}
    assert set(listed) == set(exp)
    got = matio.load(path)
    for k, e in exp.items():
        if e['class'] == 'char':
            assert got[k] == e['value']
        else:
            assert list(got[k].shape) == e['size']
            assert np.array_equal(got[k].ravel(order='F'), np.array(e['value']))


def _vars(rng):
    return {'a': rng.standard_normal((3, 4, 5)),
            'c': rng.standard_normal((6, 7, 2)) + 1j * rng.standard_normal((6, 7, 2)),
            'i8': np.arange(-5, 5, dtype=np.int8).reshape(2, 5),
            'u16': np.arange(12, dtype=np.uint16).reshape(3, 4),
            'i64': np.array([[-(2 ** 40), 7]], np.int64),
            'f32': rng.standard_normal((4, 4)).astype(np.float32),
            'c64': (rng.standard_normal((2, 3)) + 1j).astype(np.complex64),
            's': 'frame_sim_array_1.mat',
            'sc': np.array([[3.5]]),
            'ints': np.array([[1.0, 2.0, 300.0]]),   # MATLAB/scipy may shrink storage of such doubles
            'empty': np.zeros((0, 3))}


@pytest.mark.parametrize('compress', [False, True])
def test_reads_scipy_written_files(tmp_path, compress):
    v = _vars(np.random.default_rng(1))
    f = str(tmp_path / 'x.mat')
    sio.savemat(f, v, do_compression=compress)
    info = {w['name']: w for w in matio.whos(f)}
    assert info['c']['complex'] and info['c']['size'] == (6, 7, 2)
    got = matio.load(f)
    for k, val in v.items():
        if isinstance(val, str):
            assert got[k] == val
        else:
            assert got[k].shape == val.shape, k
            assert np.array_equal(got[k], val.astype(got[k].dtype)), k


@pytest.mark.parametrize('compress', [False, True])
def test_written_files_load_in_scipy(tmp_path, compress):
    v = {k: x for k, x in _vars(np.random.default_rng(2)).items() if k not in ('i8', 'u16', 'i64')}
    f = str(tmp_path / 'y.mat')
    matio.save(f, compress=compress, **v)
    r = sio.loadmat(f)
    for k, val in v.items():
        if isinstance(val, str):
            assert r[k][0] == val
        else:
            assert r[k].dtype == val.dtype and np.array_equal(r[k], val), k
    back = matio.load(f)
    assert np.array_equal(back['c'], v['c'])


def _be_element(name, arr):
    """A plain (uncompressed) big-endian miMATRIX element of a real double matrix."""
    def sub(t, payload):
        pad = (-len(payload)) % 8
        return struct.pack('>II', t, len(payload)) + payload + b'\0' * pad
    body = sub(6, struct.pack('>II', 6, 0))                           # flags: mxDOUBLE_CLASS
    body += sub(5, struct.pack('>%di' % arr.ndim, *arr.shape))       # dims
    body += sub(1, name.encode())
    body += sub(9, arr.ravel(order='F').astype('>f8').tobytes())    # miDOUBLE
    return struct.pack('>II', 14, len(body)) + body


def test_reads_big_endian_file(tmp_path):
    a = np.arange(12, dtype=np.float64).reshape(3, 4) - 5.25
    hdr = b'MATLAB 5.0 MAT-file, big-endian test'.ljust(116, b' ') + b'\0' * 8 + b'\x01\x00' + b'MI'
    f = tmp_path / 'be.mat'
    f.write_bytes(hdr + _be_element('servo_angle', a) + _be_element('z', a.T.copy()))
    got = matio.load(str(f))
    assert np.array_equal(got['servo_angle'], a) and np.array_equal(got['z'], a.T)
    assert np.array_equal(sio.loadmat(str(f))['servo_angle'], a)


@pytest.mark.parametrize('generation,compress', [(1, True), (2, True), (2, False)])
def test_frame_round_trip(tmp_path, generation, compress):
    rng = np.random.default_rng(generation)
    P, N, C = 16, 300, 8
    cube = rng.standard_normal((P, N, C)) + 1j * rng.standard_normal((P, N, C))
    ang = rng.uniform(-180, 180, P)
    f = str(tmp_path / 'frame_sim_array_1.mat')
    matio.save_frame(f, cube, ang, generation=generation, compress=compress)
    names = [w['name'] for w in matio.whos(f)]
    assert names == [('raw_iq_data_noise_sample' if generation == 2 else 'raw_iq_data'), 'servo_angle']
    c2, a2 = matio.load_frame(f)
    assert c2.shape == (P, N, C) and np.array_equal(c2, cube) and np.array_equal(a2, ang)
    c3, _ = matio.load_frame(f, dtype=np.complex64)
    assert c3.dtype == np.complex64 and np.array_equal(c3, cube.astype(np.complex64))
    # MATLAB's load of the same file (scipy as the independent reader)
    r = sio.loadmat(f)
    key = 'raw_iq_data_noise_sample' if generation == 2 else 'raw_iq_data'
    assert np.array_equal(r[key], cube) and np.array_equal(r['servo_angle'].ravel(), ang)


def test_frame_from_scipy_real_cube_without_angle(tmp_path):
    cube = np.arange(2 * 5 * 3, dtype=np.float64).reshape(2, 5, 3)
    f = str(tmp_path / 'f.mat')
    sio.savemat(f, {'raw_iq_data': cube}, do_compression=True)
    c, a = matio.load_frame(f)
    assert a is None and np.array_equal(c, cube.astype(np.complex128))


def test_errors(tmp_path):
    with pytest.raises(RspError):
        matio.whos(str(tmp_path / 'missing.mat'))
    h5 = tmp_path / 'v73.mat'   # MATLAB -v7.3 header (HDF5 user block)
    h5.write_bytes(b'MATLAB 7.3 MAT-file'.ljust(116, b' ') + b'\0' * 8 + b'\x00\x02IM' + b'\0' * 64)
    with pytest.raises(RspError, match='v7.3'):
        matio.whos(str(h5))
    f = str(tmp_path / 'a.mat')
    sio.savemat(f, {'q': np.ones((2, 2)), 'cell': np.array([[1, 'x']], dtype=object)})
    with pytest.raises(KeyError):
        matio.load(f, 'nope')
    with pytest.raises(RspError, match='class'):
        matio.load(f, 'cell')
    with pytest.raises(RspError, match='neither'):
        matio.load_frame(f)
    trunc = tmp_path / 't.mat'
    sio.savemat(str(trunc), {'big': np.ones((50, 50))}, do_compression=False)
    trunc.write_bytes(trunc.read_bytes()[:1000])
    with pytest.raises(RspError):
        matio.load(str(trunc), 'big')


@pytest.mark.gpu
def test_frame_mat_drives_device_chain(tmp_path):
    from rsp.plan import Plan
    from _scen import scenario, targets_for, noisy_cube
    s = scenario('small')
    cube = noisy_cube(s, targets_for('small'), dtype=np.complex128)
    f = str(tmp_path / 'frame_sim_array_1.mat')
    matio.save_frame(f, cube, np.zeros(cube.shape[0]), generation=2)
    loaded, _ = matio.load_frame(f)
    plan = Plan(s['cfg'], s['cfar'], s['clus'], s['pre_p'], device=0)
    a = plan.process_cube(cube, frame_idx=1, want_rdm=True)
    b = plan.process_cube(loaded, frame_idx=1, want_rdm=True)
    plan.close()
    assert np.array_equal(a['rdm'], b['rdm'])
    assert a['final_targets'] == b['final_targets']


@pytest.mark.gpu
def test_stage2_flow_from_mat(tmp_path):
    """debug_simulated_data_processing_v3.m:20-22 load, per-pulse DBF (iq * W', fsf:95),
    then process_stage2_mtd (process_stage2_mtd.m:1) vs the oracle's S6 + S7."""
    import rsp
    from oracle import chain
    from _scen import scenario, targets_for, noisy_cube
    s = scenario('small')
    cube = noisy_cube(s, targets_for('small'), dtype=np.complex128)
    f = str(tmp_path / 'frame_sim_array_1.mat')
    matio.save_frame(f, cube, np.linspace(0, 10, cube.shape[0]), generation=2)
    raw, angle = matio.load_frame(f)
    beams = chain.dbf(raw, s['pre_o']['DBF_coeffs_data_C'])
    mtd, pc = rsp.process_stage2_mtd(beams, angle, s['cfg'], precomputed_data=s['pre_p'])
    pc_o = chain.pulse_compress(beams, s['pre_o'])
    mtd_o = chain.mtd(pc_o, s['pre_o'])
    for got, ref in ((pc, pc_o), (mtd, mtd_o)):
        assert np.abs(got - ref).max() <= 2e-5 * np.abs(ref).max()
