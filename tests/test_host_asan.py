"""AddressSanitizer + UBSan build of librsp's host-only C++ (CPU, no GPU).

csrc/rsp_mat.cpp (the MAT Level-5 reader/writer that parses untrusted frame files) and
csrc/rsp_host.cpp (error sink, S10/S11 clustering of fun_process_single_frame.m:302-407,
inter-frame association of main_simulate_echoes_with_array_v8_3.m:253-352) are compiled with
g++ -fsanitize=address,undefined together with tests/native/host_fuzz.cpp and driven over:
  * the reference's MATLAB-written files and scipy-written frames;
  * crafted malformed files: a small-form element claiming 8 inline bytes (the overflow the
    round-1 review found), truncations at every 7th byte, dims larger than the data, a corrupt
    zlib stream, and seeded random byte flips;
  * random detection / track lists of up to 3000 entries with undersized output buffers.
Only sanitizer reports (non-zero exit) fail; the functions' status codes are not checked here
(tests/test_matio.py does that).
"""
import os
import shutil
import struct
import subprocess
import zlib

import numpy as np
import pytest
import scipy.io as sio

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(ROOT, 'radar-signal-simulation-and-target-detection_amd', 'csrc')
REF = os.path.join(HERE, 'golden', 'ref_mat')

pytestmark = pytest.mark.skipif(shutil.which('g++') is None, reason='needs g++')


@pytest.fixture(scope='module')
def fuzz_bin(tmp_path_factory):
    d = tmp_path_factory.mktemp('asan')
    exe = str(d / 'host_fuzz')
    cmd = ['g++', '-std=c++17', '-O1', '-g', '-fsanitize=address,undefined', '-fno-sanitize-recover=undefined',
           '-fno-omit-frame-pointer', '-I', os.path.join(ROOT, 'include'),
           os.path.join(CSRC, 'rsp_mat.cpp'), os.path.join(CSRC, 'rsp_host.cpp'),
           os.path.join(HERE, 'native', 'host_fuzz.cpp'), '-o', exe, '-lz', '-lpthread']
    subprocess.run(cmd, check=True)
    return exe


def _run(exe, *args):
    env = dict(os.environ, ASAN_OPTIONS='detect_leaks=1:verify_asan_link_order=0:abort_on_error=0',
               UBSAN_OPTIONS='print_stacktrace=1')
    r = subprocess.run([exe] + list(args), capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0 and 'ERROR: AddressSanitizer' not in r.stderr and 'runtime error' not in r.stderr, \
        r.stderr[-3000:]


def _header():
    return b'MATLAB 5.0 MAT-file, crafted'.ljust(116, b' ') + b'\0' * 8 + struct.pack('<HH', 0x0100, 0x4D49)


def _small_overflow():
    """miMATRIX whose real part is a small-form element claiming 8 inline bytes."""
    body = struct.pack('<II', 6, 8) + struct.pack('<II', 6, 0)                 # array flags: double
    body += struct.pack('<II', 5, 8) + struct.pack('<ii', 1, 2)                # dims 1 x 2
    body += struct.pack('<I', (1 << 16) | 1) + b'x\0\0\0'                      # name 'x' (small form)
    body += struct.pack('<I', (8 << 16) | 9) + struct.pack('<d', 1.0)[:4]      # small form, 8 bytes claimed
    return _header() + struct.pack('<II', 14, len(body)) + body


def _dims_exceed_data():
    body = struct.pack('<II', 6, 8) + struct.pack('<II', 6, 0)
    body += struct.pack('<II', 5, 8) + struct.pack('<ii', 100000, 100000)
    body += struct.pack('<I', (1 << 16) | 1) + b'y\0\0\0'
    body += struct.pack('<II', 9, 16) + struct.pack('<dd', 1.0, 2.0)
    return _header() + struct.pack('<II', 14, len(body)) + body


def _bad_zlib():
    z = zlib.compress(b'\x0e\0\0\0' + b'\0' * 60)
    z = z[:10] + bytes(b ^ 0x5A for b in z[10:])
    return _header() + struct.pack('<II', 15, len(z)) + z


def _files(tmp):
    out = [os.path.join(REF, 'FIR.mat'), os.path.join(REF, 'file.mat')]
    rng = np.random.default_rng(7)
    cube = rng.standard_normal((4, 6, 3)) + 1j * rng.standard_normal((4, 6, 3))
    for comp in (False, True):
        fn = os.path.join(tmp, 'frame_%d.mat' % comp)
        sio.savemat(fn, {'raw_iq_data_noise_sample': cube, 'servo_angle': np.arange(4.0)[None]},
                    do_compression=comp)
        out.append(fn)
    crafted = {'small_overflow.mat': _small_overflow(), 'dims.mat': _dims_exceed_data(), 'zlib.mat': _bad_zlib()}
    for src in list(out):
        data = open(src, 'rb').read()
        base = os.path.basename(src)
        for cut in range(128, len(data), 7):
            crafted['trunc_%s_%d.mat' % (base, cut)] = data[:cut]
        for k in range(40):
            b = bytearray(data)
            for _ in range(1 + k % 5):
                i = int(rng.integers(128, len(b)))
                b[i] = int(rng.integers(0, 256))
            crafted['flip_%s_%d.mat' % (base, k)] = bytes(b)
    for name, data in crafted.items():
        fn = os.path.join(tmp, name)
        open(fn, 'wb').write(data)
        out.append(fn)
    return out


def test_mat_reader_under_asan(fuzz_bin, tmp_path):
    files = _files(str(tmp_path))
    assert len(files) > 200
    for i in range(0, len(files), 100):
        _run(fuzz_bin, 'mat', *files[i:i + 100])


@pytest.mark.parametrize('seed', [1, 2])
def test_clustering_under_asan(fuzz_bin, seed):
    _run(fuzz_bin, 'cluster', str(seed))


def test_malformed_small_element_is_an_error(tmp_path):
    """The shipped library rejects the oversized small-form element with a status code."""
    from rsp import matio
    from rsp._abi import RspError
    fn = str(tmp_path / 'small_overflow.mat')
    open(fn, 'wb').write(_small_overflow())
    with pytest.raises(RspError):
        matio.load(fn)
