"""The S4.1 noise's ln(u) and sin/cos(2 pi u) (csrc/rsp_noise_math.h, used by k_synth) against
long-double libm on the inputs the Box-Muller transform takes, u = (x + 0.5) 2^-32: ln within 2
ulp, sin/cos within 4e-16 absolute -- closer to the exact values than the oracle's own
np.sin(2 * np.pi * u), whose rounded argument costs up to ~7e-16.  Host-compiled (g++), CPU only."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which('g++') is None, reason='needs g++')
def test_noise_math_accuracy(tmp_path):
    exe = tmp_path / 'nmc'
    subprocess.run(['g++', '-O2', '-std=c++20', os.path.join(ROOT, 'tools', 'noise_math_check.cpp'), '-o',
                    str(exe)], check=True, capture_output=True, timeout=120)
    r = subprocess.run([str(exe), str(1 << 20)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert 'rsp_nm_log' in r.stdout
