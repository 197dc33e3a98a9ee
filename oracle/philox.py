"""Philox4x32-10 + Box-Muller noise -- TEST INFRASTRUCTURE (oracle side).

Replaces MATLAB ``randn`` in the noise step of ``fun_process_single_frame.m:80-88``
(``noise = (randn + 1j*randn) .* sqrt(P_noise_floor/2)``).  MATLAB's Mersenne
Twister + ziggurat stream cannot be reproduced, so both this oracle and the
device synthesis kernel use the same documented counter-based generator:

  complex sample i (linear index in the cube's [C][N][P] storage, i.e. MATLAB
  column-major [P x N x C]) draws from philox4x32_10(counter, key) with
     counter = (lo32(i >> 1), hi32(i >> 1), frame_idx, 0x52535020)
     key     = (lo32(seed), hi32(seed))
  words (x0, x1) feed sample 2k, words (x2, x3) feed sample 2k+1;
  u = (x + 0.5) * 2^-32;  r = sqrt(-2 ln u_a);  I = r cos(2 pi u_b), Q = r sin(2 pi u_b).
"""
import numpy as np

M0 = np.uint64(0xD2511F53)
M1 = np.uint64(0xCD9E8D57)
W0 = np.uint32(0x9E3779B9)
W1 = np.uint32(0xBB67AE85)
TAG = 0x52535020
MASK32 = np.uint64(0xFFFFFFFF)


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Vectorised Philox4x32-10; all inputs uint32 arrays/scalars."""
    c0 = np.asarray(c0, np.uint32); c1 = np.asarray(c1, np.uint32)
    c2 = np.asarray(c2, np.uint32); c3 = np.asarray(c3, np.uint32)
    k0 = np.uint32(k0); k1 = np.uint32(k1)
    for rnd in range(10):
        p0 = M0 * c0.astype(np.uint64)
        p1 = M1 * c2.astype(np.uint64)
        hi0 = (p0 >> np.uint64(32)).astype(np.uint32); lo0 = (p0 & MASK32).astype(np.uint32)
        hi1 = (p1 >> np.uint64(32)).astype(np.uint32); lo1 = (p1 & MASK32).astype(np.uint32)
        c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
        if rnd < 9:
            k0 = np.uint32((int(k0) + int(W0)) & 0xFFFFFFFF)
            k1 = np.uint32((int(k1) + int(W1)) & 0xFFFFFFFF)
    return c0, c1, c2, c3


def unit_normal_complex(n_samples, frame_idx, seed, start=0, tag=TAG):
    """Complex samples I + jQ (each I, Q ~ N(0,1)) for linear indices start..start+n-1.

    ``tag`` is counter word 3 (the stream id): TAG for the echo noise, the MUSIC
    streams use their own tags (oracle/music.py)."""
    idx = np.arange(start, start + n_samples, dtype=np.uint64)
    pair = idx >> np.uint64(1)
    lo = (pair & MASK32).astype(np.uint32)
    hi = (pair >> np.uint64(32)).astype(np.uint32)
    fr = np.full(lo.shape, frame_idx & 0xFFFFFFFF, np.uint32)
    tag = np.full(lo.shape, tag, np.uint32)
    x0, x1, x2, x3 = philox4x32_10(lo, hi, fr, tag, seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)
    odd = (idx & np.uint64(1)).astype(bool)
    ua = np.where(odd, x2, x0).astype(np.float64)
    ub = np.where(odd, x3, x1).astype(np.float64)
    ua = (ua + 0.5) * 2.3283064365386963e-10
    ub = (ub + 0.5) * 2.3283064365386963e-10
    r = np.sqrt(-2.0 * np.log(ua))
    ang = 2.0 * np.pi * ub
    return r * np.cos(ang) + 1j * (r * np.sin(ang))
