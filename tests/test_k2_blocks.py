"""K2's overlap-save block sizes beside the 2560-point long block.

x2 is the only named configuration whose long segment takes the mixed-radix 2560-point block, and
such a plan sizes every K2 workgroup for it (4 per CU, k2_pc<double, 4>: 40 KB of LDS, no pads,
twiddles from L1/L2): its power-of-two blocks then run the 2048-point-workgroup instantiations (2048 / M rows per workgroup).  x2's medium
segment exercises only M = 1024 there.  These configurations keep x2's long segment (28 us pulse,
1860 gates: one 2560-point block) and shorten or lengthen the medium pulse and gate count
(fun_process_single_frame.m:115-116 with N_fft / MF_medium_fft from
main_simulate_echoes_with_array_v8.m:104-123), so that the medium segment takes M = 128, 256, 512
and 2048 (16, 8, 4 and 1 rows per workgroup); 'narrow2700' widens the narrow segment past what a
2560-point workgroup stages.  The device RD map must match the complex128 oracle to
1e-12 of its maximum (complex double) and the CFAR detection lists must be identical; in complex
single (2-per-CU workgroups, the same block sizes) the maps within 2e-5.
"""
import numpy as np
import pytest

from oracle import chain
from rsp import config as C
from rsp.plan import Plan

from _scen import oracle_precompute, product_precompute, SEED

# name: (tao (s), point_prt_segments, point_PRT) -> the medium block the plan's cost model picks.
# Every stitched gate must lie inside its segment's convolution support (the long gates are
# outputs g1 + g2 .. G - 1 of a convolution of N - seg_start_long + 1 samples, fsf:119-126):
# gates past it are exact zeros whose CFAR decisions are set by round-off, in MATLAB as here,
# hence N = 8192 for the 1800-gate medium segment.
CFGS = {
    'med128': ((0.16e-6, 1e-6, 28e-6), (228, 100, 1860), 4096, 128),
    'med256': ((0.16e-6, 2e-6, 28e-6), (228, 200, 1860), 4096, 256),
    'med512': ((0.16e-6, 4e-6, 28e-6), (228, 400, 1860), 4096, 512),
    'med2048': ((0.16e-6, 8e-6, 28e-6), (228, 1800, 1860), 8192, 2048),
    # a 2700-gate narrow segment: its direct-FIR rows (~2.7 k samples) do not fit a 2560-point
    # workgroup, so the plan falls back to 2-per-CU workgroups (RSP_K2_POINTS) that still run the
    # long segment's 2560-point block (this used to fail plan creation)
    'narrow2700': ((0.16e-6, 8e-6, 28e-6), (2700, 723, 1860), 8192, 1024),
}


def _scen(name):
    tao, segs, N, _ = CFGS[name]
    _, cfar, clus, W, ang, k = C.named_config('small')
    cfg = C.make_config(prtNum=64, point_PRT=N, channel_num=16, beam_num=4, tao=tao, point_prt_segments=segs)
    return dict(cfg=cfg, cfar=cfar, clus=clus, pre_o=oracle_precompute.precompute(cfg, W, ang, k, C.V8_FIR),
                pre_p=product_precompute(cfg, W, ang, k, C.V8_FIR))


def _targets(cfg):
    """v8_2's targets inside the configuration's range and velocity coverage, plus one in the
    medium segment's gates."""
    sc = cfg['Sig_Config']
    g1, g2, _ = sc['point_prt_segments']
    dr = sc['c'] / (2 * sc['fs'])
    rmax = 0.9 * sum(sc['point_prt_segments']) * dr
    vmax = 0.45 * sc['wavelength'] / (2 * sc['prt'])
    out = [dict(t) for t in C.v8_2_targets() if t['Range'] < rmax and abs(t['Velocity']) < vmax]
    out.append(dict(Range=(g1 + 0.5 * g2) * dr, Velocity=0.2 * vmax, ElevationAngle=8.0, SNR_dB=12.0))
    return out


def _block(mf, ga, gb):
    """The block size rsp_plan.cpp's build_fft_segment picks (cost blocks x M (log2 M + 2))."""
    h = np.fft.ifft(np.asarray(mf))
    a = np.abs(h)
    Lh = int(np.nonzero(a > 1e-10 * a.max())[0].max()) + 1
    best, bm = 1e300, 0
    for M in (64, 128, 256, 512, 1024, 2048, 2560, 4096):
        V = M - Lh + 1
        if V < 1:
            continue
        cost = -(-(gb - ga) // V) * M * (np.log2(M) + 2)
        if cost < best * 0.999:
            best, bm = cost, M
    return bm


@pytest.mark.parametrize('name', sorted(CFGS))
def test_configs_reach_the_intended_blocks(name):
    """The configurations do exercise the block sizes this file is about (host-side check of
    the plan's cost model on the product precompute)."""
    s = _scen(name)
    g1, g2, g3 = s['cfg']['Sig_Config']['point_prt_segments']
    pre = s['pre_p']
    get = (lambda n: pre[n]) if isinstance(pre, dict) else (lambda n: getattr(pre, n))
    assert _block(get('MF_medium_fft'), g1, g1 + g2) == CFGS[name][3]
    assert _block(get('MF_long_fft'), g1 + g2, g1 + g2 + g3) == 2560
    # every stitched long gate inside the long convolution's support (no all-zero columns)
    N = s['cfg']['Sig_Config']['point_PRT']
    assert g1 + g2 + g3 <= (N - get('seg_start_long') + 1) + 700 - 1


@pytest.mark.gpu
@pytest.mark.parametrize('prec', ['c128', 'c64'])
@pytest.mark.parametrize('name', sorted(CFGS))
def test_k2_block_sizes_match_oracle(name, prec):
    s = _scen(name)
    tg = _targets(s['cfg'])
    cube = (chain.synthesize_echo(tg, s['cfg'], s['pre_o']) + chain.philox_noise(s['cfg'], 1, SEED))
    cube = cube.astype(np.complex128 if prec == 'c128' else np.complex64)
    fin, st = chain.process_cube(cube.astype(np.complex128), s['cfg'], s['cfar'], s['clus'], s['pre_o'], keep=True)
    plan = Plan(s['cfg'], s['cfar'], s['clus'], s['pre_p'], precision=prec)
    try:
        out = plan.process_cube(cube, frame_idx=1, want_rdm=True)
        out_mag = plan.process_cube(cube, frame_idx=1, want_rdm=False)   # the queue's magnitude-only store
    finally:
        plan.close()
    ref = st['rdm']
    err = np.abs(out['rdm'] - ref).max() / np.abs(ref).max()
    tol = 1e-12 if prec == 'c128' else 2e-5
    assert err <= tol, 'RDM max rel err %.3g (tol %g)' % (err, tol)
    got = [(d['v_idx'], d['r_idx'], d['pair_idx']) for d in out['detections']]
    assert got == [(d['v_idx'], d['r_idx'], d['pair_idx']) for d in out_mag['detections']]
    if prec == 'c128':
        assert got == [(int(v), int(r), int(p)) for v, r, p, _ in st['dets']]
        assert len(out['final_targets']) == len(fin)
