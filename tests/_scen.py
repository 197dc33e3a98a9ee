"""Shared scenario builders for the tests (oracle = checker, rsp = product)."""
import numpy as np

from rsp import config as C
from rsp.precompute import precompute as product_precompute
from oracle import chain, precompute as oracle_precompute

SEED = 20250101


def scenario(name):
    cfg, cfar, clus, W, ang, k = C.named_config(name)
    pre_o = oracle_precompute.precompute(cfg, W, ang, k, C.V8_FIR)
    pre_p = product_precompute(cfg, W, ang, k, C.V8_FIR)
    return dict(name=name, cfg=cfg, cfar=cfar, clus=clus, pre_o=pre_o, pre_p=pre_p)


def targets_for(name):
    """v8_2's five targets (v8_2:28-51), clipped to the config's coverage."""
    cfg = C.named_config(name)[0]
    sc = cfg['Sig_Config']
    G = sum(sc['point_prt_segments'])
    rmax = 0.9 * G * sc['c'] / (2 * sc['fs'])
    vmax = 0.45 * sc['wavelength'] / (2 * sc['prt'])
    out = []
    for t in C.v8_2_targets():
        if t['Range'] < rmax and abs(t['Velocity']) < vmax:
            out.append(dict(t))
    if not out:
        out = [dict(Range=0.5 * rmax, Velocity=0.3 * vmax, ElevationAngle=10.0, SNR_dB=10.0)]
    return out


def noisy_cube(s, targets, frame_idx=1, seed=SEED, dtype=np.complex64):
    raw = chain.synthesize_echo(targets, s['cfg'], s['pre_o']) + chain.philox_noise(s['cfg'], frame_idx, seed)
    return raw.astype(dtype)


def det_key_set(dets):
    return {(int(d[0]), int(d[1]), int(d[2])) for d in dets}


def device_cube(plan, targets, frame_idx=1, seed=SEED):
    """S4 + S4.1 synthesised on the device in the plan's precision, downloaded as [P, N, C]."""
    ptr = plan.device_alloc(plan.cube_bytes)
    try:
        plan.synthesize_device(ptr, targets, frame_idx=frame_idx, seed=seed)
        plan.sync()
        flat = plan.device_download(ptr, plan.sizes.cube_elems, plan.cdtype)
    finally:
        plan.device_free(ptr)
    return flat.reshape((plan.P, plan.N, plan.C), order='F').astype(np.complex128)
