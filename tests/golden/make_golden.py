"""Generate the golden fixtures in tests/golden/ (run from the repo root:
``python tests/golden/make_golden.py``).

The reference is MATLAB and cannot run here, so these vectors come
from the oracle (oracle/, the numpy/scipy complex128 restatement of fsf S4-S11, itself
pinned by the KATs in tests/test_oracle_kat.py).  They freeze the oracle's outputs for
fixed seeded inputs so that (a) the oracle cannot drift silently (CPU test) and (b) the
GPU path is checked against stored vectors without recomputing the oracle
(tests/test_golden.py).  Inputs are fully described by (config name, targets,
frame_idx, seed): the cube is the v8_2 scene synthesised per fsf:45-78 plus Philox noise.

Per case (npz): targets [T x 4] (Range, Velocity, ElevationAngle, SNR_dB), frame_idx,
seed, cube_idx / cube_val (256 probes of the noisy cube, flat column-major index),
rdm_idx / rdm_val (512 probes of rdm_13beam), dets [n x 4] (v, r, pair, S; fsf:220),
par [n x 4] (Range, Velocity, Angle, Power; fsf:293-297), final [m x 4] (fsf:393-406),
near [k x 3] (1-based v, r, pair of cells whose CFAR margin is < 1e-4: the only cells on
which a fp32 path may decide differently).
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
for p in (ROOT, os.path.join(ROOT, 'radar-signal-simulation-and-target-detection_amd'), os.path.dirname(HERE)):
    sys.path.insert(0, p)

from oracle import chain  # noqa: E402
from rsp import config as C  # noqa: E402
from _scen import scenario, targets_for, SEED  # noqa: E402

CASES = [('plumbing', 1), ('small', 1), ('small', 2), ('x2', 1)]


def case_targets(name, frame_idx):
    s = scenario(name)
    tg = targets_for(name)
    for _ in range(frame_idx - 1):          # v8:170-173 evolution between frames
        tg = C.evolve_targets(tg, s['cfg'])
    return s, tg


def make(name, frame_idx):
    s, tg = case_targets(name, frame_idx)
    cube = chain.synthesize_echo(tg, s['cfg'], s['pre_o']) + chain.philox_noise(s['cfg'], frame_idx, SEED)
    fin, st = chain.process_cube(cube, s['cfg'], s['cfar'], s['clus'], s['pre_o'], keep=True)
    rng = np.random.default_rng(1234 + frame_idx)
    cflat = cube.ravel(order='F')
    cidx = np.sort(rng.choice(cflat.size, 256, replace=False))
    rflat = st['rdm'].ravel(order='F')
    ridx = np.sort(rng.choice(rflat.size, 512, replace=False))
    dets = np.asarray(st['dets'], float).reshape(-1, 4)
    par = np.asarray([[e['Range'], e['Velocity'], e['Angle'], e['Power']] for e in st['par']], float).reshape(-1, 4)
    final = np.asarray([[t['Range'], t['Velocity'], t['Angle'], t['Power']] for t in fin], float).reshape(-1, 4)
    if s['cfg']['Sig_Config']['beam_num'] > 1:
        mg = chain.cfar_margin(st['rdm'], s['cfar'])
        near = np.argwhere(mg < 1e-4) + 1
    else:
        near = np.zeros((0, 3), int)
    tarr = np.asarray([[t['Range'], t['Velocity'], t['ElevationAngle'], t['SNR_dB']] for t in tg], float)
    out = os.path.join(HERE, 'golden_%s_f%d.npz' % (name, frame_idx))
    np.savez_compressed(out, name=name, frame_idx=frame_idx, seed=SEED, targets=tarr,
                        cube_idx=cidx, cube_val=cflat[cidx], rdm_idx=ridx, rdm_val=rflat[ridx],
                        rdm_absmax=np.abs(rflat).max(), dets=dets, par=par, final=final, near=near.astype(np.int32))
    print(out, 'dets', len(dets), 'final', len(final), 'near', len(near), os.path.getsize(out), 'bytes')


if __name__ == '__main__':
    for n, f in CASES:
        make(n, f)
