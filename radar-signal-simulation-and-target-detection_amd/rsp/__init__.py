"""rsp -- MI355X-native per-frame radar signal processing (host side).

Drop-in for the MATLAB reference's per-frame chain
(XuZerui2023/Radar-Signal-Simulation-and-Target-Detection, Simulation/):

* ``fun_process_single_frame(targets, config, cfar_params, cluster_params,
  precomputed_data, frame_idx)``  -- fun_process_single_frame.m:13
* ``process_stage2_mtd(iq_data, angle, config)``  -- process_stage2_mtd.m:1
* ``precompute(...)`` -- the driver's "%% 3" section (v8:79-155)
* ``load_frame`` / ``save_frame`` -- the ``frame_sim_array_%d.mat`` load/save pair
  (main_simulate_echoes_with_array_v2.m:285, debug_simulated_data_processing_v3.m:20-22)

All compute runs in librsp.so (HIP kernels for gfx950 behind the C-ABI in
include/rsp.h).  There is no CPU fallback.
"""
import collections
import hashlib

import numpy as np

from .config import (named_config, make_config, default_cfar_params, default_cluster_params,
                     v8_2_targets, evolve_targets, V8_FIR, stage2_config, debug_v3_config)
from .precompute import precompute
from .plan import Plan, process_targets_multi
from ._abi import RspError
from .matio import load_frame, save_frame
from .music import MusicPlan, MUSIC_1D
from .tracks import inter_frame_cluster, default_inter_frame_params
from . import matio

# main_simulate_echoes_with_array_v2.m:257-264: PRT columns of the three gated segments
REFERENCE_GATE_COLS = ((83, 310), (311, 1033), (1034, 3486))

_PLANS = collections.OrderedDict()   # content fingerprint -> Plan (most recently used last)
_MAX_PLANS = 4


def _fingerprint(*objs):
    """SHA-1 over the contents of nested dicts / lists / scalars / numpy arrays, so that a plan
    is reused only for equal inputs (an in-place edit or a new dict with other values makes a
    new plan; a garbage-collected dict's reused id() cannot alias an old one)."""
    h = hashlib.sha1()

    def feed(o):
        if isinstance(o, dict):
            h.update(b'{')
            for k in sorted(o, key=str):
                feed(str(k))
                feed(o[k])
            h.update(b'}')
        elif isinstance(o, (list, tuple)):
            h.update(b'[')
            for x in o:
                feed(x)
            h.update(b']')
        elif isinstance(o, np.ndarray):
            h.update(b'A' + str(o.dtype).encode() + str(o.shape).encode())
            h.update(np.ascontiguousarray(o).tobytes())
        else:
            h.update(b'S' + type(o).__name__.encode() + repr(o).encode())
    for o in objs:
        feed(o)
    return h.hexdigest()


def _plan_for(config, cfar_params, cluster_params, precomputed_data, device=0, precision='c128'):
    key = _fingerprint(config, cfar_params, cluster_params, precomputed_data, device, precision)
    p = _PLANS.pop(key, None)
    if p is None:
        p = Plan(config, cfar_params, cluster_params, precomputed_data, device=device, precision=precision)
        while len(_PLANS) >= _MAX_PLANS:
            _PLANS.popitem(last=False)[1].close()
    _PLANS[key] = p
    return p


def fun_process_single_frame(targets, config, cfar_params, cluster_params, precomputed_data, frame_idx,
                             seed=20250101, device=0, precision='c128'):
    """fun_process_single_frame.m:13 -- returns ``final_targets`` (list of dicts with
    Range, Velocity, Angle, Power).  Echo synthesis (S4) and noise (S4.1) run on the
    device; MATLAB ``randn`` is replaced by the documented Philox stream (seed, frame_idx).
    Complex double by default, like MATLAB."""
    p = _plan_for(config, cfar_params, cluster_params, precomputed_data, device, precision)
    return p.process_targets(targets, frame_idx=frame_idx, seed=seed)['final_targets']


def _stage2_precompute(config):
    """precomputed_data for the stage-2 path built from ``config`` alone (the 3-argument call):
    waveform, matched filters, segment geometry and MTD window of v8:79-135; the DBF weights,
    beam angles and K-LUT are not used by stage 2 and are zero.  ``config`` is already in the
    v8 form (config.stage2_config)."""
    sc = config['Sig_Config']
    B, C = int(sc['beam_num']), int(sc['channel_num'])
    return precompute(config, np.zeros((B, C), complex), np.zeros(B), np.zeros(max(B - 1, 0)), V8_FIR)


def process_stage2_mtd(iq_data, angle, config, precomputed_data=None, gate_cols=None, device=0, precision='c128'):
    """process_stage2_mtd.m:1 -- ``[MTD_results, PC_results] = process_stage2_mtd(iq_data, angle, config)``.

    ``iq_data[m, n, b]`` is beamformed fast-time data (the DBF of
    debug_simulated_data_processing_v3.m:146-152), either the full PRT (``n`` = point_PRT) or
    gated like the v2 ``.mat`` frames (main_simulate_echoes_with_array_v2.m:256-267: PRT columns
    83:310, 311:1033, 1034:3486 side by side, n = 3404; other gatings via ``gate_cols``, 1-based
    inclusive (first, last) per segment).  Gated columns are put back at their PRT positions
    (zeros elsewhere).  ``angle`` (servo angle) is unused, as in the reference.  Returns
    complex [P, G, B] arrays, G = N_total_gate (process_stage2_mtd.m:29-30 pre-sizes 332 x 3404
    x 13 for the reference config).

    The reference's arithmetic (fun_MTD_produce -> fun_lss_pulse_compression / fun_Process_MTD,
    debug_simulated_data_processing_v2.m:259-405) is un-vendored; this backs it with the
    per-frame chain's own S6 pulse compression + S7 MTD (fsf:99-136).  ``precomputed_data``
    defaults to the one v8:79-135 builds from ``config``."""
    config = stage2_config(config)   # the v3 debug script's config form too (point_PRT = 3404, no gaps / Array)
    if precomputed_data is None:
        precomputed_data = _stage2_precompute(config)
    p = _plan_for(config, default_cfar_params(), default_cluster_params(), precomputed_data, device, precision)
    iq = np.asarray(iq_data)
    if iq.ndim == 2:
        iq = iq[:, :, None]
    if iq.shape[1] == p.N:
        return p.process_stage2(iq)
    return p.process_stage2(iq, gate_cols=gate_cols if gate_cols is not None else REFERENCE_GATE_COLS)
