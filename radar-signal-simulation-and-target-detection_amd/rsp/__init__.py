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
from .config import (named_config, make_config, default_cfar_params, default_cluster_params,
                     v8_2_targets, evolve_targets, V8_FIR)
from .precompute import precompute
from .plan import Plan
from ._abi import RspError
from .matio import load_frame, save_frame
from .music import MusicPlan, MUSIC_1D
from .tracks import inter_frame_cluster, default_inter_frame_params
from . import matio

_PLANS = {}


def _plan_for(config, cfar_params, cluster_params, precomputed_data, device=0):
    key = (id(config), id(cfar_params), id(cluster_params), id(precomputed_data), device)
    p = _PLANS.get(key)
    if p is None:
        p = Plan(config, cfar_params, cluster_params, precomputed_data, device=device)
        _PLANS[key] = p
    return p


def fun_process_single_frame(targets, config, cfar_params, cluster_params, precomputed_data, frame_idx,
                             seed=20250101, device=0):
    """fun_process_single_frame.m:13 -- returns ``final_targets`` (list of dicts with
    Range, Velocity, Angle, Power).  Echo synthesis (S4) and noise (S4.1) run on the
    device; MATLAB ``randn`` is replaced by the documented Philox stream (seed, frame_idx)."""
    p = _plan_for(config, cfar_params, cluster_params, precomputed_data, device)
    return p.process_targets(targets, frame_idx=frame_idx, seed=seed)['final_targets']


def process_stage2_mtd(iq_data, angle, config, cfar_params=None, cluster_params=None, precomputed_data=None,
                       device=0):
    """process_stage2_mtd.m:1 -- ``[MTD_results, PC_results]`` for beamformed data
    ``iq_data[m, n, b]``.  ``angle`` (servo angle) is unused, as in the reference.
    The reference's fun_MTD_produce is un-vendored; this backs it with fsf S6 + S7
    using ``precomputed_data`` (built from ``config`` when omitted)."""
    from .config import default_cfar_params as _dc, default_cluster_params as _dl
    if precomputed_data is None:
        raise ValueError('precomputed_data is required (fun_MTD_produce is not in the reference)')
    p = _plan_for(config, cfar_params or _dc(), cluster_params or _dl(), precomputed_data, device)
    return p.process_stage2(iq_data)
