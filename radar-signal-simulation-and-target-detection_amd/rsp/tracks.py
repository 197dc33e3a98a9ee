"""Inter-frame track association (main_simulate_echoes_with_array_v8_3.m:253-352).

``inter_frame_cluster(cumulative_final_log, inter_frame_params)`` turns the per-frame
``final_targets`` (with ``iFrame`` and ``iAntAngle`` injected, v8_3:236-244) into
``final_tracks_log`` the way section 5 of the v8_3 driver does; the association runs in
librsp.so (``rsp_inter_frame_cluster``, host C++).  ``default_inter_frame_params`` restates
``config.inter_frame_cluster`` (v8_3:57-65).
"""
import ctypes as ct

from . import _abi

TRACK_FIELDS = ('Range', 'Velocity', 'Angle', 'Azimuth', 'Power', 'FirstFrame', 'LastFrame', 'NumPoints')


def default_inter_frame_params(cluster_params, K=1.0):
    """config.inter_frame_cluster of v8_3:57-65 (gates = K x the intra-frame cluster_params)."""
    return {'enable': True, 'K': K, 'Gate_R': cluster_params['max_range_sep'] * K,
            'Gate_V': cluster_params['max_vel_sep'] * K, 'Gate_El': cluster_params['max_angle_sep'] * K,
            'Gate_Az': 10.0, 'Max_Frame_Gap': 3}


def inter_frame_cluster(cumulative_final_log, inter_frame_params):
    """v8_3:253-352 -> final_tracks_log (list of dicts with TRACK_FIELDS)."""
    log = list(cumulative_final_log)
    if not inter_frame_params.get('enable', True):   # v8_3:337-351: one track per detection
        return [{'Range': d['Range'], 'Velocity': d['Velocity'], 'Angle': d['Angle'], 'Azimuth': d['iAntAngle'],
                 'Power': d['Power'], 'FirstFrame': d['iFrame'], 'LastFrame': d['iFrame'], 'NumPoints': 1}
                for d in log]
    n = len(log)
    pts = (_abi.TrackPoint * max(n, 1))()
    for i, d in enumerate(log):
        pts[i] = _abi.TrackPoint(d['Range'], d['Velocity'], d['Angle'], d['Power'], d['iAntAngle'], int(d['iFrame']), 0)
    g = inter_frame_params
    gp = _abi.InterFrameParams(g['Gate_R'], g['Gate_V'], g['Gate_Az'], g['Gate_El'], int(g['Max_Frame_Gap']), 0)
    out = (_abi.Track * max(n, 1))()
    n_out = ct.c_int32()
    _abi.check(_abi.lib().rsp_inter_frame_cluster(pts, n, ct.byref(gp), out, n, ct.byref(n_out)))
    return [{f: getattr(out[i], f) for f in TRACK_FIELDS} for i in range(n_out.value)]
