"""Inter-frame track association (v8_3:253-352): native rsp_inter_frame_cluster vs the literal
BFS restatement (oracle/tracks.py), bit-identical (host only, no GPU)."""
import numpy as np
import pytest

from oracle import tracks as ot
from rsp import tracks as rt
from rsp.config import default_cluster_params


def _log(rng, n_tracks=6, frames=12, clutter=20):
    log = []
    for f in range(1, frames + 1):
        az = -30.0 + 4.0 * f                                   # servo sweep (v8_1 style)
        for t in range(n_tracks):
            if rng.random() < 0.8:                             # missed detections make frame gaps
                log.append({'Range': 2000.0 + 900.0 * t + 3.0 * f + rng.normal(0, 2), 'Velocity': -5.0 + 2.0 * t +
                            rng.normal(0, 0.05), 'Angle': -10.0 + 5.0 * t + rng.normal(0, 0.3),
                            'Power': float(rng.uniform(10, 100)), 'iFrame': f, 'iAntAngle': az})
        for _ in range(rng.integers(0, clutter // frames + 2)):
            log.append({'Range': float(rng.uniform(500, 9000)), 'Velocity': float(rng.uniform(-20, 20)),
                        'Angle': float(rng.uniform(-20, 30)), 'Power': float(rng.uniform(1, 20)), 'iFrame': f,
                        'iAntAngle': az})
    return log


@pytest.mark.parametrize('seed', [0, 1, 2, 3])
def test_native_tracks_equal_reference_bfs(seed):
    rng = np.random.default_rng(seed)
    g = rt.default_inter_frame_params(default_cluster_params())
    g['Gate_Az'] = 10.0
    log = _log(rng)
    got = rt.inter_frame_cluster(log, g)
    want = ot.inter_frame_cluster(log, g)
    assert len(got) == len(want)
    for a, b in zip(got, want):
        assert a == b   # same labels, same winner, same summation order


def test_gates_split_tracks_by_frame_gap():
    g = {'enable': True, 'Gate_R': 30.0, 'Gate_V': 0.4, 'Gate_Az': 10.0, 'Gate_El': 5.0, 'Max_Frame_Gap': 3}
    pt = lambda f, p: {'Range': 1000.0, 'Velocity': 1.0, 'Angle': 0.0, 'Power': p, 'iFrame': f, 'iAntAngle': 0.0}
    log = [pt(1, 5.0), pt(2, 7.0), pt(4, 7.0), pt(9, 1.0)]    # 4 -> 9 is a gap of 5 > 3
    tr = rt.inter_frame_cluster(log, g)
    assert [(t['FirstFrame'], t['LastFrame'], t['NumPoints']) for t in tr] == [(1, 4, 3), (9, 9, 1)]
    assert tr[0]['Power'] == 7.0                                # first max wins
    assert tr == ot.inter_frame_cluster(log, g)


def test_empty_and_disabled():
    g = rt.default_inter_frame_params(default_cluster_params())
    assert rt.inter_frame_cluster([], g) == []
    log = [{'Range': 1.0, 'Velocity': 2.0, 'Angle': 3.0, 'Power': 4.0, 'iFrame': 5, 'iAntAngle': 6.0}]
    off = dict(g, enable=False)
    assert rt.inter_frame_cluster(log, off) == [{'Range': 1.0, 'Velocity': 2.0, 'Angle': 3.0, 'Azimuth': 6.0,
                                                 'Power': 4.0, 'FirstFrame': 5, 'LastFrame': 5, 'NumPoints': 1}]
