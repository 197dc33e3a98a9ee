"""K3's exact CFAR prefilter (rsp_kernels.hip, RSP_K3_PREFILTER) under low thresholds.

K3 rejects a cell when CUT <= T mean(left range slice) and runs the full GOCA test
(fsf:192-213) only on the survivors.  At the reference's T_CFAR = 8 almost no noise cell
survives, so the default-threshold parity cases never exercise the full-test branch much.
Here T is lowered until a large share of the cells survive the prefilter and many are hits;
the device's detection list must still be the oracle's, cell for cell and in find() order
(complex double).
"""
import numpy as np
import pytest

from oracle import chain
from rsp.plan import Plan

from _scen import scenario, targets_for, noisy_cube

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('name,T', [('small', 2.0), ('small', 3.0), ('x2', 3.0), ('x2', 4.0)])
def test_low_threshold_detections_match_oracle(name, T):
    s = scenario(name)
    cube = noisy_cube(s, targets_for(name), dtype=np.complex128)
    cfar = dict(s['cfar'], T_CFAR=T)
    _, st = chain.process_cube(cube, s['cfg'], cfar, s['clus'], s['pre_o'], keep=True)
    plan = Plan(s['cfg'], cfar, s['clus'], s['pre_p'], precision='c128')
    gpu = plan.process_cube(cube, frame_idx=1)
    plan.close()
    want = [(int(d[0]), int(d[1]), int(d[2])) for d in st['dets']]
    got = [(d['v_idx'], d['r_idx'], d['pair_idx']) for d in gpu['detections']]
    assert len(want) > 100, 'threshold too high to exercise the full-test branch (%d hits)' % len(want)
    assert got == want
