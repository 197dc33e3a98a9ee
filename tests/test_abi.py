"""CPU tests of the C-ABI boundary (include/rsp.h <-> librsp.so <-> rsp._abi).

No compute calls: these run without a GPU.  They check that the in-tree library
loads, exports every function the header declares, that the ctypes mirror of
every struct has the C layout (checked against gcc on the real header), and
that argument validation / missing-device errors come back as status codes with
a message instead of crashes.
"""
import ctypes as ct
import os
import re
import subprocess
import tempfile

import pytest

from rsp import _abi
from _scen import scenario

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, 'include', 'rsp.h')


def _declared_functions():
    txt = open(HEADER).read()
    txt = re.sub(r'/\*.*?\*/', '', txt, flags=re.S)
    return sorted(set(re.findall(r'\b(rsp_[a-z0-9_]+)\s*\(', txt)))


def test_library_exports_every_declared_symbol():
    lib = _abi.lib()
    names = _declared_functions()
    assert len(names) >= 20
    for n in names:
        assert hasattr(lib, n), 'librsp.so does not export %s' % n
    assert set(names) == set(_abi.PROTOTYPES), 'ctypes prototypes out of sync with include/rsp.h'


def test_abi_version():
    assert _abi.lib().rsp_abi_version() == 4


STRUCTS = {'rsp_sig_config': _abi.SigConfig, 'rsp_cfar_params': _abi.CfarParams,
           'rsp_cluster_params': _abi.ClusterParams, 'rsp_precomputed': _abi.Precomputed,
           'rsp_target_in': _abi.TargetIn, 'rsp_target': _abi.Target, 'rsp_detection': _abi.Detection,
           'rsp_frame_out': _abi.FrameOut, 'rsp_sizes': _abi.Sizes, 'rsp_music_config': _abi.MusicConfig,
           'rsp_music_scene': _abi.MusicScene, 'rsp_music_out': _abi.MusicOut, 'rsp_track_point': _abi.TrackPoint,
           'rsp_inter_frame_params': _abi.InterFrameParams, 'rsp_track': _abi.Track,
           'rsp_plan_options': _abi.PlanOptions}


def test_struct_layouts_match_header():
    """Compile a probe against include/rsp.h with gcc and compare sizeof/offsetof."""
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "rsp.h"', 'int main(void) {']
    for cname, py in STRUCTS.items():
        lines.append('printf("%s %%zu\\n", sizeof(%s));' % (cname, cname))
        for fname, _ in py._fields_:
            lines.append('printf("%s.%s %%zu\\n", offsetof(%s, %s));' % (cname, fname, cname, fname))
    lines += ['return 0;', '}']
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, 'probe.c')
        exe = os.path.join(d, 'probe')
        open(src, 'w').write('\n'.join(lines))
        subprocess.run(['gcc', '-I', os.path.dirname(HEADER), src, '-o', exe], check=True)
        out = subprocess.run([exe], check=True, capture_output=True, text=True).stdout.split('\n')
    got = dict(l.split() for l in out if l)
    for cname, py in STRUCTS.items():
        assert int(got[cname]) == ct.sizeof(py), cname
        for fname, _ in py._fields_:
            assert int(got['%s.%s' % (cname, fname)]) == getattr(py, fname).offset, (cname, fname)


def test_null_arguments_are_rejected():
    lib = _abi.lib()
    assert lib.rsp_plan_create(None, None, None, None, 0, 1, None) == _abi.RSP_ERR_INVALID
    assert b'null' in lib.rsp_last_error()
    assert lib.rsp_query_sizes(None, None) == _abi.RSP_ERR_INVALID
    assert lib.rsp_drain(None) == _abi.RSP_ERR_INVALID
    assert lib.rsp_process_cube(None, None, 1, 0, 0, None) == _abi.RSP_ERR_INVALID
    assert lib.rsp_stage_name(99) == b'?'
    assert lib.rsp_plan_create_ex(None, None, None, None, None, None) == _abi.RSP_ERR_INVALID
    assert lib.rsp_enqueue_host(None, None, _abi.RSP_C128, 1) == _abi.RSP_ERR_INVALID
    assert lib.rsp_host_alloc(None, 16, None) == _abi.RSP_ERR_INVALID
    assert lib.rsp_host_free(None, None) == _abi.RSP_ERR_INVALID
    assert lib.rsp_process_targets_multi(None, 0, None, None, None, 0, 0, 0.0, None, 0, None) == _abi.RSP_ERR_INVALID
    assert b'bad argument' in lib.rsp_last_error()


def test_plan_options_defaults_and_validation():
    lib = _abi.lib()
    o = _abi.PlanOptions()
    assert lib.rsp_plan_options_default(ct.byref(o)) == _abi.RSP_OK
    assert (o.device, o.frames_per_launch, o.precision, o.flags) == (0, 1, _abi.RSP_C128, 0)
    from rsp.plan import Plan
    s = scenario('small')
    with pytest.raises(ValueError):
        Plan(s['cfg'], s['cfar'], s['clus'], s['pre_p'], precision='c32')


def test_bad_config_is_rejected_before_touching_the_device():
    from rsp.plan import Plan
    s = scenario('small')
    cfg = {'Sig_Config': dict(s['cfg']['Sig_Config'], prtNum=63), 'Array': s['cfg']['Array']}
    with pytest.raises(_abi.RspError) as e:
        Plan(cfg, s['cfar'], s['clus'], s['pre_p'])
    assert e.value.code == _abi.RSP_ERR_UNSUPPORTED      # odd prtNum


def test_plan_without_gpu_fails_loudly():
    """No CPU fallback: on a machine without a HIP device plan creation reports RSP_ERR_DEVICE."""
    from rsp.plan import Plan
    s = scenario('small')
    try:
        p = Plan(s['cfg'], s['cfar'], s['clus'], s['pre_p'])
    except _abi.RspError as e:
        assert e.code == _abi.RSP_ERR_DEVICE
        assert 'device' in str(e)
    else:   # a GPU is present (GPU box): the plan must be real
        assert p.sizes.G == s['pre_p']['N_total_gate']
        p.close()


def _host_cluster(dets, cp):
    lib = _abi.lib()
    arr = (_abi.Detection * max(len(dets), 1))()
    for i, d in enumerate(dets):
        arr[i] = _abi.Detection(d['v_idx'], d['r_idx'], d['pair_idx'], 0, d['Power'], d['Range'], d['Velocity'],
                                d['Angle'])
    out = (_abi.Target * 4096)()
    n = ct.c_int32()
    c = _abi.ClusterParams(cp['max_range_sep'], cp['max_vel_sep'], cp['max_angle_sep'])
    _abi.check(lib.rsp_cluster_detections(arr, len(dets), ct.byref(c), out, 4096, ct.byref(n)))
    return [dict(Range=out[i].Range, Velocity=out[i].Velocity, Angle=out[i].Angle, Power=out[i].Power)
            for i in range(n.value)]


@pytest.mark.parametrize('seed', range(6))
def test_native_clustering_equals_oracle_bfs(seed):
    """librsp's S10/S11 (union-find over a range sweep) == the oracle's literal BFS (fsf:302-407)."""
    import numpy as np
    from oracle import chain
    from rsp import config as C
    rng = np.random.default_rng(seed)
    n = int(rng.integers(1, 400))
    # clumpy detections: a few targets smeared over range/Doppler/pairs plus stragglers
    dets = []
    for i in range(n):
        c = rng.integers(0, 6)
        dets.append(dict(v_idx=int(rng.integers(16, 100)), r_idx=int(rng.integers(16, 2000)),
                         pair_idx=int(rng.integers(1, 8)),
                         Range=1000.0 * c + rng.normal(0, 25), Velocity=5.0 + 0.5 * c + rng.normal(0, 0.3),
                         Angle=3.0 * c + rng.normal(0, 3), Power=float(rng.uniform(1, 100))))
    cp = C.default_cluster_params()
    got = _host_cluster(dets, cp)
    order = sorted(range(n), key=lambda i: (dets[i]['pair_idx'], dets[i]['r_idx'], dets[i]['v_idx']))
    want = chain.cluster_stage2(chain.cluster_stage1([dets[i] for i in order], cp), cp)
    assert len(got) == len(want)
    for a, b in zip(got, want):
        for key in ('Range', 'Velocity', 'Angle', 'Power'):
            assert a[key] == pytest.approx(b[key], rel=1e-12, abs=1e-9)


C_HOST = r'''
#include <stdio.h>
#include "rsp.h"
int main(void) {
    rsp_detection d[3] = {{10, 100, 1, 0, 5.0, 1000.0, 5.0, 1.0},
                          {10, 101, 2, 0, 7.0, 1010.0, 5.1, 2.0},
                          {40, 900, 1, 0, 3.0, 5000.0, -3.0, 0.5}};
    rsp_cluster_params cp = {30.0, 0.4, 5.0};
    rsp_target out[8];
    int32_t n = -1;
    rsp_plan* plan = 0;
    if (rsp_abi_version() != RSP_ABI_VERSION) return 2;
    if (rsp_plan_create(0, 0, 0, 0, 0, 1, &plan) != RSP_ERR_INVALID) return 3;
    if (rsp_cluster_detections(d, 3, &cp, out, 8, &n) != RSP_OK) return 4;
    printf("%d %.6f %.6f\n", n, out[0].Range, out[0].Power);
    return 0;
}
'''


def test_plain_c_host_links_and_calls():
    """A plain C program (what a MEX gateway is) compiles against include/rsp.h, links
    librsp.so and gets status codes + host-side S10/S11 results without a GPU."""
    libdir = os.path.dirname(_abi.lib()._name)
    with tempfile.TemporaryDirectory() as d:
        src, exe = os.path.join(d, 'host.c'), os.path.join(d, 'host')
        open(src, 'w').write(C_HOST)
        subprocess.run(['gcc', '-std=c99', '-Wall', '-Werror', '-I', os.path.dirname(HEADER), src, '-o', exe,
                        '-L', libdir, '-lrsp', '-Wl,-rpath,' + libdir], check=True)
        out = subprocess.run([exe], check=True, capture_output=True, text=True).stdout.split()
    # stage 1 merges the two (power-weighted), stage 2 keeps both groups
    assert int(out[0]) == 2
    assert float(out[1]) == pytest.approx((5 * 1000.0 + 7 * 1010.0) / 12, abs=1e-6)
    assert float(out[2]) == pytest.approx(12.0)


def test_plan_cache_is_keyed_on_content():
    """rsp._plan_for reuses a plan only for equal inputs (round-1 review: id()-keyed cache)."""
    import numpy as np
    import rsp
    s = scenario('small')
    a = rsp._fingerprint(s['cfg'], s['cfar'], s['clus'], s['pre_p'])
    cf = dict(s['cfar'])
    assert rsp._fingerprint(s['cfg'], cf, s['clus'], s['pre_p']) == a      # equal copy: same key
    cf['T_CFAR'] = 9.0
    assert rsp._fingerprint(s['cfg'], cf, s['clus'], s['pre_p']) != a      # other threshold: new key
    pre = dict(s['pre_p'])
    pre['MTD_win'] = np.array(pre['MTD_win'])
    pre['MTD_win'][3] += 1e-12
    assert rsp._fingerprint(s['cfg'], s['cfar'], s['clus'], pre) != a      # array contents count


def test_abi_version_agrees_everywhere():
    """The library, include/rsp.h and the driver's build() check name the same ABI version."""
    import re
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    hv = int(re.search(r'#define RSP_ABI_VERSION (\d+)', open(os.path.join(root, 'include', 'rsp.h')).read()).group(1))
    assert _abi.lib().rsp_abi_version() == hv
    assert 'rsp_abi_version() == %d' % hv in open(os.path.join(root, '__graft_entry__.py')).read()
