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
    assert _abi.lib().rsp_abi_version() == 1


STRUCTS = {'rsp_sig_config': _abi.SigConfig, 'rsp_cfar_params': _abi.CfarParams,
           'rsp_cluster_params': _abi.ClusterParams, 'rsp_precomputed': _abi.Precomputed,
           'rsp_target_in': _abi.TargetIn, 'rsp_target': _abi.Target, 'rsp_detection': _abi.Detection,
           'rsp_frame_out': _abi.FrameOut, 'rsp_sizes': _abi.Sizes}


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
