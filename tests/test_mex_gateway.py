"""The committed MEX gateway (matlab/rsp_mex.c) compiles against include/rsp.h.

MATLAB is not available here or on the GPU box, so the gateway cannot run; this CPU test
compiles it (gcc -fsyntax-only, C99, -Wall -Werror) against the real C-ABI header and a
declaration-only mex.h (tests/native/mexstub/) of the documented R2018a MEX API, so that an
ABI change that breaks the gateway fails the suite.  It also checks that every librsp entry
point the gateway calls is declared in include/rsp.h and exported by librsp.so.
"""
import os
import re
import shutil
import subprocess

import pytest

from rsp import _abi

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
MEX = os.path.join(ROOT, 'radar-signal-simulation-and-target-detection_amd', 'matlab', 'rsp_mex.c')


@pytest.mark.skipif(shutil.which('gcc') is None, reason='needs gcc')
def test_gateway_compiles_against_the_header():
    subprocess.run(['gcc', '-std=c99', '-fsyntax-only', '-Wall', '-Werror', '-I', os.path.join(HERE, 'native', 'mexstub'),
                    '-I', os.path.join(ROOT, 'include'), MEX], check=True)


def test_gateway_calls_exported_symbols():
    src = re.sub(r'/\*.*?\*/|"[^"\n]*"', '', open(MEX).read(), flags=re.S)   # code only
    called = set(re.findall(r'\b(rsp_[a-z0-9_]+)\s*\(', src))
    assert {'rsp_plan_create_ex', 'rsp_process_targets', 'rsp_process_cube', 'rsp_process_stage2',
            'rsp_process_stage2_gated'} <= called
    lib = _abi.lib()
    for name in called:
        assert hasattr(lib, name), name


def test_matlab_wrappers_keep_the_reference_signatures():
    d = os.path.dirname(MEX)
    fsf = open(os.path.join(d, 'fun_process_single_frame.m')).read()
    assert re.search(r'^function final_targets = fun_process_single_frame\(targets, config, cfar_params, '
                     r'cluster_params, precomputed_data, frame_idx\)', fsf, re.M)   # fsf:13
    s2 = open(os.path.join(d, 'process_stage2_mtd.m')).read()
    assert re.search(r'^function \[MTD_results, PC_results\] = process_stage2_mtd\(iq_data, angle, config\)', s2,
                     re.M)                                                           # process_stage2_mtd.m:1


INTEGRATION = os.path.join(ROOT, 'INTEGRATION.md')


@pytest.mark.skipif(shutil.which('gcc') is None, reason='needs gcc')
def test_integration_c_snippets_compile(tmp_path):
    """Every C block of INTEGRATION.md is a self-contained unit that compiles against include/rsp.h."""
    blocks = re.findall(r'```c\n(.*?)```', open(INTEGRATION).read(), re.S)
    assert len(blocks) >= 2
    for i, b in enumerate(blocks):
        f = tmp_path / ('snippet%d.c' % i)
        f.write_text(b)
        subprocess.run(['gcc', '-std=c99', '-fsyntax-only', '-Wall', '-Werror', '-I', os.path.join(ROOT, 'include'),
                        str(f)], check=True)


def test_integration_matlab_wrappers_match_committed_files():
    """The MATLAB wrapper shown in INTEGRATION.md is the committed one, line for line (no stale copy)."""
    doc = open(INTEGRATION).read()
    d = os.path.dirname(MEX)
    committed = open(os.path.join(d, 'fun_process_single_frame.m')).read()
    block = [b for b in re.findall(r'```matlab\n(.*?)```', doc, re.S) if 'function final_targets' in b]
    assert len(block) == 1
    code = [ln for ln in committed.splitlines() if ln.strip() and not ln.lstrip().startswith('%')]
    assert [ln for ln in block[0].splitlines() if ln.strip()] == code
    assert 'persistent inited' not in doc and "rsp_mex('init'" not in doc
