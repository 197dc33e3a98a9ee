"""rsp_hbm_copy_probe at a few buffer sizes (the box's stream-copy rate)."""
import ctypes as ct
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..',
                                'radar-signal-simulation-and-target-detection_amd'))
from rsp import _abi  # noqa: E402
if os.environ.get('AB_LIB'):   # timing experiments only: an A/B variant of librsp.so
    _abi.LIB_PATH = os.environ['AB_LIB']

for b in (1 << 28, 1 << 30, 1 << 31):
    g = ct.c_double()
    rc = _abi.lib().rsp_hbm_copy_probe(0, b, 20, ct.byref(g))
    print(b, rc, round(g.value, 1))
