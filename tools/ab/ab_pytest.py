"""Run pytest in-process against a variant library (A/B builds only).
usage: ab_pytest.py LIB_PATH [pytest args...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, 'radar-signal-simulation-and-target-detection_amd'))
sys.path.insert(0, ROOT)
from rsp import _abi   # noqa: E402
_abi.LIB_PATH = os.path.abspath(sys.argv[1])
import pytest   # noqa: E402
sys.exit(pytest.main(sys.argv[2:]))
