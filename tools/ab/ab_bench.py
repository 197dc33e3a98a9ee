"""A/B bench: run bench.py's main() against a variant library (timing experiments only).
usage: ab_bench.py LIB_PATH|base [bench args...]   -> prints one summary line."""
import json
import os
import runpy
import sys
import io
import contextlib

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, 'radar-signal-simulation-and-target-detection_amd'))
lib = sys.argv[1]
if lib != 'base':
    from rsp import _abi
    _abi.LIB_PATH = lib
sys.argv = ['bench.py'] + sys.argv[2:] + ['--no-cpu-baseline']
buf = io.StringIO()
with contextlib.redirect_stdout(buf):
    try:
        runpy.run_path(os.path.join(ROOT, 'bench.py'), run_name='__main__')
    except SystemExit as e:
        if e.code:
            raise
d = json.loads(buf.getvalue().strip().splitlines()[-1])
print('%s value %.0f ms_per_step %.4f' % (os.path.basename(lib), d['value'], d['ms_per_step']))
