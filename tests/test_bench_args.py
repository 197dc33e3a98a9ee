"""bench.py --gpus N (CPU): the launch decision and its error exits.  No GPU is touched: the
errors are raised before any HIP call, and device counting does not create a HIP context."""
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)

import bench  # noqa: E402


@pytest.mark.parametrize('gpus,env,vis,same,backend,want', [
    (1, None, 0, False, 'nccl', 'run'),
    (1, 1, 1, False, 'nccl', 'run'),
    (8, 8, 8, False, 'nccl', 'run'),        # a torchrun rank of the driver's N = 8 run
    (2, None, 8, False, 'nccl', 'spawn'),   # bare `bench.py --gpus 2` on a node
    (2, None, 1, True, 'gloo', 'spawn'),    # rehearsal: two ranks on the one GPU
    (8, None, 1, False, 'nccl', 'error'),   # fewer visible devices than asked for
    (2, 4, 4, False, 'nccl', 'error'),      # WORLD_SIZE differs from --gpus
    (2, None, 1, True, 'nccl', 'error'),    # RCCL refuses two ranks on one device
    (0, None, 1, False, 'nccl', 'error'),
])
def test_launch_mode(gpus, env, vis, same, backend, want):
    mode, msg = bench.launch_mode(gpus, env, vis, same, backend)
    assert mode == want, msg
    assert (msg is not None) == (want == 'error')


def _run(args, **env):
    e = dict(os.environ)
    for k in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK'):
        e.pop(k, None)
    e.update(env)
    return subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py')] + args, env=e, capture_output=True,
                          text=True, timeout=240)


def test_world_size_mismatch_exits_nonzero():
    r = _run(['--gpus', '2'], WORLD_SIZE='3', RANK='0', LOCAL_RANK='0')
    assert r.returncode == 2 and 'WORLD_SIZE=3' in r.stderr
    assert r.stdout == ''


def test_too_few_visible_devices_exits_nonzero():
    """This container has no GPU: --gpus 8 without --same-device must refuse, naming the count."""
    r = _run(['--gpus', '8'], HIP_VISIBLE_DEVICES='')
    assert r.returncode == 2 and '--gpus 8 but only' in r.stderr
    assert r.stdout == ''
