"""bench.py's device-list route (``--devices N``: one process, the C ABI's
fitoct_config.devices, the route R's fitExpGP(n_gpus = N) takes through .Call):
argument and error paths, checked on the CPU before anything touches a GPU."""
from __future__ import annotations

import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, env=None):
    e = dict(os.environ, **(env or {}))
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT,
                          env=e, capture_output=True, text=True, timeout=300)


@pytest.mark.parametrize("args,env,msg", [
    # the device list is the single-process route: not under torchrun
    (["--gpus", "2", "--devices", "2"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"},
     "without torchrun"),
    # --devices and --device-ids disagree
    (["--devices", "3", "--device-ids", "0,0"], {}, "--device-ids lists 2"),
    # more GPUs than visible (none here)
    (["--devices", "2"], {}, "device 1 of 0 visible"),
    (["--device-ids", "0,0"], {}, "device 0 of 0 visible"),
    # torchrun's world must match --gpus
    (["--gpus", "2"], {}, "WORLD_SIZE=1"),
])
def test_device_list_arguments(args, env, msg):
    r = _bench(*args, env=env)
    assert r.returncode != 0
    assert msg in (r.stderr + r.stdout), r.stderr[-2000:]
