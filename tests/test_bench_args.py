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


def test_convergence_counts_chains_trapped_mid_run():
    """bench.convergence's trapped rule: more than half of a chain's
    transitions divergent over the run OR over either half of it -- a chain that falls
    into the funnel mid-run (seed 1019 at the hard-geometry profile: 96 % of its
    second-half transitions diverge, 48 % over the run) is counted; R-hat is reported
    with and without such chains, and per-chain bulk ESS next to it."""
    import numpy as np
    sys.path.insert(0, ROOT)
    import bench
    rng = np.random.default_rng(0)
    C, W, S = 40, 10, 400
    cols = ["lp__", "accept_stat__", "stepsize__", "treedepth__", "n_leapfrog__",
            "divergent__", "energy__", "theta.1", "theta.2"]
    d = np.zeros((C, W + S, len(cols)))
    d[:, :, 7:] = rng.standard_normal((C, W + S, 2))
    d[3, W + S // 2:, 5] = 1.0           # chain 3 diverges on its whole second half
    d[3, W + S // 2:, 7] = 8.0           # ... stuck far from the bulk
    d[5, W:, 5] = (rng.random(S) < 0.45).astype(float)   # 45 % everywhere: not trapped
    out = bench.convergence(d, W, cols)
    assert out["stuck_chains"] == 1
    assert out["rhat_max"] > 1.1 and out["rhat_max_excl_stuck"] < 1.02
    assert out["ess_per_chain_min"] > 0
    assert [c for c, _ in out["ess_per_chain_lowest_columns"]][:1] in (["theta.1"], ["theta.2"])


@pytest.mark.parametrize("world,visible,env,want", [
    (8, 8, "", (0, 1, 2, 3, 4, 5, 6, 7)),   # the driver's node: one rank per GPU
    (8, 1, "", (0,) * 8),                   # rehearsal on one GPU: visible ordinals only
    (2, 1, "0,0", (0, 0)),
    (4, 2, "", (0, 1, 0, 1)),
])
def test_device_list_leg_uses_visible_ordinals(world, visible, env, want, monkeypatch):
    """The torchrun line's device-list sub-object (bench._dl_devices): one entry per rank,
    each a visible ordinal, so an 8-rank rehearsal on one GPU populates it instead of
    failing with 'device ordinal out of range' (round 4's profiles/r04_rehearse8.txt)."""
    sys.path.insert(0, ROOT)
    import bench
    monkeypatch.setenv("FITOCT_BENCH_DEVICE_LIST", env)
    assert bench._dl_devices(world, visible) == want


def test_device_list_leg_rejects_invisible_ordinals(monkeypatch):
    sys.path.insert(0, ROOT)
    import bench
    monkeypatch.setenv("FITOCT_BENCH_DEVICE_LIST", "0,3")
    with pytest.raises(ValueError, match="not among the 2 visible"):
        bench._dl_devices(2, 2)
