"""The device list of the C ABI (fitoct_config.devices; SURVEY.md §8b "device list",
R fitExpGP(n_gpus = k)), which replaces rstan's chain parallelism over host cores,
options(mc.cores = parallel::detectCores()) at FitOCT.R:13 / ShinyInterface/server.R:19.

The box has one GPU, so every multi-device case lists device 0 several times: each
entry is a separate plan (own host thread, own HBM buffers, own launch), exactly as
on distinct GPUs except that the launches share one card.  Asserted: draws, step
sizes, metrics, last positions and leapfrog counts equal a one-device run bit for bit
for even and uneven chain splits, through the Python Plan, the one-shot
fitoct_expgp_sample, the R shim's driver (Stan CSV files) and batch mode; the
in-place and copied (xGMI peer copy) gather into a caller's device buffer; and one
device's failure cancels the others and is the one status returned.
"""
from __future__ import annotations

import ctypes as C
import dataclasses

import numpy as np
import pytest

from fitoct_amd import _lib
from fitoct_amd.api import Batch, ExpGPProblem, Plan, SamplerConfig, sample
from fitoct_amd.synth import MODULATIONS, default_prior, synth_decay

pytestmark = pytest.mark.gpu


def _prob(prior="normal", N=512, Nn=10, seed=3, mod="sincExp"):
    t0, S0 = default_prior()
    d = synth_decay(N, mod, seed)
    return ExpGPProblem(d["x"], d["y"], d["uy"], Nn=Nn, gridType="extremal", theta0=t0,
                        Sigma0=S0, prior_type=prior)


def _same(a, b):
    np.testing.assert_array_equal(a.draws, b.draws)
    np.testing.assert_array_equal(a.stepsize, b.stepsize)
    np.testing.assert_array_equal(a.inv_metric, b.inv_metric)
    np.testing.assert_array_equal(a.last_q, b.last_q)
    assert a.total_leapfrogs == b.total_leapfrogs


@pytest.mark.parametrize("chains,devices", [(64, (0, 0)), (37, (0, 0, 0)), (5, (0,) * 8)])
def test_plan_split_equals_one_device(chains, devices):
    """Even and uneven splits (37 = 13 + 12 + 12; 5 chains over 8 entries use 5)."""
    prob = _prob("horseshoe", 700, 10)
    cfg = SamplerConfig(chains=chains, warmup=80, samples=60, seed=31, max_treedepth=8,
                        chain_offset=11)
    ref = sample(prob, cfg)
    multi = dataclasses.replace(cfg, devices=devices)
    with Plan(prob, multi) as pl:
        assert pl.info["n_devices"] == min(len(devices), chains)
        assert pl.info["chains"] == chains
        assert pl.info["draws_bytes"] == ref.draws.nbytes
        pl.run()
        out = pl.download()
    _same(out, ref)


def test_progress_and_cancel_over_devices():
    """poll sums the devices' transitions; cancel stops every device (FITOCT_E_CANCELLED)."""
    prob = _prob()
    cfg = SamplerConfig(chains=24, warmup=50, samples=50, seed=5, max_treedepth=6,
                        devices=(0, 0, 0))
    seen = []
    with Plan(prob, cfg) as pl:
        pl.run(progress=lambda d, t: seen.append((d, t)), poll_s=0.01)
        pl.download()
    assert seen[-1] == (24 * 100, 24 * 100)
    assert all(b[0] >= a[0] for a, b in zip(seen, seen[1:]))
    long = dataclasses.replace(cfg, samples=200000)
    with Plan(prob, long) as pl:
        pl.launch()
        pl.cancel()
        pl.wait()
        with pytest.raises(_lib.FitOCTError) as ei:
            pl.download()
    assert ei.value.code == -8


def test_one_shot_expgp_sample_equals_one_device():
    """fitoct_expgp_sample (the entry the R shim's documentation names) with a device
    list: per-device host threads, draws in the caller's host buffer in chain order."""
    prob = _prob("lasso", 900, 12)
    cfg = SamplerConfig(chains=33, warmup=60, samples=40, seed=8)
    ref = sample(prob, cfg)

    def one_shot(c):
        p, cc = prob.to_c(), c.to_c()
        D = prob.D
        draws = np.full(ref.draws.shape, np.nan)
        eps, minv, lq = np.empty(c.chains), np.empty((c.chains, D)), np.empty((c.chains, D))
        st = np.full(c.chains, 99, dtype=np.int32)
        r = _lib.Result()
        r.draws, r.draws_capacity = _lib.dptr(draws), draws.size
        r.stepsize, r.inv_metric, r.last_q = _lib.dptr(eps), _lib.dptr(minv), _lib.dptr(lq)
        r.chain_status = st.ctypes.data_as(C.POINTER(C.c_int32))
        _lib.check(_lib.lib().fitoct_expgp_sample(C.byref(p), C.byref(cc), C.byref(r)))
        assert (st == 0).all()
        return draws, eps, minv, lq, r.total_leapfrogs

    a = one_shot(cfg)
    b = one_shot(dataclasses.replace(cfg, devices=(0, 0, 0, 0)))
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)
    np.testing.assert_array_equal(a[0], ref.draws)


@pytest.mark.parametrize("force_copy", [False, True])
def test_gather_into_caller_device_buffer(monkeypatch, force_copy):
    """d_draws on the caller's device: blocks on that device are written in place, the
    others are copied peer-to-peer (FITOCT_GATHER_COPY=1 takes the copy path on one GPU).
    The env knob is read once per process, so the copy case runs in a child process."""
    if force_copy:
        import subprocess
        import sys
        code = ("import sys; sys.path.insert(0, 'tests'); import test_gpu_multidevice as t; "
                "t._gather_case()")
        env = dict(__import__("os").environ, FITOCT_GATHER_COPY="1")
        r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True,
                           text=True, timeout=300)
        assert r.returncode == 0, r.stdout + r.stderr
        return
    _gather_case()


def _gather_case():
    import torch
    prob = _prob("normal", 600, 10)
    cfg = SamplerConfig(chains=20, warmup=50, samples=50, seed=12)
    ref = sample(prob, cfg)
    with Plan(prob, dataclasses.replace(cfg, devices=(0, 0))) as pl:
        buf = torch.full((pl.info["draws_bytes"] // 8,), float("nan"), dtype=torch.float64,
                         device="cuda")
        pl.run(d_draws=buf.data_ptr())
        got = buf.view(ref.draws.shape).cpu().numpy()
        with pytest.raises(_lib.FitOCTError) as ei:   # multi-device: default streams only
            pl.run(d_draws=buf.data_ptr(), stream=torch.cuda.Stream().cuda_stream)
        assert ei.value.code == -1
    np.testing.assert_array_equal(got, ref.draws)


def test_one_device_failure_cancels_the_others():
    """Every chain on device 0 fails at once (non-finite given start: FITOCT_E_INIT).
    The library then cancels device 1's chains (100k iterations each, queued behind
    device 0 on the same GPU) instead of letting them run on, and the call returns the
    failing device's status, not the cancellation."""
    import time
    prob = _prob()
    base = SamplerConfig(chains=8, warmup=30, samples=30, seed=3, max_treedepth=6)
    prev = sample(prob, base)
    q = prev.last_q.copy()
    q[:4, 0] = 800.0   # theta1 = exp(800): lp = -inf on chains 0-3 (device 0's block)
    cfg = dataclasses.replace(base, warmup=0, samples=100000, adapt_engaged=False,
                              devices=(0, 0))
    t0 = time.time()
    with Plan(prob, cfg) as pl:
        pl.set_init(q, prev.stepsize, prev.inv_metric)
        pl.run()
        r = _lib.Result()
        st = np.zeros(8, dtype=np.int32)
        r.chain_status = st.ctypes.data_as(C.POINTER(C.c_int32))
        rc = _lib.lib().fitoct_plan_download(pl._h, C.byref(r))
    assert rc == -4, _lib.lib().fitoct_last_error()
    assert (st[:4] == -4).all() and (st[4:] == -8).all(), st
    assert time.time() - t0 < 60


def test_batch_split_equals_one_device():
    """FitOCT.R batch mode (config 5) over a device list: 7 files in blocks 3 + 2 + 2,
    every file's draws equal the one-device batch."""
    t0, S0 = default_prior()
    probs = []
    for f in range(7):
        d = synth_decay(481, MODULATIONS[f % 4], 1234 + f)
        probs.append(ExpGPProblem(d["x"], d["y"], d["uy"], Nn=15, gridType="extremal",
                                  theta0=t0, Sigma0=S0, prior_type="normal"))
    cfg = SamplerConfig(chains=4, warmup=60, samples=60, seed=2000, chain_offset=40)
    with Batch(probs, cfg) as b:
        b.run()
        ref = [b.download(p) for p in range(len(probs))]
    import torch
    with Batch(probs, dataclasses.replace(cfg, devices=(0, 0, 0))) as b:
        assert b.info["n_devices"] == 3 and b.info["chains"] == 28
        buf = torch.full((b.info["draws_bytes"] // 8,), float("nan"), dtype=torch.float64,
                         device="cuda")
        b.run(d_draws=buf.data_ptr())
        got = [b.download(p) for p in range(len(probs))]
        dev = buf.view(len(probs), *ref[0].draws.shape).cpu().numpy()
    for p in range(len(probs)):
        _same(got[p], ref[p])
        np.testing.assert_array_equal(dev[p], ref[p].draws)
        assert got[p].chain_offset == ref[p].chain_offset == 40 + 4 * p


def test_rshim_driver_csv_over_devices(tmp_path):
    """fitoct_drive_sample_csv (what fitoct_R_sample calls for fitExpGP(n_gpus = 2)):
    the per-chain Stan CSV files hold the one-device draws."""
    import stancsv_reader
    from test_rshim_driver import _drive_csv
    prob = _prob("horseshoe", 512, 10)
    cfg = SamplerConfig(chains=5, warmup=100, samples=100, seed=21, max_treedepth=8)
    (tmp_path / "one").mkdir()
    (tmp_path / "two").mkdir()
    rc1, p1, lines1 = _drive_csv(prob, cfg, tmp_path / "one")
    rc2, p2, lines2 = _drive_csv(prob, dataclasses.replace(cfg, devices=(0, 0)), tmp_path / "two")
    assert rc1 == 0 and rc2 == 0, _lib.lib().fitoct_last_error()
    assert lines2 and lines2[-1] == lines1[-1]
    for a, b in zip(p1, p2):
        ra, rb = stancsv_reader.read(a), stancsv_reader.read(b)
        assert ra["header"] == rb["header"]
        np.testing.assert_array_equal(ra["rows"], rb["rows"])
        assert ra["stepsize"] == rb["stepsize"]
        np.testing.assert_array_equal(ra["inv_metric"], rb["inv_metric"])


def test_fitexpgp_n_gpus():
    """fitExpGP(..., n_gpus=k) (the Python mirror of the R argument) takes devices
    0..k-1: every GPU of this box gives the one-device draws, an explicit repeated list
    too, and asking for more GPUs than exist is FITOCT_E_ARG naming the device."""
    from fitoct_amd.api import fitExpGP
    p = _prob("normal", 400, 8)
    kw = dict(dataType=2, Nn=8, gridType="extremal", theta0=p.theta0, Sigma0=p.Sigma0,
              nb_warmup=60, nb_iter=120, nb_chains=6, seed=77, refresh=0)
    n = _lib.lib().fitoct_device_count()
    a = fitExpGP(p.x, p.y, p.uy, **kw)
    b = fitExpGP(p.x, p.y, p.uy, n_gpus=n, **kw)
    c = fitExpGP(p.x, p.y, p.uy, devices=(0, 0, 0), **kw)
    np.testing.assert_array_equal(a["fit"]._draws, b["fit"]._draws)
    np.testing.assert_array_equal(a["fit"]._draws, c["fit"]._draws)
    with pytest.raises(_lib.FitOCTError) as ei:
        fitExpGP(p.x, p.y, p.uy, n_gpus=n + 1, **kw)
    assert ei.value.code == -1 and f"device {n}" in str(ei.value)


def test_in_place_shards_wait_for_callers_null_stream_work():
    """Ordering rule (include/fitoct.h, fitoct_plan_run): the in-place shards run on
    private non-blocking streams, yet start only after the work the caller queued on the
    buffer device's NULL stream.  Slow FP64 matmuls and then a NaN fill of the buffer are
    queued on torch's default (NULL) stream right before run(): without the library's
    fence the fill would land on top of the draws."""
    import torch
    prob = _prob("normal", 600, 10)
    cfg = SamplerConfig(chains=16, warmup=40, samples=40, seed=19)
    ref = sample(prob, cfg)
    assert torch.cuda.current_stream().cuda_stream == 0   # torch's default = NULL stream
    with Plan(prob, dataclasses.replace(cfg, devices=(0, 0))) as pl:
        buf = torch.zeros(pl.info["draws_bytes"] // 8, dtype=torch.float64, device="cuda")
        x = torch.randn(4096, 4096, dtype=torch.float64, device="cuda")
        torch.cuda.synchronize()
        for _ in range(8):   # ~0.1 s of NULL-stream work ahead of the fill
            x = (x @ x) * 1e-4
        buf.fill_(float("nan"))
        pl.run(d_draws=buf.data_ptr())
        got = buf.view(ref.draws.shape).cpu().numpy()
    np.testing.assert_array_equal(got, ref.draws)


def test_batch_device_failure_cancels_the_others():
    """A multi-device batch whose entry 0 fails (FITOCT_TEST_FAIL_ENTRY=0, read once per
    process, so in a child) returns that status, and the other entries' chains (100k
    iterations each) are cancelled at a transition boundary instead of running on."""
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, 'tests'); import test_gpu_multidevice as t; "
            "t._batch_fail_case()")
    env = dict(__import__("os").environ, FITOCT_TEST_FAIL_ENTRY="0")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr


def _batch_fail_case():
    import time
    t0, S0 = default_prior()
    probs = []
    for f in range(4):
        d = synth_decay(481, MODULATIONS[f % 4], 1234 + f)
        probs.append(ExpGPProblem(d["x"], d["y"], d["uy"], Nn=15, gridType="extremal",
                                  theta0=t0, Sigma0=S0, prior_type="normal"))
    cfg = SamplerConfig(chains=4, warmup=50, samples=100000, seed=7, devices=(0, 0))
    start = time.time()
    with Batch(probs, cfg) as b:
        with pytest.raises(_lib.FitOCTError) as ei:
            b.run()
    assert ei.value.code == -7 and "injected" in str(ei.value), str(ei.value)
    assert time.time() - start < 60


def test_set_init_checks_every_block_before_any_device():
    """A warm-restart block rejected on device entry 1 (NaN start) leaves entry 0's
    block unset too: the plan then runs from the default start, as one device would."""
    prob = _prob()
    cfg = SamplerConfig(chains=8, warmup=20, samples=20, seed=4, max_treedepth=6)
    ref = sample(prob, cfg)
    with Plan(prob, dataclasses.replace(cfg, devices=(0, 0))) as pl:
        q = np.zeros((8, prob.D))
        q[6, 0] = np.nan                   # chain 6: entry 1's block (chains 4..7)
        with pytest.raises(_lib.FitOCTError) as ei:
            pl.set_init(q_init=q, stepsize=np.full(8, 0.1))
        assert ei.value.code == -1 and "q_init" in str(ei.value)
        pl.run()
        out = pl.download()
    _same(out, ref)
