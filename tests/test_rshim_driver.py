"""The R-free half of the R `.Call` shim (rshim/src/fitoct_drive.c), called through
ctypes as fitoct_R.c calls it from R: plan -> launch -> poll loop (progress lines,
user-interrupt checks) -> wait -> download -> destroy (errors,
threading, ownership; server.R:457-484 progress), and the three methods the R
wrapper routes to the GPU (sample -> Stan CSV, optim, vb -> variational CSV).

CPU: the driver builds against include/fitoct.h and the in-tree libfitoct, exports
its entry points, and passes argument / no-device errors through with nothing called
back.  GPU: a driven run's draws equal a plain Plan.run bit for bit with monotone
progress ending at the total; the CSV files carry those draws in the output layout
and the progress lines decode, through the Shiny parser, to a monotone 0..100; an
interrupt cancels the run (FITOCT_E_CANCELLED) after the kernel drained; optim and vb
match the Python mirror.
"""
from __future__ import annotations

import ctypes as C
import os
import time

import numpy as np
import pytest

from fitoct_amd import _lib
from fitoct_amd.api import ExpGPProblem, Plan, SamplerConfig
from fitoct_amd.synth import default_prior, synth_decay
from rshim import build as rbuild

PROGRESS = C.CFUNCTYPE(None, C.c_void_p, C.c_int64, C.c_int64)
INTERRUPT = C.CFUNCTYPE(C.c_int32, C.c_void_p)
LINE = C.CFUNCTYPE(None, C.c_void_p, C.c_char_p)
_dp = C.POINTER(C.c_double)


def _drive_lib():
    _lib.lib()   # libfitoct first (the driver's NEEDED entry resolves to the same object)
    L = C.CDLL(rbuild.build())
    L.fitoct_drive_sample.restype = C.c_int32
    L.fitoct_drive_sample.argtypes = [C.POINTER(_lib.Problem), C.POINTER(_lib.Config),
                                      C.POINTER(_lib.Result), C.c_int32, PROGRESS, INTERRUPT,
                                      C.c_void_p]
    L.fitoct_drive_sample_csv.restype = C.c_int32
    L.fitoct_drive_sample_csv.argtypes = [C.POINTER(_lib.Problem), C.POINTER(_lib.Config),
                                          C.POINTER(C.c_char_p), C.c_int32, LINE, INTERRUPT,
                                          C.c_void_p]
    L.fitoct_drive_sample_bulk.restype = C.c_int32
    L.fitoct_drive_sample_bulk.argtypes = [C.POINTER(_lib.Problem), C.POINTER(_lib.Config),
                                           _dp, C.c_int64, _dp, _dp, _dp, C.c_int32, LINE,
                                           INTERRUPT, C.c_void_p]
    L.fitoct_drive_bulk_layout.restype = C.c_int32
    L.fitoct_drive_bulk_layout.argtypes = [C.POINTER(_lib.Problem), C.c_int32, C.c_int64, _dp,
                                           _dp]
    L.fitoct_drive_optimize.restype = C.c_int32
    L.fitoct_drive_optimize.argtypes = [C.POINTER(_lib.Problem), C.POINTER(_lib.OptimConfig),
                                        _dp, _dp, _dp, _dp, _dp, _dp, _dp,
                                        C.POINTER(C.c_int32)]
    L.fitoct_drive_vb_csv.restype = C.c_int32
    L.fitoct_drive_vb_csv.argtypes = [C.POINTER(_lib.Problem), C.POINTER(_lib.VbConfig), _dp,
                                      C.c_char_p]
    return L


def _drive_csv(prob, cfg, tmp_path, interrupt=None):
    """fitoct_drive_sample_csv as fitoct_R_sample calls it: (status, paths, lines)."""
    p, c = prob.to_c(), cfg.to_c()
    paths = [str(tmp_path / f"chain_{i + 1}.csv").encode() for i in range(max(cfg.chains, 1))]
    arr = (C.c_char_p * len(paths))(*paths)
    lines = []
    cb_l = LINE(lambda _ctx, line: lines.append(line.decode()))
    cb_i = INTERRUPT(lambda _ctx: int(bool(interrupt and interrupt(lines))))
    rc = _drive_lib().fitoct_drive_sample_csv(C.byref(p), C.byref(c), arr, 5, cb_l, cb_i, None)
    return rc, [q.decode() for q in paths], lines


def _drive(prob, cfg, interrupt_after=None, poll_ms=5):
    """Run the driver; returns (status, draws, progress calls, interrupt polls)."""
    p, c = prob.to_c(), cfg.to_c()
    iters = cfg.warmup + cfg.samples
    draws = np.full((cfg.chains, iters, len(prob.column_names())), np.nan)
    eps = np.empty(cfg.chains)
    r = _lib.Result()
    r.draws = draws.ctypes.data_as(C.POINTER(C.c_double))
    r.draws_capacity = draws.size
    r.stepsize = eps.ctypes.data_as(C.POINTER(C.c_double))
    seen, polls = [], [0]

    def on_progress(_ctx, done, total):
        seen.append((done, total))

    def on_interrupt(_ctx):
        polls[0] += 1
        return int(interrupt_after is not None and bool(seen) and seen[-1][0] >= interrupt_after)

    cb_p, cb_i = PROGRESS(on_progress), INTERRUPT(on_interrupt)
    rc = _drive_lib().fitoct_drive_sample(C.byref(p), C.byref(c), C.byref(r), poll_ms, cb_p,
                                          cb_i, None)
    return rc, draws, seen, polls[0]


def _prob(N=512, Nn=10):
    t0, S0 = default_prior()
    d = synth_decay(N, "sincExp", 3)
    return ExpGPProblem(d["x"], d["y"], d["uy"], Nn=Nn, gridType="extremal", theta0=t0,
                        Sigma0=S0, prior_type="normal")


def test_driver_builds_and_exports():
    L = _drive_lib()
    for f in ("fitoct_drive_sample", "fitoct_drive_sample_csv", "fitoct_drive_optimize",
              "fitoct_drive_vb_csv", "fitoct_drive_sample_bulk", "fitoct_drive_bulk_layout"):
        assert hasattr(L, f)


def _bulk_expected(prob, raw):
    """fitoct_R_sample_bulk's array from raw kernel draws [chains, rows, n_cols]: every
    chain's output-layout rows (stanfit.materialise, the CSV writer's layout) transposed to
    column runs, i.e. R's array(dim = c(rows, n_out, chains)) in memory order."""
    from fitoct_amd.stanfit import materialise
    return np.ascontiguousarray(np.transpose(materialise(raw, prob), (0, 2, 1)))


@pytest.mark.parametrize("family", ["normal", "lasso", "horseshoe"])
def test_bulk_layout_matches_output_rows(family):
    """The host layout step of the bulk route on synthetic raw rows (300 rows, so the
    256-row blocking is crossed): equal to the per-row output layout, transposed."""
    t0, S0 = default_prior()
    d = synth_decay(64, "sincExp", 5)
    prob = ExpGPProblem(d["x"], d["y"], d["uy"], Nn=6, gridType="extremal", theta0=t0,
                        Sigma0=S0, prior_type=family)
    rng = np.random.default_rng(3)
    raw = rng.uniform(0.1, 2.0, (3, 300, len(prob.column_names())))
    want = _bulk_expected(prob, raw)
    out = np.full(want.shape, np.nan)
    p = prob.to_c()
    rc = _drive_lib().fitoct_drive_bulk_layout(C.byref(p), 3, 300, raw.ctypes.data_as(_dp),
                                               out.ctypes.data_as(_dp))
    assert rc == 0
    np.testing.assert_array_equal(out, want)


def test_bulk_driver_argument_errors():
    """chains = 0 -> the library's FITOCT_E_ARG; a too small draws buffer -> FITOCT_E_ARG
    before anything runs (no line, no interrupt poll)."""
    L = _drive_lib()
    prob = _prob(N=64)
    out = np.zeros(10)
    for cfg in (SamplerConfig(chains=0, warmup=5, samples=5),
                SamplerConfig(chains=2, warmup=5, samples=5)):
        p, c = prob.to_c(), cfg.to_c()
        lines = []
        cb_l = LINE(lambda _ctx, line: lines.append(line))
        cb_i = INTERRUPT(lambda _ctx: 0)
        rc = L.fitoct_drive_sample_bulk(C.byref(p), C.byref(c), out.ctypes.data_as(_dp),
                                        out.size, None, None, None, 5, cb_l, cb_i, None)
        assert rc == -1 and lines == []


def test_csv_driver_argument_errors(tmp_path):
    """chains = 0 / samples = 0: FITOCT_E_ARG with the library's message; no line, no file."""
    for bad in (dict(chains=0), dict(samples=0)):
        rc, paths, lines = _drive_csv(_prob(N=64), SamplerConfig(warmup=5, **{"samples": 5, **bad}),
                                      tmp_path)
        assert rc == -1 and lines == []
        assert not any(os.path.exists(q) for q in paths)
    assert b"chains" in _lib.lib().fitoct_last_error() or b"samples" in _lib.lib().fitoct_last_error()


@pytest.mark.skipif(_lib.lib().fitoct_device_count() > 0, reason="a GPU is visible")
def test_csv_driver_no_device(tmp_path):
    rc, paths, lines = _drive_csv(_prob(N=64), SamplerConfig(chains=2, warmup=5, samples=5),
                                  tmp_path)
    assert rc == -3 and lines == []


def test_driver_passes_argument_errors_through():
    """chains = 0: FITOCT_E_ARG from plan creation, nothing launched or called back."""
    rc, _, seen, polls = _drive(_prob(N=64), SamplerConfig(chains=0, warmup=5, samples=5))
    assert rc == -1 and seen == [] and polls == 0
    assert b"chains" in _lib.lib().fitoct_last_error()


@pytest.mark.skipif(_lib.lib().fitoct_device_count() > 0, reason="a GPU is visible")
def test_driver_no_device():
    rc, _, seen, polls = _drive(_prob(N=64), SamplerConfig(chains=2, warmup=5, samples=5))
    assert rc == -3 and seen == [] and polls == 0


@pytest.mark.gpu
def test_driver_matches_plan_and_reports_progress():
    prob = _prob()
    cfg = SamplerConfig(chains=64, warmup=100, samples=100, seed=11, max_treedepth=8)
    rc, draws, seen, polls = _drive(prob, cfg)
    assert rc == 0, _lib.lib().fitoct_last_error()
    total = 64 * 200
    assert seen and seen[-1] == (total, total)
    dones = [d for d, _ in seen]
    assert all(b >= a for a, b in zip(dones, dones[1:])), "progress went backwards"
    assert polls >= 1
    with Plan(prob, cfg) as pl:
        pl.run()
        ref = pl.download()
    assert np.array_equal(draws, ref.draws, equal_nan=True)


@pytest.mark.gpu
def test_driver_interrupt_cancels_and_drains():
    """Sized so that a failed cancellation would still end within ~30 s."""
    prob = _prob()
    cfg = SamplerConfig(chains=32, warmup=100, samples=20000, seed=12, max_treedepth=8)
    t0 = time.time()
    rc, _, seen, polls = _drive(prob, cfg, interrupt_after=32 * 16)
    dt = time.time() - t0
    assert rc == -8
    assert seen and seen[-1][0] < seen[-1][1]
    assert dt < 20.0, f"interrupted run took {dt:.1f} s"
    # the library is usable afterwards (no leaked plan state)
    rc2, _, seen2, _ = _drive(prob, SamplerConfig(chains=4, warmup=20, samples=20, seed=13,
                                                  max_treedepth=6))
    assert rc2 == 0 and seen2[-1] == (160, 160)


@pytest.mark.gpu
@pytest.mark.parametrize("family,prior_PD", [("normal", 0), ("horseshoe", 0), ("lasso", 1)])
def test_csv_driver_matches_plan(tmp_path, family, prior_PD):
    """What fitoct_R_sample hands to rstan::read_stan_csv: per-chain CSV files holding
    a plain Plan.run's draws in the output layout, and rstan-format progress lines the
    Shiny parser (server.R:457-472) reads as a monotone 0..100."""
    import stancsv_reader
    from fitoct_amd.stanfit import StanFit
    from shiny_progress import replay
    t0, S0 = default_prior()
    d = synth_decay(512, "sincExp", 3)
    prob = ExpGPProblem(d["x"], d["y"], d["uy"], Nn=10, gridType="extremal", theta0=t0,
                        Sigma0=S0, prior_type=family, prior_PD=prior_PD)
    cfg = SamplerConfig(chains=4, warmup=150, samples=150, seed=21, max_treedepth=8)
    rc, paths, lines = _drive_csv(prob, cfg, tmp_path)
    assert rc == 0, _lib.lib().fitoct_last_error()
    shown = replay(lines)
    assert lines and shown[-1] == 100 and all(b >= a for a, b in zip(shown, shown[1:]))
    with Plan(prob, cfg) as pl:
        pl.run()
        fit = StanFit.from_output(pl.download(), prob)
    for ch, path in enumerate(paths):
        r = stancsv_reader.read(path)
        assert r["header"] == fit.columns
        assert r["rows_before_adaptation"] == 150
        np.testing.assert_array_equal(r["rows"], fit._draws[ch])
        assert r["stepsize"] == fit.stepsize[ch]
        assert r["times"]["Total"] > 0


@pytest.mark.gpu
def test_csv_driver_interrupt(tmp_path):
    prob = _prob()
    cfg = SamplerConfig(chains=32, warmup=100, samples=20000, seed=12, max_treedepth=8)
    rc, paths, lines = _drive_csv(prob, cfg, tmp_path, interrupt=lambda ls: len(ls) >= 1)
    assert rc == -8
    assert not any(os.path.exists(q) for q in paths)


@pytest.mark.gpu
@pytest.mark.parametrize("family", ["normal", "horseshoe", "monoexp"])
def test_optimize_driver_matches_mirror(family):
    """fitoct_R_optimize's numbers (rstan::optimizing shape after R regroups par) equal
    the Python mirror's: par in the output layout, value, Hessian, m / resid / dL."""
    from fitoct_amd.genquant import expgp_curves
    from fitoct_amd.monoexp import mono_problem
    from fitoct_amd.optim_vb import optimizing
    from fitoct_amd.stanfit import output_columns
    t0, S0 = default_prior()
    d = synth_decay(512, "sincExp", 3)
    if family == "monoexp":
        prob = mono_problem(d["x"], d["y"], d["uy"], 2)
    else:
        prob = ExpGPProblem(d["x"], d["y"], d["uy"], Nn=10, gridType="extremal", theta0=t0,
                            Sigma0=S0, prior_type=family)
    D, N = prob.D, prob.N
    names = output_columns(prob, lead=())
    par, H = np.empty(len(names)), np.empty((D, D))
    dL, m, resid = np.empty(N), np.empty(N), np.empty(N)
    value, code = C.c_double(), C.c_int32()
    oc = _lib.OptimConfig()
    _lib.lib().fitoct_default_optim_config(C.byref(oc))
    p = prob.to_c()
    dp = _lib.dptr
    rc = _drive_lib().fitoct_drive_optimize(C.byref(p), C.byref(oc), None, dp(par), dp(H),
                                            None if family == "monoexp" else dp(dL), dp(m),
                                            dp(resid), C.byref(value), C.byref(code))
    assert rc == 0, _lib.lib().fitoct_last_error()
    ref = optimizing(prob)
    assert value.value == ref.value and code.value == ref.return_code
    np.testing.assert_array_equal(H, ref.hessian)
    flat = np.concatenate([np.atleast_1d(ref.par[k]) for k in dict.fromkeys(
        n.split(".")[0] for n in names)])
    np.testing.assert_array_equal(par, flat)
    ygp = None if family == "monoexp" else ref.par["yGP"]
    g = expgp_curves(prob, ref.par["theta"], ygp)
    np.testing.assert_array_equal(m, g["m"][0])
    np.testing.assert_array_equal(resid, g["resid"][0])
    if family != "monoexp":
        np.testing.assert_array_equal(dL, g["dL"][0])
    assert par[names.index("br")] == pytest.approx(np.mean(resid ** 2), rel=1e-10)


@pytest.mark.gpu
def test_vb_driver_csv(tmp_path):
    """fitoct_R_vb's file: CmdStan variational CSV with the mirror's ADVI draws."""
    import stancsv_reader
    from fitoct_amd.optim_vb import vb
    prob = _prob()
    vc = _lib.VbConfig()
    _lib.lib().fitoct_default_vb_config(C.byref(vc))
    vc.seed = 5
    p = prob.to_c()
    path = str(tmp_path / "vb.csv")
    rc = _drive_lib().fitoct_drive_vb_csv(C.byref(p), C.byref(vc), None, path.encode())
    assert rc == 0, _lib.lib().fitoct_last_error()
    r = stancsv_reader.read(path)
    fit = vb(prob, seed=5)
    assert r["values"]["method"] == "variational"
    assert r["header"] == fit.columns
    np.testing.assert_array_equal(r["rows"][1:], fit._draws[0])
    fit.write_stan_csv(str(tmp_path / "py"))
    r2 = stancsv_reader.read(str(tmp_path / "py" / "chain_vb.csv"))
    np.testing.assert_array_equal(r2["rows"], r["rows"])      # one writer, same file


@pytest.mark.gpu
def test_bulk_driver_at_config4_chain_count():
    """fitExpGP(nb_chains = 8192) through the bulk route (fitoct_R_sample_bulk ->
    fitoct_drive_sample_bulk): config 4's shape (lasso, N = 4096, Nn = 15, 8192 chains;
    short warmup / sampling), the array equals the plan's draws in the output layout
    transposed to R's [rows, n_out, chains] order, step sizes and metrics equal the
    plan's, the elapsed split sums to the kernel time and the progress ends at 100 %."""
    t0, S0 = default_prior()
    d = synth_decay(4096, "sincExp", 1234)
    prob = ExpGPProblem(d["x"], d["y"], d["uy"], Nn=15, gridType="extremal", theta0=t0,
                        Sigma0=S0, prior_type="lasso", lambda_scale=10.0)
    cfg = SamplerConfig(chains=8192, warmup=15, samples=10, seed=1000, max_treedepth=6)
    with Plan(prob, cfg) as pl:
        pl.run()
        ref = pl.download()
    want = _bulk_expected(prob, ref.draws)
    n_out = want.shape[1]
    out = np.full(want.shape, np.nan)
    eps, minv = np.empty(8192), np.empty((8192, prob.D))
    el = np.empty((8192, 2))
    p, c = prob.to_c(), cfg.to_c()
    lines = []
    cb_l = LINE(lambda _ctx, line: lines.append(line.decode()))
    cb_i = INTERRUPT(lambda _ctx: 0)
    rc = _drive_lib().fitoct_drive_sample_bulk(
        C.byref(p), C.byref(c), out.ctypes.data_as(_dp), out.size, eps.ctypes.data_as(_dp),
        minv.ctypes.data_as(_dp), el.ctypes.data_as(_dp), 20, cb_l, cb_i, None)
    assert rc == 0, _lib.lib().fitoct_last_error()
    assert out.shape == (8192, n_out, 25)
    np.testing.assert_array_equal(out, want)
    np.testing.assert_array_equal(eps, ref.stepsize)
    np.testing.assert_array_equal(minv, ref.inv_metric)
    assert np.all(el >= 0) and np.allclose(el.sum(1), el.sum(1)[0])
    assert lines and "100%" in lines[-1]
