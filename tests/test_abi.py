"""The drop-in boundary (include/fitoct.h) without a GPU: the library loads,
exports every declared symbol, struct layouts agree with the ctypes mirror,
host-side helpers (basis, names, diagnostics) agree with the oracles, and the
error contract holds (negative status + message, no exception crossing the ABI).
"""
from __future__ import annotations

import ctypes as C
import os
import re

import numpy as np
import pytest

from conftest import ROOT, golden_files, load_golden, problems_from_fixture
from fitoct_amd import _lib
from fitoct_amd.api import ExpGPProblem, SamplerConfig
from oracle import diag_np
from oracle import model_np as M

HEADER = os.path.join(ROOT, "include", "fitoct.h")


def header_symbols():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(fitoct_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_header_symbol():
    L = _lib.lib()
    syms = header_symbols()
    assert len(syms) >= 19
    for s in syms:
        assert hasattr(L, s), f"libfitoct.so does not export {s}"
    assert sorted(n for n, _, _ in _lib.SIGNATURES) == syms


def test_exports_are_c_linkage():
    out = os.popen(f"nm -D --defined-only {_lib.LIB_PATH}").read()
    exported = set(re.findall(r"\b(fitoct_[a-z0-9_]+)$", out, flags=re.M))
    assert set(header_symbols()) <= exported


def test_struct_layouts_match_ctypes():
    sizes = _lib.struct_sizes()
    assert sizes == (C.sizeof(_lib.Problem), C.sizeof(_lib.Config), C.sizeof(_lib.Result),
                     C.sizeof(_lib.PlanInfo))
    assert _lib.lib().fitoct_abi_version() == 8 == _lib.ABI_VERSION


def test_default_config_is_stan_default():
    c = _lib.Config()
    _lib.lib().fitoct_default_config(C.byref(c))
    assert (c.chains, c.warmup, c.samples, c.max_treedepth) == (4, 500, 1000, 10)
    assert (c.adapt_delta, c.gamma, c.kappa, c.t0) == (0.8, 0.05, 0.75, 10.0)
    assert (c.init_buffer, c.term_buffer, c.window) == (75, 50, 25)
    assert c.init_radius == 2.0 and c.save_warmup == 1 and c.adapt_engaged == 1
    p = _lib.Problem()
    _lib.lib().fitoct_default_problem(C.byref(p))
    assert list(p.theta0) == [1000.0, 2000.0, 300.0] and p.lambda_rate == 0.1
    assert p.Sigma0[0] == pytest.approx(2500.0) and p.Sigma0[1] == 0.0
    assert p.theta_prior == 0   # ABI 5: the model's own theta prior unless asked


@pytest.mark.parametrize("fam", ["normal", "lasso", "horseshoe"])
@pytest.mark.parametrize("Nn", [5, 15, 24])
def test_dims_and_column_names(fam, Nn):
    code = _lib.PRIOR[fam]
    L = _lib.lib()
    D = M.dim(code, Nn)
    assert L.fitoct_dim(code, Nn) == D
    cols = _lib.column_names(code, Nn)
    assert len(cols) == D + 8 == L.fitoct_n_cols(code, Nn)
    assert cols[:7] == ["lp__", "accept_stat__", "stepsize__", "treedepth__", "n_leapfrog__",
                        "divergent__", "energy__"]
    # constrained parameters in model order, Stan's flattened naming (plotExpGP.R:41)
    want = [n.replace("[", ".").replace("]", "") for n in M.param_names(code, Nn)]
    assert cols[7:7 + D] == want and cols[-1] == "br"


def test_column_name_errors():
    buf = C.create_string_buffer(4)
    L = _lib.lib()
    assert L.fitoct_column_name(0, 5, 10_000, buf, 4) == -1
    assert L.fitoct_column_name(0, 5, 1, buf, 4) == -1          # "accept_stat__" > 4 bytes
    assert b"buffer" in L.fitoct_last_error()
    assert L.fitoct_dim(7, 5) < 0


@pytest.mark.parametrize("path", golden_files("logp"), ids=lambda p: os.path.basename(p))
def test_build_basis_matches_oracle(path):
    fx = load_golden(path)
    if fx["meta"]["family"] == "monoexp":
        pytest.skip("no GP basis in the mono-exponential model")
    prob, _ = problems_from_fixture(fx)
    B, xg = prob.basis()
    np.testing.assert_allclose(B, fx["B"], rtol=0, atol=1e-11)
    np.testing.assert_allclose(xg, fx["xGP"], atol=1e-15)


def _ar1(rng, chains, n, phi, shift=None):
    x = np.zeros((chains, n))
    e = rng.standard_normal((chains, n))
    for t in range(1, n):
        x[:, t] = phi * x[:, t - 1] + e[:, t]
    if shift is not None:
        x += np.asarray(shift)[:, None]
    return x


@pytest.mark.parametrize("case", ["iid", "ar1", "ar1_neg", "shifted", "short", "odd"])
def test_split_rhat_ess_matches_restatement(case):
    rng = np.random.Generator(np.random.PCG64(4))
    x = {"iid": lambda: rng.standard_normal((4, 1000)),
         "ar1": lambda: _ar1(rng, 4, 1000, 0.9),
         "ar1_neg": lambda: _ar1(rng, 8, 500, -0.5),
         "shifted": lambda: _ar1(rng, 4, 400, 0.3, shift=[0, 0, 0, 1.5]),
         "short": lambda: rng.standard_normal((2, 20)),
         "odd": lambda: _ar1(rng, 3, 301, 0.6)}[case]()
    from fitoct_amd.stanfit import split_rhat_ess
    r, e = split_rhat_ess(x)
    assert r == pytest.approx(diag_np.split_rhat(x), rel=1e-10)
    assert e == pytest.approx(diag_np.split_ess(x), rel=1e-8)


def test_rank_rhat_detects_nonmixing():
    from fitoct_amd.stanfit import rank_rhat
    rng = np.random.Generator(np.random.PCG64(1))
    good = rng.standard_normal((4, 500))
    bad = good + np.array([0, 0, 0, 3.0])[:, None]
    assert rank_rhat(good) < 1.01
    assert rank_rhat(bad) > 1.1


def test_problem_validation_before_device():
    """Argument errors are reported as FITOCT_E_ARG even without a device."""
    x = np.linspace(20, 500, 16)
    prob = ExpGPProblem(x, x * 0 + 1000, x * 0 + 1.0, Nn=5)
    prob.uy[3] = 0.0
    with pytest.raises(_lib.FitOCTError) as ei:
        from fitoct_amd.api import logp_grad
        logp_grad(prob, np.zeros((1, prob.D)))
    assert ei.value.code == -1 and "uy > 0" in str(ei.value)
    prob.uy[3] = 1.0
    prob.Nn = 30
    p = prob.to_c()
    assert _lib.lib().fitoct_build_basis(C.byref(p), None, None) == -1


def test_config_validation():
    from fitoct_amd.api import Plan
    x = np.linspace(20, 500, 16)
    prob = ExpGPProblem(x, x * 0 + 1000, x * 0 + 1.0, Nn=5)
    for bad in [dict(chains=0), dict(samples=0), dict(max_treedepth=17), dict(adapt_delta=1.0),
                dict(stepsize=0.0)]:
        with pytest.raises(_lib.FitOCTError) as ei:
            Plan(prob, SamplerConfig(**bad))
        assert ei.value.code == -1


@pytest.mark.skipif(_lib.lib().fitoct_device_count() > 0, reason="a GPU is visible")
def test_no_device_fails_loudly():
    """No CPU fallback: without a HIP device the sampler returns FITOCT_E_NODEVICE."""
    x = np.linspace(20, 500, 16)
    prob = ExpGPProblem(x, x * 0 + 1000, x * 0 + 1.0, Nn=5)
    with pytest.raises(_lib.FitOCTError) as ei:
        from fitoct_amd.api import sample
        sample(prob, SamplerConfig(chains=1, warmup=5, samples=5))
    assert ei.value.code == -3


def test_missing_library_raises(monkeypatch, tmp_path):
    monkeypatch.setattr(_lib, "_LIB", None)
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "libfitoct.so"))
    with pytest.raises(ImportError):
        _lib.lib()


@pytest.mark.parametrize("case", ["constant_x", "one_bin", "nan_y", "inf_x", "neg_uy"])
def test_degenerate_inputs_rejected(case):
    """Degenerate data (SURVEY.md §8 edge cases: empty / ragged / non-finite) fail with
    FITOCT_E_ARG and a message, before any device work."""
    from fitoct_amd.api import logp_grad
    x = np.linspace(20, 500, 16)
    y, uy = 1000 + 0 * x, 1 + 0 * x
    if case == "constant_x":
        x = 0 * x + 20.0
    elif case == "one_bin":
        x, y, uy = x[:1], y[:1], uy[:1]
    elif case == "nan_y":
        y = y.copy()
        y[5] = np.nan
    elif case == "inf_x":
        x = x.copy()
        x[0] = np.inf
    else:
        uy = uy.copy()
        uy[2] = -1.0
    prob = ExpGPProblem(x, y, uy, Nn=5)   # no Python-side value checks: the ABI must refuse
    with pytest.raises(_lib.FitOCTError) as ei:
        logp_grad(prob, np.zeros((1, prob.D)))
    assert ei.value.code == -1 and len(str(ei.value)) > 0


def test_oversize_n_rejected():
    """N above FITOCT_MAX_BINS (include/fitoct.h) fails with FITOCT_E_ARG before any
    allocation sized by N, with or without a device."""
    hdr = open(HEADER).read()
    max_bins = eval(re.search(r"#define FITOCT_MAX_BINS \((.*)\)", hdr).group(1))
    from fitoct_amd.api import logp_grad
    x = np.linspace(20.0, 500.0, max_bins + 1)
    prob = ExpGPProblem(x, 1000.0 + 0 * x, 1.0 + 0 * x, Nn=5)
    with pytest.raises(_lib.FitOCTError) as ei:
        logp_grad(prob, np.zeros((1, prob.D)))
    assert ei.value.code == -1 and "FITOCT_MAX_BINS" in str(ei.value)
    out = np.empty(3)
    assert _lib.lib().fitoct_mono_initial_theta(max_bins + 1, _lib.dptr(x), _lib.dptr(x), 2,
                                                _lib.dptr(out)) == -1


def test_set_init_needs_a_plan():
    """fitoct_plan_set_init (warm restart) reports a NULL plan as FITOCT_E_ARG."""
    L = _lib.lib()
    assert L.fitoct_plan_set_init(None, None, None, None) == -1
    assert b"plan" in L.fitoct_last_error()


def _tiny_problem():
    x = np.linspace(20, 500, 16)
    return ExpGPProblem(x, x * 0 + 1000, x * 0 + 1.0, Nn=5)


@pytest.mark.parametrize("devices,n_override,msg", [
    ((0,) * 17, None, "n_devices"),          # more than FITOCT_MAX_DEVICES
    ((0, -1), None, "negative"),             # a negative ordinal
    ((0, 1), -2, "n_devices"),               # n_devices < 0
])
def test_device_list_argument_errors(devices, n_override, msg):
    """fitoct_config.devices (SURVEY.md §8b device list): a bad list is FITOCT_E_ARG with a
    message, before any device is touched (so also on a host without a GPU)."""
    from fitoct_amd.api import Plan
    L = _lib.lib()
    cfg = SamplerConfig(chains=8, warmup=5, samples=5)
    c = cfg.to_c()
    n = len(devices) if n_override is None else n_override
    c.n_devices = n
    for i, d in enumerate(devices[:_lib.MAX_DEVICES]):
        c.devices[i] = d
    p = _tiny_problem().to_c()
    h = C.c_void_p()
    assert L.fitoct_plan_create(C.byref(p), C.byref(c), C.byref(h)) == -1
    assert msg in L.fitoct_last_error().decode()
    assert not h.value
    assert L.fitoct_expgp_sample(C.byref(p), C.byref(c), None) == -1
    arr = (_lib.Problem * 2)(p, p)
    assert L.fitoct_batch_create(arr, 2, C.byref(c), C.byref(h)) == -1
    if n_override is None and len(devices) <= _lib.MAX_DEVICES:
        with pytest.raises(_lib.FitOCTError) as ei:
            Plan(_tiny_problem(), SamplerConfig(chains=8, warmup=5, samples=5, devices=devices))
        assert ei.value.code == -1
    with pytest.raises(ValueError):
        SamplerConfig(devices=(0,) * 17).to_c()


@pytest.mark.skipif(_lib.lib().fitoct_device_count() > 0, reason="a GPU is visible")
@pytest.mark.parametrize("entry", ["plan", "sample", "batch"])
def test_device_list_without_gpu_fails_per_device(entry):
    """The per-device host threads report their failure to the caller's thread
    (fitoct_last_error is thread-local): FITOCT_E_NODEVICE naming the device."""
    from fitoct_amd.api import Batch, Plan, sample
    cfg = SamplerConfig(chains=5, warmup=5, samples=5, devices=(0, 0, 0))
    with pytest.raises(_lib.FitOCTError) as ei:
        if entry == "plan":
            Plan(_tiny_problem(), cfg)
        elif entry == "sample":
            sample(_tiny_problem(), cfg)
        else:
            Batch([_tiny_problem()] * 4, cfg)
    assert ei.value.code == -3 and "device 0" in str(ei.value) and "no HIP device" in str(ei.value)


@pytest.mark.parametrize("kw,msg", [
    (dict(prior_type="normal", theta_prior=1), "mono-exponential model's switch"),
    (dict(prior_type="monoexp", theta_prior=2), "theta_prior must be 0 or 1"),
    (dict(prior_type="monoexp", theta_prior=1, lambda_scale=0.0), "lambda_scale"),
    (dict(prior_type="monoexp", prior_PD=1), "flat prior"),   # improper without theta_prior
])
def test_theta_prior_switch_validation(kw, msg):
    """theta_prior (ABI 5, Tests/testGamma.R's model on the mono-exponential family) is
    checked before any device work."""
    from fitoct_amd.api import logp_grad
    x = np.linspace(20, 500, 16)
    prob = ExpGPProblem(x, 1000 + 0 * x, 1 + 0 * x, Nn=5, **kw)
    with pytest.raises(_lib.FitOCTError) as ei:
        logp_grad(prob, np.zeros((1, prob.D)))
    assert ei.value.code == -1 and msg in str(ei.value)


def test_theta_prior_oracles_agree():
    """The exponential theta prior in the C oracle and the numpy restatement: lp and
    gradient agree, and differ from the flat prior by -(1/lambda_scale) sum(theta)."""
    from oracle import model_np as M
    from oracle import nuts_c
    x = np.linspace(20, 500, 16)
    rng = np.random.default_rng(4)
    for pd in (0, 1):
        prob = ExpGPProblem(x, 1000 + 50 * rng.standard_normal(16), 30 + 0 * x, Nn=2,
                            prior_type="monoexp", theta_prior=1, prior_PD=pd, lambda_scale=10.0,
                            theta0=np.array([900.0, 1800.0, 250.0]))
        npp = M.Problem(prob.x, prob.y, prob.uy, Nn=2, family=M.MONOEXP, prior_PD=pd,
                        theta_prior=1, lambda_scale=10.0, theta0=prob.theta0)
        flat = M.Problem(prob.x, prob.y, prob.uy, Nn=2, family=M.MONOEXP, prior_PD=pd,
                         theta0=prob.theta0)
        q = np.log(prob.theta0) + 0.1 * rng.standard_normal((3, 3))
        lp_c, g_c, _ = nuts_c.logp_grad(prob, q)
        for i in range(3):
            lp_n, g_n, _ = M.logp_grad(q[i], npp)
            lp_f, g_f, _ = M.logp_grad(q[i], flat)
            assert lp_c[i] == pytest.approx(lp_n, rel=1e-12, abs=1e-9)
            np.testing.assert_allclose(g_c[i], g_n, rtol=1e-10, atol=1e-10)
            th = np.exp(q[i])
            if pd:   # flat prior + likelihood off: only the Jacobian remains
                assert lp_n == pytest.approx(q[i].sum() - th.sum() / 10.0, rel=1e-12)
            else:
                assert lp_n - lp_f == pytest.approx(-th.sum() / 10.0, rel=1e-10)


@pytest.mark.parametrize("status,report", [
    ([0, 0, 0], -1),
    ([0, -6, 0], 1),                 # a timeout
    ([-8, -8, -6, -8], 2),           # its own failure before the cancellations it caused
    ([-8, 0, -8], 0),                # cancelled only (fitoct_plan_cancel)
    ([0, -4, -6], 1),                # the first own failure (init) wins
])
def test_chain_outcome_timeout_bookkeeping(status, report):
    """fitoct_plan_download's host bookkeeping (no kernel needed): a chain whose status is
    FITOCT_E_TIMEOUT (a real-time bounded wait in the kernel expired) reports NaN
    warm-restart outputs (fitoct_plan_set_init rejects a non-finite start); every other chain's outputs
    are left as the kernel wrote them; the call reports the first chain's own failure
    before any cancellation."""
    L = _lib.lib()
    f = L.fitoct_internal_chain_outcome
    f.restype = C.c_int32
    Cn, D = len(status), 3
    st = np.array(status, dtype=np.int32)
    eps = np.arange(1, Cn + 1, dtype=np.float64)
    minv = np.ones((Cn, D))
    q = np.full((Cn, D), 2.0)
    r = f(Cn, D, st.ctypes.data_as(C.POINTER(C.c_int32)), _lib.dptr(eps), _lib.dptr(minv),
          _lib.dptr(q))
    assert r == report
    tim = st == -6   # FITOCT_E_TIMEOUT
    assert np.all(np.isnan(eps[tim])) and np.all(np.isnan(minv[tim])) and np.all(np.isnan(q[tim]))
    assert np.all(eps[~tim] == np.arange(1, Cn + 1)[~tim])
    assert np.all(minv[~tim] == 1.0) and np.all(q[~tim] == 2.0)
    # NULL outputs are allowed
    assert f(Cn, D, st.ctypes.data_as(C.POINTER(C.c_int32)), None, None, None) == report
