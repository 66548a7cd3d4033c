"""Upstream preparation (fitoct_amd.prep): selX,
estimateNoise (smoothing spline at a given df + ML noise model), estimateExpPrior
and Courbe.csv I/O, plus the FitOCT.R control-file handling of the pipeline.
FitOCTLib is absent: these check the restated behaviour against
properties and known answers ("parity unpinned" vs FitOCTLib)."""
from __future__ import annotations

import numpy as np
import pytest

from fitoct_amd import prep
from fitoct_amd.pipeline import DEFAULT_CTRL, load_ctrl
from fitoct_amd.synth import synth_decay

# ctrlParams.yaml of the reference (5 data lines), as a fixture
CTRL_YAML = "nb_warmup: 100\nnb_sample: 100\ngridType: extremal\nNn: 15\nrho_scale: 0\n"


def test_selx_window_and_subsample():
    x = np.arange(0.0, 600.0)
    y = 2 * x
    c = prep.selX(x, y, (20, 500), 3)
    assert c["x"][0] == 20 and c["x"][-1] <= 500
    assert np.all(np.diff(c["x"]) == 3)
    np.testing.assert_array_equal(c["y"], 2 * c["x"])
    np.testing.assert_array_equal(prep.selX(x, y)["x"], x)
    with pytest.raises(ValueError):
        prep.selX(x, y[:-1])


@pytest.mark.parametrize("df", [2.5, 5, 15, 30])
def test_smoothing_spline_df_and_linear_invariance(df):
    x = np.linspace(20, 500, 200)
    S = prep.SmoothingSpline(x)
    lam = S.lam_for_df(df)
    assert abs(S.df(lam) - df) < 1e-8
    # the penalty (integral of f''^2) is zero on lines: any df reproduces a line
    line = 3.0 - 0.01 * x
    ys, _ = S.fit(line, df)
    np.testing.assert_allclose(ys, line, atol=1e-8)


def test_smoothing_spline_limits():
    rng = np.random.default_rng(0)
    x = np.sort(rng.uniform(0, 10, 80))
    y = np.sin(x) + rng.normal(0, 0.1, x.size)
    S = prep.SmoothingSpline(x)
    lo, _ = S.fit(y, 2.0001)                       # -> least-squares line
    coef = np.polyfit(x, y, 1)
    np.testing.assert_allclose(lo, np.polyval(coef, x), atol=1e-3)
    hi, _ = S.fit(y, x.size - 1e-4)                # -> interpolation
    np.testing.assert_allclose(hi, y, atol=1e-3)
    mid = prep.smooth_spline(x, y, 8)
    assert np.std(y - mid) < np.std(y - lo)


def test_estimate_noise_recovers_noise_model():
    # known a1, a2: uy = a1 exp(-x/a2) around a smooth decay (ui.R:81)
    a1, a2 = 20.0, 250.0
    x = np.linspace(20, 500, 2000)
    truth = 1000 + 2000 * np.exp(-x / 150)
    rng = np.random.default_rng(3)
    y = truth + rng.normal(0, 1, x.size) * a1 * np.exp(-x / a2)
    out = prep.estimateNoise(x, y, df=15)
    assert abs(out["theta"][0] / a1 - 1) < 0.1
    assert abs(out["theta"][1] / a2 - 1) < 0.1
    np.testing.assert_allclose(out["uy"], out["theta"][0] * np.exp(-x / out["theta"][1]))
    assert np.std(out["ySmooth"] - truth) < 0.2 * a1


def test_estimate_noise_on_synthdata_decay():
    d = synth_decay(481, "sincExp", 5)
    out = prep.estimateNoise(d["x"], d["y"], 15)
    ratio = out["uy"] / d["uy"]       # synthData.R:23 noise sd, close to a1 exp(-x/a2)
    assert 0.8 < np.median(ratio) < 1.2


def test_estimate_exp_prior_mono_and_abc():
    th = np.array([1000.0, 2000.0, 300.0])
    cor = np.array([[1, 0.3, -0.2], [0.3, 1, 0.1], [-0.2, 0.1, 1]])
    out = {"best.theta": th, "cor.theta": cor}
    x = np.linspace(20, 500, 481)
    uy = 20 * np.exp(-x / 300)
    m = prep.estimateExpPrior(x, uy, 2, "mono", out=out, ru_theta=0.05)
    D = np.diag(0.05 * th)
    np.testing.assert_allclose(m["Sigma0"], D @ cor @ D)
    np.testing.assert_array_equal(m["theta0"], th)
    a = prep.estimateExpPrior(x, uy, 2, "abc", out=out, eps=1e-3, n_sim=100_000)
    assert a["accepted"] == 100
    assert np.all(np.abs(a["theta0"] / th - 1) < 0.05)
    assert np.all(np.linalg.eigvalsh(a["Sigma0"]) > 0)
    with pytest.raises(ValueError):
        prep.estimateExpPrior(x, uy, 2, "flat", out=out)


def test_courbe_round_trip(tmp_path):
    d = synth_decay(481, "sincExp", 1)
    p = tmp_path / "Courbe.csv"
    prep.write_courbe(p, d["x"], d["y"])
    assert p.read_text().splitlines()[0] == '"x","y"'     # R write.csv header
    x, y = prep.read_courbe(p)
    np.testing.assert_array_equal(x, d["x"])
    np.testing.assert_array_equal(y, d["y"])


def test_load_ctrl_overrides(tmp_path):
    p = tmp_path / "ctrlParams.yaml"
    p.write_text(CTRL_YAML)
    c = load_ctrl(str(p))
    assert c["nb_warmup"] == 100 and c["Nn"] == 15 and c["gridType"] == "extremal"
    assert c["rho_scale"] == 0 and c["dataType"] == DEFAULT_CTRL["dataType"]
    assert load_ctrl(str(p), Nn=10)["Nn"] == 10
    assert load_ctrl(None) == DEFAULT_CTRL
