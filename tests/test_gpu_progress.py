"""Run-time progress and cancellation of a planned run (fitoct_plan_launch / poll /
cancel / wait).  They replace rstan's stan.log progress read by the Shiny server
(server.R:457-484) and the R_CheckUserInterrupt contract of SURVEY.md §8b.

* Progress is monotone, ends at chains * (warmup + samples), and leaves the draws
  bit-identical to a plain run.
* A cancelled run drains within a few transitions per chain and reports
  FITOCT_E_CANCELLED.  The cancelled runs here are sized so that, even if
  cancellation failed, the kernel would still end within ~30 s.
"""
from __future__ import annotations

import time

import numpy as np
import pytest

from fitoct_amd import ExpGPProblem, Plan, SamplerConfig, fitExpGP
from fitoct_amd._lib import FitOCTError
from fitoct_amd.synth import default_prior, synth_decay

pytestmark = pytest.mark.gpu


def _prob(N=512, Nn=10):
    t0, S0 = default_prior()
    d = synth_decay(N, "sincExp", 3)
    return ExpGPProblem(d["x"], d["y"], d["uy"], Nn=Nn, gridType="extremal", theta0=t0,
                        Sigma0=S0, prior_type="normal")


def test_progress_monotone_and_draws_unchanged():
    prob = _prob()
    cfg = SamplerConfig(chains=64, warmup=150, samples=150, seed=5, max_treedepth=8)
    with Plan(prob, cfg) as pl:
        pl.launch()
        seen = []
        t_end = time.time() + 60
        while time.time() < t_end:
            done, total, fin = pl.poll()
            seen.append(done)
            if fin:
                break
            time.sleep(0.005)
        pl.wait()
        done, total, fin = pl.poll()
        out = pl.download()
    assert fin and total == 64 * 300 and done == total
    assert all(b >= a for a, b in zip(seen, seen[1:])), "progress went backwards"
    assert any(0 < s < total for s in seen) or len(seen) <= 2
    with Plan(prob, cfg) as pl:
        pl.run()
        ref = pl.download()
    assert np.array_equal(out.draws, ref.draws, equal_nan=True)


def test_cancel_drains_and_reports():
    prob = _prob()
    cfg = SamplerConfig(chains=32, warmup=100, samples=20000, seed=6, max_treedepth=8)
    with Plan(prob, cfg) as pl:
        pl.launch()
        t_end = time.time() + 30
        while pl.poll()[0] < 32 * 16 and not pl.poll()[2] and time.time() < t_end:
            time.sleep(0.005)
        t0 = time.time()
        pl.cancel()
        pl.wait()
        dt = time.time() - t0
        done, total, fin = pl.poll()
        with pytest.raises(FitOCTError) as ei:
            pl.download()
    assert ei.value.code == -8
    assert fin and done < total
    assert dt < 5.0, f"cancelled run took {dt:.1f} s to drain"
    # a run driven through a progress callback completes normally
    cfg2 = SamplerConfig(chains=4, warmup=20, samples=20, seed=7, max_treedepth=6)
    with Plan(prob, cfg2) as pl:
        pl.run(progress=lambda d, t: None)
        assert pl.poll()[0] == 4 * 40
        pl.download()


def test_interrupt_in_progress_callback_cancels():
    prob = _prob()
    cfg = SamplerConfig(chains=16, warmup=100, samples=20000, seed=8, max_treedepth=8)

    def cb(done, total):
        if done > 16 * 16:
            raise KeyboardInterrupt

    with Plan(prob, cfg) as pl:
        t0 = time.time()
        with pytest.raises(KeyboardInterrupt):
            pl.run(progress=cb, poll_s=0.01)
        assert time.time() - t0 < 30
        with pytest.raises(FitOCTError) as ei:
            pl.download()
        assert ei.value.code == -8


def test_fitexpgp_prints_rstan_progress(capsys):
    """open_progress = FALSE as FitOCT.R:123 and server.R:425 pass it: the rstan-format
    lines still reach stdout, and the Shiny parser (server.R:457-472, ported in
    tests/shiny_progress.py) reads a monotone 0..100 from them."""
    from shiny_progress import replay
    d = synth_decay(256, "sincExp", 4)
    t0, S0 = default_prior()
    res = fitExpGP(d["x"], d["y"], d["uy"], dataType=2, Nn=8, gridType="extremal",
                   theta0=t0, Sigma0=S0, nb_warmup=100, nb_iter=200, open_progress=False,
                   nb_chains=4, seed=3, max_treedepth=6)
    out = capsys.readouterr().out
    lines = [l for l in out.splitlines() if l.startswith("Chain ")]
    assert lines and "[100%]" in lines[-1] and "(Sampling)" in lines[-1]
    shown = replay(lines)
    assert shown[-1] == 100
    assert all(b >= a for a, b in zip(shown, shown[1:]))
    assert res["fit"] is not None
