"""Profiling build only (FITOCT_VARIANT=prof FITOCT_PROFILE=1): gradient-wave busy time
per sweep with the sampler's work between sweeps removed (FITOCT_BENCH_SWEEPS), against
the full sampler, at config 3's shape (horseshoe, N = 2048, Nn = 15, 1024 chains) and
config 4's (lasso, N = 4096)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["FITOCT_STAMPS"] = "1"
from fitoct_amd import ExpGPProblem, SamplerConfig, sample  # noqa: E402
from fitoct_amd.synth import default_prior, synth_decay  # noqa: E402
t0, S0 = default_prior()
for fam, N in (("horseshoe", 2048), ("lasso", 4096)):
    d = synth_decay(N, "sincExp", 1234)
    prob = ExpGPProblem(d["x"], d["y"], d["uy"], Nn=15, gridType="extremal", theta0=t0,
                        Sigma0=S0, prior_type=fam, lambda_scale=10.0)
    for mode in ("sweeps only", "sampler"):
        if mode == "sweeps only":
            os.environ["FITOCT_BENCH_SWEEPS"] = "2000"
        else:
            os.environ.pop("FITOCT_BENCH_SWEEPS", None)
        print(f"=== {fam} N={N} 1024 chains: {mode}", file=sys.stderr, flush=True)
        try:
            out = sample(prob, SamplerConfig(chains=1024, warmup=60, samples=60, seed=42))
            print(f"{fam} N={N} {mode}: kernel {out.kernel_ms:.1f} ms", flush=True)
        except Exception as e:   # the sweep-only run stops chains early: draws are not valid
            print(f"{fam} N={N} {mode}: {e}", flush=True)
