"""Profiling build only: NUTS action / sub-action cycles at latency-bound (G=1) and
batch-like (G=4, small N) shapes."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["FITOCT_STAMPS"] = "1"
from fitoct_amd import ExpGPProblem, SamplerConfig, sample  # noqa: E402
from fitoct_amd.synth import default_prior, synth_decay  # noqa: E402
t0, S0 = default_prior()
for fam, N, C in (("normal", 512, 128), ("normal", 481, 1024), ("horseshoe", 2048, 1024)):
    d = synth_decay(N, "sincExp", 1)
    prob = ExpGPProblem(d["x"], d["y"], d["uy"], Nn=15, gridType="extremal", theta0=t0,
                        Sigma0=S0, prior_type=fam)
    cfg = SamplerConfig(chains=C, warmup=100, samples=100, seed=42, max_treedepth=8)
    print(f"=== {fam} N={N} C={C}", file=sys.stderr, flush=True)
    out = sample(prob, cfg)
    print(f"{fam} N={N} C={C}: kernel {out.kernel_ms:.1f} ms, gradients/chain "
          f"{out.total_leapfrogs / C:.0f}, us per chain-gradient "
          f"{out.kernel_ms * 1e3 / (out.total_leapfrogs / C):.2f}", flush=True)
