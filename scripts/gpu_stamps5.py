"""Profiling build only (FITOCT_PROFILE=1): per-action NUTS cycle costs and
sweep latency breakdown at the headline shape (G=4) and a latency-bound shape (G=1)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["FITOCT_STAMPS"] = "1"
from fitoct_amd import ExpGPProblem, SamplerConfig, sample  # noqa: E402
from fitoct_amd.synth import default_prior, synth_decay  # noqa: E402
t0, S0 = default_prior()
d = synth_decay(2048, "sincExp", 1)
prob = ExpGPProblem(d["x"], d["y"], d["uy"], Nn=15, gridType="extremal", theta0=t0, Sigma0=S0,
                    prior_type="horseshoe")
for C in (1024, 256):
    cfg = SamplerConfig(chains=C, warmup=100, samples=100, seed=42, max_treedepth=8)
    out = sample(prob, cfg)
    print(f"C={C}: kernel {out.kernel_ms:.1f} ms, gradients/chain {out.total_leapfrogs / C:.0f}, "
          f"us per chain-gradient {out.kernel_ms * 1e3 / (out.total_leapfrogs / C):.2f}", flush=True)
