"""Profiling build only: config-2 shape (normal, N = 512, 128 chains, one chain per tile)
with and without speculative leaves (FITOCT_NO_SPEC), per-action stamps on stderr."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["FITOCT_STAMPS"] = "1"
from fitoct_amd import ExpGPProblem, SamplerConfig, sample  # noqa: E402
from fitoct_amd.synth import default_prior, synth_decay  # noqa: E402
t0, S0 = default_prior()
d = synth_decay(512, "sincExp", 1)
prob = ExpGPProblem(d["x"], d["y"], d["uy"], Nn=15, gridType="extremal", theta0=t0,
                    Sigma0=S0, prior_type="normal")
for spec in (1, 0, 1, 0):
    if spec:
        os.environ.pop("FITOCT_NO_SPEC", None)
    else:
        os.environ["FITOCT_NO_SPEC"] = "1"
    cfg = SamplerConfig(chains=128, warmup=100, samples=100, seed=42, max_treedepth=10)
    print(f"=== spec={spec}", file=sys.stderr, flush=True)
    out = sample(prob, cfg)
    print(f"spec={spec}: kernel {out.kernel_ms:.1f} ms, gradients/chain "
          f"{out.total_leapfrogs / 128:.0f}, us per chain-gradient "
          f"{out.kernel_ms * 1e3 / (out.total_leapfrogs / 128):.2f}", file=sys.stderr, flush=True)
