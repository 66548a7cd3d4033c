# short config-2-shaped run (normal, N = 512, 128 chains: one chain per tile) for PMC
# collection; argv[1] = prior_PD (1: NUTS work only, no sweep)
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fitoct_amd import ExpGPProblem, SamplerConfig, sample  # noqa: E402
from fitoct_amd.synth import default_prior, synth_decay  # noqa: E402
t0, S0 = default_prior()
d = synth_decay(512, "sincExp", 1234)
prob = ExpGPProblem(d["x"], d["y"], d["uy"], dataType=2, Nn=15, gridType="extremal", theta0=t0,
                    Sigma0=S0, prior_type="normal", prior_PD=int(sys.argv[1]))
out = sample(prob, SamplerConfig(chains=128, warmup=100, samples=100, seed=1000, max_treedepth=10))
print("kernel ms", out.kernel_ms, "leapfrogs", out.total_leapfrogs)
