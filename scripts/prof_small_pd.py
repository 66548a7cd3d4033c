# short run for PMC collection; argv[1] = prior_PD (1: NUTS work only, no sweep)
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fitoct_amd import ExpGPProblem, SamplerConfig, sample
from fitoct_amd.synth import synth_decay, default_prior
t0, S0 = default_prior()
d = synth_decay(2048, "sincExp", 1)
prob = ExpGPProblem(d["x"], d["y"], d["uy"], Nn=15, gridType="extremal", theta0=t0, Sigma0=S0,
                    prior_type="horseshoe", prior_PD=int(sys.argv[1]))
out = sample(prob, SamplerConfig(chains=1024, warmup=60, samples=60, seed=42, max_treedepth=8))
print("kernel ms", out.kernel_ms, "leapfrogs", out.total_leapfrogs)
