import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["FITOCT_STAMPS"] = "1"
from fitoct_amd import ExpGPProblem, SamplerConfig, sample
from fitoct_amd.synth import synth_decay, default_prior
t0, S0 = default_prior()
d = synth_decay(2048, "sincExp", 1)
for pd in (1, 0):
    for C in (1024, 256):
        prob = ExpGPProblem(d["x"], d["y"], d["uy"], Nn=15, gridType="extremal", theta0=t0, Sigma0=S0, prior_type="horseshoe", prior_PD=pd)
        out = sample(prob, SamplerConfig(chains=C, warmup=100, samples=100, seed=42, max_treedepth=8))
        print(f"prior_PD={pd} C={C}: kernel {out.kernel_ms:.1f} ms leapfrogs/chain {out.total_leapfrogs/C:.0f}", flush=True)
