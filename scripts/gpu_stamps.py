import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["FITOCT_STAMPS"] = "1"
import numpy as np
from fitoct_amd import ExpGPProblem, SamplerConfig, sample
from fitoct_amd.synth import synth_decay, default_prior
t0, S0 = default_prior()
d = synth_decay(2048, "sincExp", 1)
for fam in ("horseshoe",):
    prob = ExpGPProblem(d["x"], d["y"], d["uy"], Nn=15, gridType="extremal", theta0=t0, Sigma0=S0, prior_type=fam)
    for prec in ("f64", "mixed"):
        for C in (1024,):
            cfg = SamplerConfig(chains=C, warmup=100, samples=100, seed=42, precision=prec, max_treedepth=8)
            out = sample(prob, cfg)
            post = out.draws[:, 100:, :]
            print(f"{fam} {prec} C={C}: kernel {out.kernel_ms:.1f} ms leapfrogs/chain {out.total_leapfrogs/C:.0f} us/leapfrog-step {out.kernel_ms*1e3/(out.total_leapfrogs/C):.2f} depth {post[:,:,3].mean():.2f}", flush=True)
