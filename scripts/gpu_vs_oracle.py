"""GPU sampler vs C oracle: same inputs, same seed -> compare trajectories draw by draw."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from fitoct_amd import ExpGPProblem, SamplerConfig, sample
from fitoct_amd.synth import synth_decay, default_prior
from oracle import nuts_c as O
t0, S0 = default_prior()
for fam, N, Nn, W, S in [("normal", 256, 10, 150, 100), ("horseshoe", 300, 8, 150, 100), ("lasso", 200, 12, 100, 100), ("normal", 1000, 15, 150, 50)]:
    d = synth_decay(N, "sincExp", 11)
    prob = ExpGPProblem(d["x"], d["y"], d["uy"], Nn=Nn, gridType="extremal", theta0=t0, Sigma0=S0, prior_type=fam)
    cfg = SamplerConfig(chains=8, warmup=W, samples=S, seed=77, max_treedepth=8)
    g = sample(prob, cfg)
    o = O.sample(prob, cfg, nthreads=8)
    gd, od = g.draws, o["draws"]
    # first iteration at which each chain diverges (relative difference > 1e-6 in any column)
    rel = np.abs(gd - od) / (1e-300 + np.abs(od) + 1e-12)
    rel = np.nan_to_num(rel, nan=0.0)
    bad = (rel > 1e-6).any(axis=2)
    first = [int(np.argmax(b)) if b.any() else W + S for b in bad]
    print(f"{fam} N={N} Nn={Nn}: first mismatching iteration per chain {first}")
    print("   max rel diff over first 20 iters:", float(rel[:, :20].max()), " lf gpu/cpu:", g.total_leapfrogs, int(o["leapfrogs"].sum()))
    print("   eps gpu", np.round(g.stepsize, 5), "cpu", np.round(o["stepsize"], 5))
    pm_g, pm_o = gd[:, W:, 7:10].reshape(-1, 3).mean(0), od[:, W:, 7:10].reshape(-1, 3).mean(0)
    print("   theta post means gpu", pm_g, "cpu", pm_o)
