"""First GPU probe: logp/grad parity vs the numpy oracle, then a short sampler run."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from fitoct_amd import ExpGPProblem, SamplerConfig, logp_grad, sample
from fitoct_amd.synth import synth_decay, default_prior
from oracle import model_np as M

t0, S0 = default_prior()
for N, fam, Nn in [(512, "normal", 15), (2048, "horseshoe", 15), (4096, "lasso", 15), (481, "normal", 10), (700, "horseshoe", 20)]:
    d = synth_decay(N, "sincExp", 7)
    for pd in (0, 1):
        prob = ExpGPProblem(d["x"], d["y"], d["uy"], Nn=Nn, gridType="extremal", theta0=t0, Sigma0=S0, prior_type=fam, prior_PD=pd)
        mp = M.Problem(d["x"], d["y"], d["uy"], Nn=Nn, grid_type="extremal", theta0=t0, Sigma0=S0, family=M.FAMILIES[fam], prior_PD=pd)
        rng = np.random.default_rng(N + pd)
        P = 9
        q = rng.normal(0, 0.3, (P, prob.D)); q[:, 0:3] = np.log(t0) + rng.normal(0, 0.02, (P, 3)); q[:, -1] = rng.normal(0, .3, P)
        for prec in ("f64", "mixed"):
            lp, g, s2 = logp_grad(prob, q, prec)
            worst_lp = worst_g = 0
            for i in range(P):
                rl, rg, rs = M.logp_grad(q[i], mp)
                worst_lp = max(worst_lp, abs(lp[i] - rl) / (1 + abs(rl)))
                worst_g = max(worst_g, np.max(np.abs(g[i] - rg) / (1 + np.abs(rg))))
            print(f"N={N} {fam} Nn={Nn} PD={pd} {prec}: lp rel {worst_lp:.2e} grad rel {worst_g:.2e}", flush=True)

d = synth_decay(2048, "sincExp", 1)
prob = ExpGPProblem(d["x"], d["y"], d["uy"], Nn=15, gridType="extremal", theta0=t0, Sigma0=S0, prior_type="horseshoe")
for C, W, S in [(4, 100, 100), (1024, 150, 150)]:
    cfg = SamplerConfig(chains=C, warmup=W, samples=S, seed=42)
    t = time.perf_counter()
    out = sample(prob, cfg)
    dt = time.perf_counter() - t
    dr = out.draws
    post = dr[:, W:, :]
    print(f"C={C} W={W} S={S}: kernel {out.kernel_ms:.1f} ms wall {dt*1e3:.1f} ms leapfrogs {out.total_leapfrogs} draws/s {C*S/(out.kernel_ms/1e3):.3e}")
    print("  mean treedepth", post[:, :, 3].mean(), "n_leapfrog", post[:, :, 4].mean(), "div", post[:, :, 5].mean(), "accept", post[:, :, 1].mean(), "eps", out.stepsize[:4])
    print("  theta means", post[:, :, 7:10].reshape(-1, 3).mean(0), "sigma", post[:, :, 7 + prob.D - 1].mean(), "br", post[:, :, -1].mean())
