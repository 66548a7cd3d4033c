"""Per-chain diagnosis of the headline run (config 3): which chains inflate R-hat?"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from fitoct_amd import SamplerConfig, sample
from fitoct_amd.stanfit import split_rhat_ess
import bench
prob = bench.make_problem()
cols = prob.column_names()
ci = {c: i for i, c in enumerate(cols)}
seed = int(sys.argv[1]) if len(sys.argv) > 1 else 42
cfg = SamplerConfig(chains=1024, warmup=500, samples=1000, seed=seed)
t = time.time(); g = sample(prob, cfg); print("run", time.time() - t, "s kernel", g.kernel_ms, "lf", g.total_leapfrogs)
W = 500
d = g.draws
post = d[:, W:, :]
np.savez_compressed("gpurun_out/headline_chainstats.npz", means=post.mean(1), sds=post.std(1),
                    eps=g.stepsize, minv=g.inv_metric, div=post[:, :, 5].mean(1), td=post[:, :, 3].mean(1),
                    acc=post[:, :, 1].mean(1), lp=post[:, :, 0].mean(1), warm_lp=d[:, :W, 0].mean(1))
for name in ["theta.1", "theta.2", "theta.3", "sigma", "z.4", "r1_global", "lp__"]:
    x = post[:, :, ci[name]]
    r, e = split_rhat_ess(x)
    m = x.mean(1)
    med = np.median(m); mad = np.median(np.abs(m - med)) * 1.4826
    out = np.where(np.abs(m - med) > 5 * mad)[0]
    print(f"{name}: rhat {r:.4f} ess {e:.0f} chain-mean med {med:.5g} mad {mad:.3g} outliers {len(out)} {out[:12].tolist()}")
    if len(out):
        keep = np.setdiff1d(np.arange(1024), out)
        print(f"    rhat without outliers {split_rhat_ess(x[keep])[0]:.4f}")
th3 = post[:, :, ci["theta.3"]].mean(1)
o = np.argsort(np.abs(th3 - np.median(th3)))[-8:]
for c in o:
    print(f"chain {c}: th3 mean {th3[c]:.2f} sd {post[c,:,ci['theta.3']].std():.2f} eps {g.stepsize[c]:.4g} div {post[c,:,5].mean():.3f} td {post[c,:,3].mean():.2f} acc {post[c,:,1].mean():.3f} lp {post[c,:,0].mean():.2f} sigma {post[c,:,ci['sigma']].mean():.3f}")
print("median chain: eps", np.median(g.stepsize), "td", np.median(post[:, :, 3].mean(1)), "acc", np.median(post[:, :, 1].mean(1)), "lp", np.median(post[:, :, 0].mean(1)))
print("div overall", post[:, :, 5].mean(), "chains with div>5%", int((post[:, :, 5].mean(1) > 0.05).sum()))
