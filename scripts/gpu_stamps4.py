"""Stage timings vs load: 1 chain per tile vs 4, and with the likelihood off."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["FITOCT_STAMPS"] = "1"
from fitoct_amd import SamplerConfig, sample
import bench
for C, pd in [(256, 0), (1024, 0), (1024, 1)]:
    prob = bench.make_problem()
    prob.prior_PD = pd
    out = sample(prob, SamplerConfig(chains=C, warmup=150, samples=150, seed=42))
    print(f"C={C} prior_PD={pd}: kernel {out.kernel_ms:.1f} ms gradients/chain {out.total_leapfrogs / C:.0f}", flush=True)
