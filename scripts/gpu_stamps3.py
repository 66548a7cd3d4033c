"""Per-action NUTS latency profile (FITOCT_STAMPS) at the headline shape."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["FITOCT_STAMPS"] = "1"
from fitoct_amd import SamplerConfig, sample
import bench
prob = bench.make_problem()
W, S = (int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "500,1000").split(","))
out = sample(prob, SamplerConfig(chains=1024, warmup=W, samples=S, seed=42))
print(f"kernel {out.kernel_ms:.1f} ms, gradients {out.total_leapfrogs}, per chain-gradient "
      f"{out.kernel_ms * 1e3 / (out.total_leapfrogs / 1024):.2f} us", flush=True)
