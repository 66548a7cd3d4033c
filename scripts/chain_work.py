"""Per-chain work of the headline workload (config 3, full length): n_leapfrog of every
chain at every iteration (warmup included), saved as int16 to gpurun_out/chain_work.npz.
The tail study (scripts/tail_sim.py) replays it against scheduling policies."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import bench  # noqa: E402
from fitoct_amd import Plan  # noqa: E402

prob = bench.make_problem("horseshoe", 2048)
cfg = bench.make_config(1000, 1024, 0, 0, 500, 1000)
cfg.save_warmup = True
with Plan(prob, cfg) as pl:
    pl.run()
    o = pl.download()
col = o.columns.index("n_leapfrog__")
nl = o.draws[:, :, col].astype(np.int16)
os.makedirs("gpurun_out", exist_ok=True)
np.savez_compressed("gpurun_out/chain_work.npz", n_leapfrog=nl, kernel_ms=o.kernel_ms)
w = nl.sum(1).astype(np.float64)
print(f"kernel {o.kernel_ms:.1f} ms total {w.sum():.0f} (reported {o.total_leapfrogs}); per chain "
      f"mean {w.mean():.0f} max/mean {w.max() / w.mean():.3f} p90/mean "
      f"{np.percentile(w, 90) / w.mean():.3f} min/mean {w.min() / w.mean():.3f}")
