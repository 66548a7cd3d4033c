"""Per-tile work balance of the headline run (config 3): gradients per chain
from the draws' n_leapfrog__ column, summed over each tile's chains."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from fitoct_amd import Plan  # noqa: E402

prob = bench.make_problem("horseshoe", 2048)
cfg = bench.make_config(1000, 1024, 0, 0, 500, 1000)
with Plan(prob, cfg) as pl:
    pl.run()
    o = pl.download()
lf = o.draws[:, :, 4].sum(1)
G = pl.info["chains_per_tile"]
tiles = lf.reshape(-1, G).sum(1)
res = {"kernel_ms": o.kernel_ms, "total_lf": int(o.total_leapfrogs), "chain_lf_mean": lf.mean(),
       "chain_lf_max": lf.max(), "chain_lf_p99": float(np.percentile(lf, 99)),
       "tile_mean": tiles.mean(), "tile_max": tiles.max(), "tile_max_over_mean": tiles.max() / tiles.mean(),
       "tile_p90_over_mean": float(np.percentile(tiles, 90) / tiles.mean()),
       "chain_max_over_mean": lf.max() / lf.mean()}
print(json.dumps({k: float(v) for k, v in res.items()}))
os.makedirs("gpurun_out", exist_ok=True)
np.save("gpurun_out/chain_lf.npy", lf)
