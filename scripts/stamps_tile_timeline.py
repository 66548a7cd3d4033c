"""Profiling build only: the headline workload (config 3) at full length with per-tile
timeline stamps -- when each tile's first chain finishes and when the tile ends, as a
fraction of the launch -- with and without chain migration.  The gap between the mean
tile end and 1.0 is the share of the machine idle in the launch's tail."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["FITOCT_STAMPS"] = "1"
import bench  # noqa: E402
from fitoct_amd import Plan  # noqa: E402

prob = bench.make_problem("horseshoe", 2048)
for mig in (1, 0):
    if mig:
        os.environ.pop("FITOCT_NO_MIGRATE", None)
    else:
        os.environ["FITOCT_NO_MIGRATE"] = "1"
    cfg = bench.make_config(1000, 1024, 0, 0, 500, 1000)
    print(f"=== migration={mig}", file=sys.stderr, flush=True)
    with Plan(prob, cfg) as pl:
        pl.run()
        o = pl.download(with_draws=False)
    print(f"migration={mig}: kernel {o.kernel_ms:.1f} ms, migrations {o.migrations}, "
          f"gradients {o.total_leapfrogs}", file=sys.stderr, flush=True)
