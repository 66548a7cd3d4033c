"""Profiling build only (FITOCT_LIB_PATH=ablib/lib_prof.so): tile occupancy of the headline
workload (config 3, full length) -- the share of all tiles' time and of all sweeps spent
while a tile hosted k = 0..4 live chains.  The launch's tail is its thinned-out tiles:
how much of the machine-time they take bounds what a faster lone-chain path can recover."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["FITOCT_STAMPS"] = "1"
import bench  # noqa: E402
from fitoct_amd import Plan  # noqa: E402

W, S = (int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "500,1000").split(","))
prob = bench.make_problem("horseshoe", 2048)
cfg = bench.make_config(1000, 1024, 0, 0, W, S)
with Plan(prob, cfg) as pl:
    pl.run()
    o = pl.download(with_draws=False)
print(f"config 3 W={W} S={S}: kernel {o.kernel_ms:.1f} ms, migrations {o.migrations}, "
      f"gradients {o.total_leapfrogs}", file=sys.stderr, flush=True)
