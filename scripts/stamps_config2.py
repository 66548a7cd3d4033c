"""Profiling build only (FITOCT_LIB_PATH=ablib/lib_prof.so): the config-2 shape (normal,
N = 512, 128 chains, one chain per tile) with stamps, two-ended (default) and one-ended
(FITOCT_NO_BIDI=1): gradient-wave busy per sweep and per-gradient sub-action costs."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["FITOCT_STAMPS"] = "1"
import bench  # noqa: E402
from fitoct_amd import Plan  # noqa: E402

prob = bench.make_problem("normal", 512)
for bidi in (1, 0):
    if bidi:
        os.environ.pop("FITOCT_NO_BIDI", None)
    else:
        os.environ["FITOCT_NO_BIDI"] = "1"
    print(f"=== two-ended={bidi}", file=sys.stderr, flush=True)
    cfg = bench.make_config(1000, 128, 0, 0, 500, 1000)
    with Plan(prob, cfg) as pl:
        pl.run()
        o = pl.download(with_draws=False)
    print(f"two-ended={bidi}: kernel {o.kernel_ms:.1f} ms, gradients {o.total_leapfrogs}",
          file=sys.stderr, flush=True)
