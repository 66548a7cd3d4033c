"""Per-chain work of config 5 (FitOCT.R batch: 256 files x 4 chains, N=481, W=100 S=100, the
bench's first step seed): n_leapfrog of every chain at every iteration, saved to
gpurun_out/chain_work_c5.npz, with the launch time.  A tile of this batch hosts one file's
four chains and cannot hand them off, so it runs as long as its heaviest chain."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import bench  # noqa: E402
from fitoct_amd import Batch, ExpGPProblem, SamplerConfig  # noqa: E402
from fitoct_amd.synth import MODULATIONS, default_prior, synth_decay  # noqa: E402

conf = bench.CONFIGS[5]
t0, S0 = default_prior()
probs = []
for f in range(conf["files"]):
    d = synth_decay(conf["N"], MODULATIONS[f % 4], 1234 + f)
    probs.append(ExpGPProblem(d["x"], d["y"], d["uy"], dataType=2, Nn=bench.NN, gridType="extremal",
                              theta0=t0, Sigma0=S0, prior_type=conf["prior"]))
cfg = SamplerConfig(chains=conf["chains"], warmup=100, samples=100, seed=2000, adapt_delta=0.8,
                    max_treedepth=10, device=0)
b = Batch(probs, cfg)
b.run()
b.run()
nl = []
for f in range(len(probs)):
    o = b.download(f)
    nl.append(o.draws[:, :, o.columns.index("n_leapfrog__")].astype(np.int16))
nl = np.stack(nl)   # [file, chain, iter]
os.makedirs("gpurun_out", exist_ok=True)
np.savez_compressed("gpurun_out/chain_work_c5.npz", n_leapfrog=nl, kernel_ms=o.kernel_ms)
w = nl.astype(np.float64).sum(2)
print(f"config 5: kernel {o.kernel_ms:.1f} ms, info {b.info['chains_per_tile']} chains/tile "
      f"{b.info['tiles']} tiles; per chain mean {w.mean():.0f} max/mean {w.max() / w.mean():.3f}; "
      f"per tile (file) max-chain mean/overall max {w.max(1).mean() / w.max():.3f}; "
      f"per-file heaviest/second {np.median(np.sort(w, 1)[:, -1] / np.sort(w, 1)[:, -2]):.3f} (median)")
