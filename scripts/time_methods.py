"""Wall time of the non-sampling methods and of fitMonoExp (config 1) on the GPU.

    python scripts/time_methods.py > gpurun_out/methods.json
"""
import json
import sys
import time

import numpy as np

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from fitoct_amd import fitExpGP, fitMonoExp  # noqa: E402
from fitoct_amd.synth import default_prior, synth_decay  # noqa: E402


def timed(f, reps=3):
    f()                                   # warm: plan/JIT-free, but first-call HIP init
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        r = f()
        t.append(time.perf_counter() - t0)
    return min(t), r


out = {}
d = synth_decay(256, "monoExp", 1)
t, r = timed(lambda: fitMonoExp(d["x"], d["y"], d["uy"], method="optim"))
out["fitMonoExp_optim_N256_s"] = t
out["fitMonoExp_optim_evals"] = r["fit"].iterations
t, r = timed(lambda: fitMonoExp(d["x"], d["y"], d["uy"], method="sample", seed=1), reps=1)
out["fitMonoExp_sample_N256_4ch_s"] = t
t0, S0 = default_prior()
for fam, N in [("normal", 512), ("horseshoe", 2048)]:
    e = synth_decay(N, "sincExp", 2)
    kw = dict(Nn=15, gridType="extremal", theta0=t0, Sigma0=S0, prior_type=fam)
    t, r = timed(lambda: fitExpGP(e["x"], e["y"], e["uy"], method="optim", **kw))
    out[f"optim_{fam}_N{N}_s"] = t
    out[f"optim_{fam}_N{N}_iters"] = r["fit"].iterations
    out[f"optim_{fam}_N{N}_termination"] = r["fit"].termination
    for seed in (3, 4, 5):   # ADVI from Stan's unit-scale start fails for some seeds
        try:
            t, r = timed(lambda: fitExpGP(e["x"], e["y"], e["uy"], method="vb", seed=seed, **kw),
                         reps=1)
        except Exception as ex:  # noqa: BLE001 -- recorded, not hidden
            out[f"vb_{fam}_N{N}_seed{seed}_error"] = str(ex)
            continue
        out[f"vb_{fam}_N{N}_s"] = t
        out[f"vb_{fam}_N{N}_seed"] = seed
        out[f"vb_{fam}_N{N}_iters"] = r["fit"].meta["iterations"]
        out[f"vb_{fam}_N{N}_evals"] = r["fit"].meta["n_evals"]
        break
print(json.dumps(out, indent=1))
