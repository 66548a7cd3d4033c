"""Bitwise A/B of variant libraries: every ablib/lib_*.so samples the same short
runs (configs 2, 3, 4 shapes and a batch of config-5 files), and each variant's draws
are compared bit for bit (SHA-256 of the draw arrays) with ablib/lib_base.so.  Latency-only changes (same
arithmetic) must print 'identical'.  ablib/env_<name> (KEY=VALUE lines), when present, is added to
lib_<name>'s environment (e.g. a copy of a library run with a switch set).

    python scripts/ab_bitwise.py            # on the GPU box
"""
import glob
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out", "abbit")

RUNNER = r"""
import sys, numpy as np
sys.path.insert(0, %r)
from fitoct_amd import ExpGPProblem, SamplerConfig, sample, sample_batch
from fitoct_amd.synth import MODULATIONS, default_prior, synth_decay
t0, S0 = default_prior()
res = {}
for name, fam, N, C, mtd in (("c2", "normal", 512, 128, 10), ("c3", "horseshoe", 2048, 256, 10),
                             ("c4", "lasso", 4096, 64, 10)):
    d = synth_decay(N, "sincExp", 1234)
    prob = ExpGPProblem(d["x"], d["y"], d["uy"], Nn=15, gridType="extremal", theta0=t0,
                        Sigma0=S0, prior_type=fam, lambda_scale=10.0)
    out = sample(prob, SamplerConfig(chains=C, warmup=100, samples=60, seed=7, max_treedepth=mtd))
    res[name] = out.draws
probs = []
for f in range(16):
    d = synth_decay(481, MODULATIONS[f %% 4], 1234 + f)
    probs.append(ExpGPProblem(d["x"], d["y"], d["uy"], Nn=15, gridType="extremal", theta0=t0,
                              Sigma0=S0, prior_type="normal"))
outs = sample_batch(probs, SamplerConfig(chains=4, warmup=60, samples=40, seed=9))
res["c5"] = np.stack([o.draws for o in outs])
import hashlib, json
json.dump({k: hashlib.sha256(np.ascontiguousarray(v).tobytes()).hexdigest() for k, v in res.items()},
          open(sys.argv[1], "w"))
"""


def main():
    os.makedirs(OUT, exist_ok=True)
    libs = sorted(glob.glob(os.path.join(ROOT, "ablib", "lib_*.so")))
    for lib in libs:
        name = os.path.basename(lib)[4:-3]
        env = dict(os.environ, FITOCT_LIB_PATH=lib)
        envf = os.path.join(ROOT, "ablib", "env_" + name)
        if os.path.exists(envf):
            env.update(line.strip().split("=", 1) for line in open(envf) if "=" in line)
        r = subprocess.run([sys.executable, "-c", RUNNER % ROOT, os.path.join(OUT, name + ".json")],
                           env=env, timeout=300)
        if r.returncode != 0:
            print(f"{name}: run failed ({r.returncode})", flush=True)
            return 1
    import json
    base = json.load(open(os.path.join(OUT, "base.json")))
    for lib in libs:
        name = os.path.basename(lib)[4:-3]
        if name == "base":
            continue
        got = json.load(open(os.path.join(OUT, name + ".json")))
        for k in base:
            print(f"{name} {k}: {'identical' if base[k] == got[k] else 'DIFFERENT'}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
