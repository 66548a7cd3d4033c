"""Generate the committed golden fixtures under tests/golden/.

The reference holds no test with expected values (no golden
vectors / KATs in-tree; R, rstan and FitOCTLib are absent here), so the
fixtures are produced in this container by the oracles:

* ``logp_<case>.npz``   -- inputs (x, y, uy, theta0, Sigma0, switches), the GP
  basis B and, at seeded unconstrained points q, ``lp``, ``grad``, ``sumr2``
  from the numpy restatement (oracle/model_np.py).  Inputs come from the
  restated synthData.R generator (fitoct_amd/synth.py) so the decays have the
  reference's shape (x = 20..500 um, a=1000, b=2000, l0=150).
* ``draws_<case>.npz``  -- a short NUTS run of the C oracle (oracle/fitoct_oracle.c)
  at a fixed seed: the HIP sampler uses the same Philox addressing, so its
  leading draws must reproduce these.
* ``philox_kat.json``   -- Random123 Philox4x32-10 known-answer vectors
  (published with Random123's kat_vectors; not from the FitOCT reference).

Run:  python tests/golden/make_golden.py     (deterministic; rewrites the files)
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from fitoct_amd.synth import default_prior, synth_decay  # noqa: E402
from oracle import model_np as M  # noqa: E402

# name: (family, N, Nn, grid, prior_PD, kernel_conv, lambda_conv, data_type, modulation)
LOGP_CASES = {
    "normal_n64": ("normal", 64, 6, "extremal", 0, 0, 0, 2, "sincExp"),
    "normal_prior_n64": ("normal", 64, 6, "extremal", 1, 0, 0, 2, "sincExp"),
    "normal_conv1_n50": ("normal", 50, 5, "internal", 0, 1, 1, 1, "sincExp1"),
    "lasso_n97": ("lasso", 97, 8, "internal", 0, 0, 0, 2, "sincExp2"),
    "horseshoe_n128": ("horseshoe", 128, 10, "extremal", 0, 0, 0, 2, "sincExp3"),
    "horseshoe_n481": ("horseshoe", 481, 15, "extremal", 0, 0, 0, 2, "sincExp"),
    # FitOCTLib::fitMonoExp model (config 1 shape: one synthData.R decay, N=256)
    "monoexp_n256": ("monoexp", 256, 2, "extremal", 0, 0, 0, 2, "monoExp"),
}

DRAW_CASES = {
    # name: (family, N, Nn, chains, warmup, samples, seed, max_treedepth)
    "normal_n64": ("normal", 64, 6, 4, 60, 40, 2024, 6),
    "horseshoe_n64": ("horseshoe", 64, 4, 4, 60, 40, 99, 6),
    "monoexp_n256": ("monoexp", 256, 2, 4, 60, 40, 5, 6),
}

PHILOX_KAT = [
    {"ctr": [0, 0, 0, 0], "key": [0, 0], "out": [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]},
    {"ctr": [0xffffffff] * 4, "key": [0xffffffff] * 2,
     "out": [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]},
    {"ctr": [0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344], "key": [0xa4093822, 0x299f31d0],
     "out": [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]},
]


def sample_q(fam: int, Nn: int, theta0, rng, n=4):
    D = M.dim(fam, Nn)
    Q = np.zeros((n, D))
    for j in range(n):
        q = np.zeros(D)
        q[0:3] = np.log(theta0) + 0.03 * rng.standard_normal(3)
        if fam == M.MONOEXP:
            Q[j] = q
            continue
        if fam == M.HORSESHOE:
            q[3:3 + Nn] = rng.standard_normal(Nn)
            q[3 + Nn:5 + 3 * Nn] = -1.0 + 0.5 * rng.standard_normal(2 + 2 * Nn)
        else:
            q[3:3 + Nn] = 0.05 * rng.standard_normal(Nn)
            if fam == M.NORMAL:
                q[3 + Nn] = np.log(0.1) + 0.3 * rng.standard_normal()
        q[D - 1] = 0.2 * rng.standard_normal()
        Q[j] = q
    return Q


def np_problem(d, fam, Nn, grid, pd, kc, lc, dt, theta0, Sigma0):
    return M.Problem(d["x"], d["y"], d["uy"], data_type=dt, Nn=Nn, grid_type=grid,
                     theta0=theta0, Sigma0=Sigma0, family=M.FAMILIES[fam], prior_PD=pd,
                     kernel_conv=kc, lambda_conv=lc)


def make_logp():
    theta0, Sigma0 = default_prior()
    for i, (name, (fam, N, Nn, grid, pd, kc, lc, dt, mod)) in enumerate(LOGP_CASES.items()):
        d = synth_decay(N, mod, seed=100 + i)
        t0 = theta0.copy()
        if dt == 1:
            t0[2] = 150.0
        S0 = np.diag((0.05 * t0) ** 2)
        P = np_problem(d, fam, Nn, grid, pd, kc, lc, dt, t0, S0)
        rng = np.random.Generator(np.random.PCG64(7 + i))
        Q = sample_q(P.family, Nn, t0, rng)
        out = [M.logp_grad(q, P) for q in Q]
        meta = dict(family=fam, N=N, Nn=Nn, grid_type=grid, prior_PD=pd, kernel_conv=kc,
                    lambda_conv=lc, data_type=dt, modulation=mod, lambda_rate=P.lambda_rate,
                    lambda_scale=P.lambda_scale, nu=P.nu, sigma_scale=P.sigma_scale,
                    nugget=P.nugget, rho=P.rho)
        np.savez_compressed(
            os.path.join(HERE, f"logp_{name}.npz"), meta=np.array(json.dumps(meta)),
            x=d["x"], y=d["y"], uy=d["uy"], theta0=t0, Sigma0=S0, B=P.B, xGP=P.xGP, q=Q,
            lp=np.array([o[0] for o in out]), grad=np.array([o[1] for o in out]),
            sumr2=np.array([o[2] for o in out]))


def make_draws():
    from fitoct_amd.api import ExpGPProblem, SamplerConfig
    from oracle import nuts_c
    theta0, Sigma0 = default_prior()
    for i, (name, (fam, N, Nn, C, W, S, seed, mtd)) in enumerate(DRAW_CASES.items()):
        d = synth_decay(N, "sincExp", seed=300 + i)
        prob = ExpGPProblem(d["x"], d["y"], d["uy"], Nn=Nn, gridType="extremal", theta0=theta0,
                            Sigma0=Sigma0, prior_type=fam)
        cfg = SamplerConfig(chains=C, warmup=W, samples=S, seed=seed, max_treedepth=mtd)
        o = nuts_c.sample(prob, cfg, nthreads=4)
        meta = dict(family=fam, N=N, Nn=Nn, chains=C, warmup=W, samples=S, seed=seed,
                    max_treedepth=mtd, grid_type="extremal")
        np.savez_compressed(os.path.join(HERE, f"draws_{name}.npz"),
                            meta=np.array(json.dumps(meta)), x=d["x"], y=d["y"], uy=d["uy"],
                            theta0=theta0, Sigma0=Sigma0, draws=o["draws"],
                            stepsize=o["stepsize"], inv_metric=o["inv_metric"],
                            leapfrogs=o["leapfrogs"])


def load(path):
    """Load one fixture (no pickles): dict of arrays + parsed ``meta``."""
    with np.load(path, allow_pickle=False) as z:
        out = {k: z[k] for k in z.files}
    out["meta"] = json.loads(str(out["meta"]))
    return out


if __name__ == "__main__":
    make_logp()
    make_draws()
    with open(os.path.join(HERE, "philox_kat.json"), "w") as f:
        json.dump(PHILOX_KAT, f, indent=1)
    print("golden fixtures written to", HERE)
