"""Shared test plumbing.

Markers: ``gpu`` -- needs an MI355X (run with ``-m gpu`` on the GPU box);
everything else runs on the CPU (``-m "not gpu"``).
"""
from __future__ import annotations

import glob
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    """Build libfitoct.so (hipcc cross-compiles without a GPU) and the C oracle
    before collection -- test modules load the library at import time, and a
    rebuild after that would leave two instances of it in the process (the R-shim
    driver binds the rebuilt file).  Incremental in the build container; on the GPU
    box (gpurun exports GRAFT_REPO_ROOT) only if missing: it uses the prebuilt files."""
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X)")
    config.addinivalue_line("markers", "slow: long-running test")
    from fitoct_amd import build as B
    if not os.path.exists(B.LIB) or not os.environ.get("GRAFT_REPO_ROOT"):
        B.build()
    from oracle import nuts_c
    nuts_c.build()


def golden_files(prefix):
    return sorted(glob.glob(os.path.join(GOLDEN, f"{prefix}_*.npz")))


def load_golden(path):
    sys.path.insert(0, GOLDEN)
    from make_golden import load
    return load(path)


def problems_from_fixture(fx):
    """(ExpGPProblem for the library, model_np.Problem for the numpy oracle)."""
    from fitoct_amd import ExpGPProblem
    from oracle import model_np as M
    m = fx["meta"]
    common = dict(Nn=m["Nn"], theta0=fx["theta0"], Sigma0=fx["Sigma0"],
                  prior_PD=m.get("prior_PD", 0), kernel_conv=m.get("kernel_conv", 0),
                  lambda_conv=m.get("lambda_conv", 0))
    lp = ExpGPProblem(fx["x"], fx["y"], fx["uy"], dataType=m.get("data_type", 2),
                      gridType=m["grid_type"], prior_type=m["family"], **common)
    npp = M.Problem(fx["x"], fx["y"], fx["uy"], data_type=m.get("data_type", 2),
                    grid_type=m["grid_type"], family=M.FAMILIES[m["family"]], **common)
    return lp, npp


def rel_err(a, b, floor=1e-300):
    a, b = np.asarray(a, float), np.asarray(b, float)
    return np.abs(a - b) / np.maximum(np.abs(b), floor)
