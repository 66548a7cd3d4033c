"""fitoct_amd -- MI355X-native NUTS sampler for FitOCT's ExpGP posterior.

Product path: Python (this package) -> ctypes -> libfitoct.so (C ABI,
include/fitoct.h) -> HIP kernels for gfx950.  See DESIGN.md.
"""
from .api import (Batch, ExpGPProblem, Plan, SampleOutput, SamplerConfig, fitExpGP, logp_grad,
                  sample, sample_batch)
from ._lib import FitOCTError, lib
from .monoexp import fitMonoExp, printBr
from .optim_vb import Evaluator, OptimFit, optimizing, vb

__all__ = ["ExpGPProblem", "SamplerConfig", "Plan", "Batch", "SampleOutput", "fitExpGP",
           "logp_grad", "sample", "sample_batch", "FitOCTError", "lib", "fitMonoExp", "printBr",
           "Evaluator", "OptimFit", "optimizing", "vb"]
