"""ctypes binding of libfitoct.so (include/fitoct.h).

This is the Python counterpart of the R ``.Call`` shim described in
INTEGRATION.md: plain C structs, caller-owned numpy buffers, status codes
turned into exceptions.  Loading fails loudly if the in-tree library is absent:
there is no CPU fallback on the product path.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FITOCT_LIB_PATH") or os.path.join(HERE, "libfitoct.so")   # override: A/B experiments

PRIOR = {"normal": 0, "lasso": 1, "horseshoe": 2, "monoexp": 3}   # monoexp: FITOCT_MODEL_MONOEXP
GRID = {"internal": 0, "extremal": 1}
PREC = {"f64": 0, "mixed": 1}

STATUS = {
    0: "FITOCT_OK", -1: "FITOCT_E_ARG", -2: "FITOCT_E_HIP", -3: "FITOCT_E_NODEVICE",
    -4: "FITOCT_E_INIT", -5: "FITOCT_E_NUMERIC", -6: "FITOCT_E_TIMEOUT", -7: "FITOCT_E_INTERNAL",
    -8: "FITOCT_E_CANCELLED",
}

_dp = C.POINTER(C.c_double)
_ip = C.POINTER(C.c_int32)


class Problem(C.Structure):
    _fields_ = [
        ("N", C.c_int32), ("x", _dp), ("y", _dp), ("uy", _dp),
        ("data_type", C.c_int32), ("Nn", C.c_int32), ("grid_type", C.c_int32),
        ("rho", C.c_double), ("B", _dp),
        ("theta0", C.c_double * 3), ("Sigma0", C.c_double * 9),
        ("prior_type", C.c_int32), ("lambda_rate", C.c_double), ("lambda_scale", C.c_double),
        ("nu", C.c_double), ("prior_PD", C.c_int32), ("kernel_conv", C.c_int32),
        ("lambda_conv", C.c_int32), ("sigma_scale", C.c_double), ("nugget", C.c_double),
        ("theta_prior", C.c_int32),
    ]


class Config(C.Structure):
    _fields_ = [
        ("chains", C.c_int32), ("chain_offset", C.c_int32), ("warmup", C.c_int32),
        ("samples", C.c_int32), ("seed", C.c_uint64), ("adapt_delta", C.c_double),
        ("max_treedepth", C.c_int32), ("adapt_engaged", C.c_int32), ("stepsize", C.c_double),
        ("gamma", C.c_double), ("kappa", C.c_double), ("t0", C.c_double),
        ("init_buffer", C.c_int32), ("term_buffer", C.c_int32), ("window", C.c_int32),
        ("init_radius", C.c_double), ("save_warmup", C.c_int32), ("precision", C.c_int32),
        ("device", C.c_int32), ("n_devices", C.c_int32), ("devices", C.c_int32 * 16),
    ]


MAX_DEVICES = 16   # include/fitoct.h FITOCT_MAX_DEVICES


class Result(C.Structure):
    _fields_ = [
        ("draws", _dp), ("draws_capacity", C.c_int64), ("stepsize", _dp),
        ("inv_metric", _dp), ("last_q", _dp), ("chain_status", _ip),
        ("n_cols", C.c_int32), ("iters_saved", C.c_int32), ("dim", C.c_int32),
        ("migrations", C.c_int32), ("total_leapfrogs", C.c_int64), ("kernel_ms", C.c_double),
        ("wall_ms", C.c_double), ("two_ended_transitions", C.c_int64),
        ("paired_transitions", C.c_int64),
    ]


class PlanInfo(C.Structure):
    _fields_ = [
        ("dim", C.c_int32), ("n_cols", C.c_int32), ("iters_saved", C.c_int32),
        ("chains", C.c_int32), ("tiles", C.c_int32), ("chains_per_tile", C.c_int32),
        ("bins_per_thread", C.c_int32), ("threads_per_tile", C.c_int32),
        ("lds_bytes", C.c_int32), ("n_pad", C.c_int32), ("draws_bytes", C.c_int64),
        ("sampler", C.c_int32), ("n_devices", C.c_int32),
        ("two_ended", C.c_int32), ("ring_records", C.c_int32), ("ring_records_in_levels", C.c_int32),
        ("paired", C.c_int32), ("workgroups", C.c_int32), ("basis_mode", C.c_int32),
    ]


class OptimConfig(C.Structure):
    _fields_ = [
        ("iter", C.c_int32), ("history", C.c_int32), ("init_alpha", C.c_double),
        ("tol_obj", C.c_double), ("tol_rel_obj", C.c_double), ("tol_grad", C.c_double),
        ("tol_rel_grad", C.c_double), ("tol_param", C.c_double), ("hessian", C.c_int32),
        ("jacobian", C.c_int32), ("hessian_step", C.c_double), ("precision", C.c_int32),
        ("device", C.c_int32),
    ]


class OptimResult(C.Structure):
    _fields_ = [
        ("par", _dp), ("hessian", _dp), ("value", C.c_double), ("sumr2", C.c_double),
        ("iterations", C.c_int32), ("n_evals", C.c_int32), ("termination", C.c_int32),
        ("return_code", C.c_int32),
    ]


class VbConfig(C.Structure):
    _fields_ = [
        ("iter", C.c_int32), ("grad_samples", C.c_int32), ("elbo_samples", C.c_int32),
        ("eval_elbo", C.c_int32), ("eta", C.c_double), ("adapt_engaged", C.c_int32),
        ("adapt_iter", C.c_int32), ("tol_rel_obj", C.c_double), ("output_samples", C.c_int32),
        ("pad_", C.c_int32), ("seed", C.c_uint64), ("precision", C.c_int32), ("device", C.c_int32),
    ]


class VbResult(C.Structure):
    _fields_ = [
        ("mu", _dp), ("omega", _dp), ("draws", _dp), ("log_p", _dp), ("log_g", _dp),
        ("sumr2", _dp), ("eta", C.c_double), ("elbo", C.c_double), ("iterations", C.c_int32),
        ("converged", C.c_int32), ("n_evals", C.c_int32), ("pad_", C.c_int32),
    ]


TERMINATION = {0: "success", 10: "absolute parameter change", 20: "absolute objective change",
               21: "relative objective change", 30: "gradient norm", 31: "relative gradient",
               40: "maximum iterations", -1: "line search failed"}

# every symbol declared in include/fitoct.h: (name, restype, argtypes)
SIGNATURES = [
    ("fitoct_abi_version", C.c_int32, []),
    ("fitoct_last_error", C.c_char_p, []),
    ("fitoct_device_count", C.c_int32, []),
    ("fitoct_struct_sizes", C.c_int32, [_ip, _ip, _ip, _ip]),
    ("fitoct_default_config", None, [C.POINTER(Config)]),
    ("fitoct_default_problem", None, [C.POINTER(Problem)]),
    ("fitoct_dim", C.c_int32, [C.c_int32, C.c_int32]),
    ("fitoct_n_cols", C.c_int32, [C.c_int32, C.c_int32]),
    ("fitoct_column_name", C.c_int32, [C.c_int32, C.c_int32, C.c_int32, C.c_char_p, C.c_int32]),
    ("fitoct_build_basis", C.c_int32, [C.POINTER(Problem), _dp, _dp]),
    ("fitoct_mono_initial_theta", C.c_int32, [C.c_int32, _dp, _dp, C.c_int32, _dp]),
    ("fitoct_logp_grad", C.c_int32,
     [C.POINTER(Problem), C.c_int32, _dp, _dp, _dp, _dp, C.c_int32, C.c_int32]),
    ("fitoct_expgp_sample", C.c_int32, [C.POINTER(Problem), C.POINTER(Config), C.POINTER(Result)]),
    ("fitoct_plan_create", C.c_int32,
     [C.POINTER(Problem), C.POINTER(Config), C.POINTER(C.c_void_p)]),
    ("fitoct_plan_get_info", C.c_int32, [C.c_void_p, C.POINTER(PlanInfo)]),
    ("fitoct_plan_run", C.c_int32, [C.c_void_p, C.c_void_p, C.c_void_p]),
    ("fitoct_plan_launch", C.c_int32, [C.c_void_p, C.c_void_p, C.c_void_p]),
    ("fitoct_plan_poll", C.c_int32, [C.c_void_p, C.POINTER(C.c_int64), C.POINTER(C.c_int64),
                                     C.POINTER(C.c_int32)]),
    ("fitoct_plan_cancel", C.c_int32, [C.c_void_p]),
    ("fitoct_plan_wait", C.c_int32, [C.c_void_p]),
    ("fitoct_plan_set_init", C.c_int32, [C.c_void_p, _dp, _dp, _dp]),
    ("fitoct_plan_download", C.c_int32, [C.c_void_p, C.POINTER(Result)]),
    ("fitoct_plan_destroy", None, [C.c_void_p]),
    ("fitoct_batch_create", C.c_int32,
     [C.POINTER(Problem), C.c_int32, C.POINTER(Config), C.POINTER(C.c_void_p)]),
    ("fitoct_batch_get_info", C.c_int32, [C.c_void_p, C.POINTER(PlanInfo)]),
    ("fitoct_batch_run", C.c_int32, [C.c_void_p, C.c_void_p, C.c_void_p]),
    ("fitoct_batch_download", C.c_int32, [C.c_void_p, C.c_int32, C.POINTER(Result)]),
    ("fitoct_batch_destroy", None, [C.c_void_p]),
    ("fitoct_evaluator_create", C.c_int32,
     [C.POINTER(Problem), C.c_int32, C.c_int32, C.c_int32, C.POINTER(C.c_void_p)]),
    ("fitoct_evaluator_run", C.c_int32,
     [C.c_void_p, C.c_int32, _dp, C.c_int32, C.c_int32, _dp, _dp, _dp]),
    ("fitoct_evaluator_destroy", None, [C.c_void_p]),
    ("fitoct_constrain", C.c_int32, [C.c_int32, C.c_int32, C.c_int32, _dp, _dp]),
    ("fitoct_default_optim_config", None, [C.POINTER(OptimConfig)]),
    ("fitoct_optimize", C.c_int32,
     [C.POINTER(Problem), C.POINTER(OptimConfig), _dp, C.POINTER(OptimResult)]),
    ("fitoct_default_vb_config", None, [C.POINTER(VbConfig)]),
    ("fitoct_vb", C.c_int32, [C.POINTER(Problem), C.POINTER(VbConfig), _dp, C.POINTER(VbResult)]),
    ("fitoct_output_n_params", C.c_int32, [C.POINTER(Problem)]),
    ("fitoct_output_param_name", C.c_int32, [C.POINTER(Problem), C.c_int32, C.c_char_p, C.c_int32]),
    ("fitoct_output_rows", C.c_int32, [C.POINTER(Problem), C.c_int32, C.c_int64, _dp, _dp]),
    ("fitoct_write_stan_csv", C.c_int32,
     [C.c_char_p, C.POINTER(Problem), C.POINTER(Config), C.c_int32, _dp, C.c_double, _dp,
      C.c_double, C.c_double]),
    ("fitoct_write_vb_csv", C.c_int32,
     [C.c_char_p, C.POINTER(Problem), C.POINTER(VbConfig), _dp, C.c_double, C.c_int32, _dp, _dp,
      _dp, _dp, C.c_double]),
    ("fitoct_expgp_curves", C.c_int32,
     [C.POINTER(Problem), C.c_int32, _dp, _dp, _dp, _dp, _dp, _dp]),
    ("fitoct_progress_line", C.c_int32,
     [C.c_int64, C.c_int64, C.c_int32, C.c_int32, C.c_char_p, C.c_int32]),
    ("fitoct_split_rhat_ess", C.c_int32, [_dp, C.c_int32, C.c_int32, _dp, _dp]),
    ("fitoct_rank_rhat", C.c_int32, [_dp, C.c_int32, C.c_int32, _dp]),
]

_LIB = None


class FitOCTError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{STATUS.get(code, code)}: {msg}")
        self.code = code


def _single_hip_runtime():
    """Keep ONE HIP runtime per process.  PyTorch-ROCm bundles its own
    libamdhip64 (soname libamdhip64.so.7, the same as /opt/rocm's); if libfitoct
    loaded /opt/rocm's copy first, torch would later load a second HIP/HSA
    runtime and find no GPU.  Loading torch first makes the dynamic linker bind
    libfitoct to torch's already-loaded runtime.  Without torch (e.g. the R
    shim) libfitoct uses /opt/rocm's runtime."""
    if os.environ.get("FITOCT_SYSTEM_HIP_RUNTIME"):
        return
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


ABI_VERSION = 8   # include/fitoct.h FITOCT_ABI_VERSION


def lib():
    """Load the in-tree libfitoct.so (fails loudly if it was not built or is not the
    ABI this binding was written for)."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} not found: build it with `python -m fitoct_amd.build` "
                "(the HIP sampler has no CPU fallback)")
        _single_hip_runtime()
        L = C.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        # the binding's structs must be the library's
        if L.fitoct_abi_version() != ABI_VERSION:
            raise ImportError(f"{LIB_PATH}: ABI {L.fitoct_abi_version()}, this binding needs "
                              f"{ABI_VERSION} (rebuild with `python -m fitoct_amd.build`)")
        sz = [C.c_int32() for _ in range(4)]
        L.fitoct_struct_sizes(*[C.byref(v) for v in sz])
        want = (C.sizeof(Problem), C.sizeof(Config), C.sizeof(Result), C.sizeof(PlanInfo))
        if tuple(v.value for v in sz) != want:
            raise ImportError(f"{LIB_PATH}: struct sizes {tuple(v.value for v in sz)} != binding {want}")
        _LIB = L
    return _LIB


def check(code: int):
    if code != 0:
        raise FitOCTError(code, lib().fitoct_last_error().decode())


def dptr(a: np.ndarray):
    return a.ctypes.data_as(_dp) if a is not None else None


def struct_sizes():
    sz = [C.c_int32() for _ in range(4)]
    lib().fitoct_struct_sizes(*[C.byref(s) for s in sz])
    return tuple(s.value for s in sz)


def column_names(prior_type: int, Nn: int):
    L = lib()
    n = L.fitoct_n_cols(prior_type, Nn)
    buf = C.create_string_buffer(64)
    out = []
    for i in range(n):
        check(L.fitoct_column_name(prior_type, Nn, i, buf, 64))
        out.append(buf.value.decode())
    return out
