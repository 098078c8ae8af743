"""ctypes binding of ``libstark_hip.so`` (C ABI in ``include/stark_hip.h``).

The library is built in-tree (``stark_amd/_lib/libstark_hip.so``, see
``__graft_entry__.build``).  If it is missing this module raises at import time: the
product path has no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("STARK_HIP_LIB", os.path.join(_HERE, "_lib", "libstark_hip.so"))

STK_OK = 0
ERRORS = {-1: "STK_E_ARG", -2: "STK_E_HIP", -3: "STK_E_NOMEM", -4: "STK_E_STATE",
          -5: "STK_E_NUMERIC", -6: "STK_E_NAN", -7: "STK_E_LINALG"}
STK_SCHOOLS, STK_LINREG, STK_LOGREG = 1, 2, 3
N_STATS = 6
STAT_NAMES = ("accept_stat__", "stepsize__", "treedepth__", "n_leapfrog__", "divergent__", "energy__")


class StarkHipError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"{ERRORS.get(code, code)}: {msg}")
        self.code = code


class LinAlgError(StarkHipError):
    """Raised where the reference raises numpy.linalg.LinAlgError (singular covariance)."""


class Shard(ctypes.Structure):
    _fields_ = [("n_rows", ctypes.c_int64), ("n_cols", ctypes.c_int32),
                ("x", ctypes.c_void_p), ("y", ctypes.c_void_p), ("y_int", ctypes.c_void_p),
                ("sigma", ctypes.c_void_p)]


class Config(ctypes.Structure):
    _fields_ = [("num_warmup", ctypes.c_int32), ("num_samples", ctypes.c_int32),
                ("chains", ctypes.c_int32), ("max_depth", ctypes.c_int32),
                ("adapt_delta", ctypes.c_double), ("adapt_gamma", ctypes.c_double),
                ("adapt_kappa", ctypes.c_double), ("adapt_t0", ctypes.c_double),
                ("stepsize", ctypes.c_double), ("init_radius", ctypes.c_double),
                ("adapt_init_buffer", ctypes.c_int32), ("adapt_term_buffer", ctypes.c_int32),
                ("adapt_window", ctypes.c_int32), ("adapt_engaged", ctypes.c_int32),
                ("seed", ctypes.c_uint64), ("init", ctypes.c_void_p), ("inv_metric", ctypes.c_void_p),
                ("skip_init_stepsize", ctypes.c_int32), ("iter_offset", ctypes.c_int32),
                ("save_warmup", ctypes.c_int32), ("shard_ids", ctypes.c_void_p),
                ("stepsize_jitter", ctypes.c_double), ("nuts_criterion", ctypes.c_int32),
                ("chains_per_wave", ctypes.c_int32)]


class RunInfo(ctypes.Structure):
    _fields_ = [("grad_evals", ctypes.c_int64), ("leapfrogs", ctypes.c_int64), ("steps", ctypes.c_int64),
                ("sweeps", ctypes.c_int64), ("sweep_ms", ctypes.c_double), ("divergent", ctypes.c_int32),
                ("errors", ctypes.c_int32), ("min_iter", ctypes.c_int32), ("done", ctypes.c_int32),
                ("shard_sweeps", ctypes.c_int64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


# (name, restype, argtypes) for every entry point declared in include/stark_hip.h
_vp, _i32, _i64, _u64, _dbl = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64, ctypes.c_double
_pp = ctypes.POINTER(ctypes.c_void_p)
SIGNATURES = [
    ("stk_last_error", ctypes.c_char_p, []),
    ("stk_version", ctypes.c_int, []),
    ("stk_config_default", None, [ctypes.POINTER(Config)]),
    ("stk_ctx_create", ctypes.c_int, [ctypes.c_int, _pp]),
    ("stk_ctx_create_on_stream", ctypes.c_int, [ctypes.c_int, _vp, _pp]),
    ("stk_ctx_destroy", ctypes.c_int, [_vp]),
    ("stk_ctx_sync", ctypes.c_int, [_vp]),
    ("stk_ctx_set_profiling", ctypes.c_int, [_vp, ctypes.c_int]),
    ("stk_ctx_stream", _vp, [_vp]),
    ("stk_model_create", ctypes.c_int, [_vp, ctypes.c_int, ctypes.POINTER(Shard), ctypes.c_int, _pp]),
    ("stk_model_create_synthetic", ctypes.c_int,
     [_vp, ctypes.c_int, ctypes.c_int, _i64, _i64, _i32, _u64, _dbl, _vp, _dbl, _pp]),
    ("stk_gen_beta", ctypes.c_int, [_u64, _i32, _vp]),
    ("stk_model_set_prior", ctypes.c_int, [_vp, _dbl, _dbl]),
    ("stk_model_destroy", ctypes.c_int, [_vp]),
    ("stk_model_info", ctypes.c_int, [_vp, ctypes.c_int, ctypes.POINTER(_i32), ctypes.POINTER(_i32),
                                      ctypes.POINTER(_i64)]),
    ("stk_model_copy_data", ctypes.c_int, [_vp, ctypes.c_int, _vp, _vp, _vp]),
    ("stk_model_device_bytes", ctypes.c_int, [_vp, ctypes.POINTER(_i64)]),
    ("stk_log_density_grad", ctypes.c_int, [_vp, ctypes.c_int, _vp, _i32, _vp, _vp]),
    ("stk_sampler_create", ctypes.c_int, [_vp, ctypes.POINTER(Config), _pp]),
    ("stk_sampler_run", ctypes.c_int, [_vp, _i32, _i64]),
    ("stk_sampler_info", ctypes.c_int, [_vp, ctypes.POINTER(RunInfo)]),
    ("stk_sampler_draws", ctypes.c_int, [_vp, ctypes.c_int, _vp, _vp]),
    ("stk_sampler_draws_unconstrained", ctypes.c_int, [_vp, ctypes.c_int, _vp]),
    ("stk_sampler_adaptation", ctypes.c_int, [_vp, _vp, _vp]),
    ("stk_sampler_iterations", ctypes.c_int, [_vp, _vp]),
    ("stk_sampler_destroy", ctypes.c_int, [_vp]),
    ("stk_sampler_state_bytes", ctypes.c_int, [_vp, ctypes.POINTER(_i64)]),
    ("stk_sampler_save_state", ctypes.c_int, [_vp, _vp, _i64]),
    ("stk_sampler_load_state", ctypes.c_int, [_vp, _vp, _i64]),
    ("stk_sampler_grad_block", ctypes.c_int, [_vp, ctypes.POINTER(_i64)]),
    ("stk_sampler_set_allreduce", ctypes.c_int, [_vp, _vp, _vp, _vp]),
    ("stk_sample", ctypes.c_int, [_vp, ctypes.POINTER(Config), _vp, _vp, ctypes.POINTER(RunInfo)]),
    ("stk_transition", ctypes.c_int, [_vp, ctypes.c_int, _vp, _i32, _u64, _i32, _dbl, _vp, _i32, _vp, _vp]),
    ("stk_consensus_products", ctypes.c_int, [_vp, _vp, _i32, _i32, _i32, _vp, _vp, _vp]),
    ("stk_consensus_solve", ctypes.c_int, [_vp, _vp, _vp, _i32, _i32, _vp]),
    ("stk_consensus", ctypes.c_int, [_vp, _vp, _i32, _i32, _i32, _vp, _vp]),
    ("stk_consensus_blocked", ctypes.c_int, [_vp, _vp, _i32, _i32, _i32, _vp, _vp, _vp]),
]

# int (*stk_allreduce_fn)(void* user, double* block, int64_t count, void* stream)
ALLREDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p)

_lib = None


def load():
    """Load the HIP library; raises loudly if it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"stark_amd: {LIB_PATH} not found -- build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(there is no CPU fallback for the hot path)")
    # One HIP runtime per process: torch's wheel bundles its own libamdhip64 (soname
    # libamdhip64.so.7, NEEDED by torch as "libamdhip64.so").  Loaded after ours, it would be
    # a second runtime that finds no GPU; loaded first, ours binds to it by soname.  So torch
    # (plumbing for torch.distributed / full-data mode) is imported before the library.
    if os.environ.get("STARK_NO_TORCH_PRELOAD") != "1":
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
    lib = ctypes.CDLL(LIB_PATH)
    for name, res, args in SIGNATURES:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc):
    if rc != STK_OK:
        msg = load().stk_last_error().decode(errors="replace")
        if rc == -7:
            raise LinAlgError(rc, msg)
        raise StarkHipError(rc, msg)
    return rc


def default_config() -> Config:
    c = Config()
    load().stk_config_default(ctypes.byref(c))
    return c
