"""Object layer over ``libstark_hip.so``: contexts, shard models, samplers, combine.

This is the host side of the hot path; ``stark_amd.stark`` builds the reference's driver
API (``stark/stark.py``) on top of it and ``bench.py`` drives it directly with synthetic
shards generated in HBM.
"""
from __future__ import annotations

import atexit
import ctypes
import weakref
from dataclasses import dataclass, field

import numpy as np

from . import _lib
from ._lib import (N_STATS, STAT_NAMES, STK_LINREG, STK_LOGREG, STK_SCHOOLS, Config, RunInfo, Shard,
                   StarkHipError, check)

FAMILIES = {"schools": STK_SCHOOLS, "linear": STK_LINREG, "logistic": STK_LOGREG}

# Live library handles, closed in dependency order (samplers, models, contexts) before the
# HIP runtime's own exit handlers run; after that every close() is a no-op.
_live = {"sampler": weakref.WeakSet(), "model": weakref.WeakSet(), "ctx": weakref.WeakSet()}
_finalized = False


@atexit.register
def _shutdown():
    global _finalized
    for kind in ("sampler", "model", "ctx"):
        for obj in list(_live[kind]):
            try:
                obj.close()
            except Exception:
                pass
    _finalized = True
FAMILY_NAMES = {v: k for k, v in FAMILIES.items()}


def _ptr(a):
    """Address of a host numpy array or a device torch tensor (None -> NULL)."""
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        if not a.flags["C_CONTIGUOUS"]:
            raise ValueError("array must be C-contiguous")
        return a.ctypes.data
    if hasattr(a, "data_ptr"):
        if not a.is_contiguous():
            raise ValueError("tensor must be contiguous")
        return a.data_ptr()
    raise TypeError(f"unsupported buffer type {type(a)}")


class Context:
    """One device + one HIP stream (``stk_ctx``)."""

    def __init__(self, device: int = 0, profiling: bool = False, stream: int | None = None):
        """stream: None (the context's own HIP stream) or a caller's hipStream_t handle, e.g.
        ``torch.cuda.current_stream(device).cuda_stream``, so the library's kernels and the
        caller's torch.distributed collectives are ordered on one stream (full-data mode)."""
        lib = _lib.load()
        h = ctypes.c_void_p()
        if stream is None:
            check(lib.stk_ctx_create(int(device), ctypes.byref(h)))
        else:
            check(lib.stk_ctx_create_on_stream(int(device), ctypes.c_void_p(int(stream)), ctypes.byref(h)))
        self._h = h
        self.device = device
        _live["ctx"].add(self)
        if profiling:
            self.set_profiling(True)

    def set_profiling(self, on):
        """HIP events around the data sweeps: False/0 off, True/1 every step, n > 1 every n-th
        step (the events are stream barriers; sampling keeps them off the step time)."""
        check(_lib.load().stk_ctx_set_profiling(self._h, int(on)))

    def sync(self):
        check(_lib.load().stk_ctx_sync(self._h))

    @property
    def stream(self) -> int:
        return _lib.load().stk_ctx_stream(self._h) or 0

    def close(self):
        if getattr(self, "_h", None) and not _finalized:
            _lib.load().stk_ctx_destroy(self._h)
        self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_default_ctx: dict[int, Context] = {}


def default_context(device: int | None = None) -> Context:
    if device is None:
        import os
        device = int(os.environ.get("LOCAL_RANK", "0"))
    if device not in _default_ctx:
        _default_ctx[device] = Context(device)
    return _default_ctx[device]


@dataclass
class SampleResult:
    draws: list            # per shard: P x (chains*num_samples), columns chain-major
    stats: list            # per shard: (chains*num_samples) x 6
    info: dict
    chains: int
    num_samples: int
    stat_names: tuple = field(default=STAT_NAMES)


def make_config(num_warmup=1000, num_samples=1000, chains=1, max_depth=10, adapt_delta=0.8, adapt_gamma=0.05,
                adapt_kappa=0.75, adapt_t0=10.0, stepsize=1.0, init_radius=2.0, adapt_init_buffer=75,
                adapt_term_buffer=50, adapt_window=25, adapt_engaged=True, seed=1234, init=None,
                inv_metric=None, skip_init_stepsize=False, iter_offset=0, shard_ids=None,
                save_warmup=False, stepsize_jitter=0.0, nuts_criterion="stan2.19", chains_per_wave=0):
    """Stan sampler settings (pystan 2 `sampling()` keywords + control block).
    nuts_criterion: "stan2.19" (the reference's pystan 2: one U-turn test per merged subtree)
    or "stan2.23" (plus the checks across subtree junctions of Stan >= 2.23)."""
    c = _lib.default_config()
    c.num_warmup, c.num_samples, c.chains, c.max_depth = int(num_warmup), int(num_samples), int(chains), int(max_depth)
    c.adapt_delta, c.adapt_gamma, c.adapt_kappa, c.adapt_t0 = adapt_delta, adapt_gamma, adapt_kappa, adapt_t0
    c.stepsize, c.init_radius = stepsize, init_radius
    c.stepsize_jitter = float(stepsize_jitter)
    crit = {"stan2.19": 0, "stan2.23": 1, 0: 0, 1: 1}
    if nuts_criterion not in crit:
        raise ValueError(f"nuts_criterion must be 'stan2.19' or 'stan2.23', got {nuts_criterion!r}")
    c.nuts_criterion = crit[nuts_criterion]
    c.chains_per_wave = int(chains_per_wave)
    c.adapt_init_buffer, c.adapt_term_buffer, c.adapt_window = adapt_init_buffer, adapt_term_buffer, adapt_window
    c.adapt_engaged = int(bool(adapt_engaged))
    c.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    keep = []
    if init is not None:
        init = np.ascontiguousarray(init, np.float64)
        keep.append(init)
        c.init = init.ctypes.data
    if inv_metric is not None:
        inv_metric = np.ascontiguousarray(inv_metric, np.float64)
        keep.append(inv_metric)
        c.inv_metric = inv_metric.ctypes.data
    if shard_ids is not None:
        shard_ids = np.ascontiguousarray(shard_ids, np.int32)
        keep.append(shard_ids)
        c.shard_ids = shard_ids.ctypes.data
    c.skip_init_stepsize = int(bool(skip_init_stepsize))
    c.save_warmup = int(bool(save_warmup))
    c.iter_offset = int(iter_offset)
    c._keep = keep   # keep buffers alive with the struct
    return c


class Model:
    """Shards of one model family resident on one device (``stk_model``)."""

    def __init__(self, ctx: Context, family, shards=None, _handle=None):
        self.ctx = ctx
        self.family = FAMILIES.get(family, family)
        if _handle is not None:
            self._h = _handle
        else:
            self._h = self._create(shards)
        _live["model"].add(self)
        lib = _lib.load()
        self.nshards = len(shards) if shards is not None else self._nshards
        self.D, self.P, self.n_rows = [], [], []
        for s in range(self.nshards):
            D, P, n = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int64()
            check(lib.stk_model_info(self._h, s, ctypes.byref(D), ctypes.byref(P), ctypes.byref(n)))
            self.D.append(D.value)
            self.P.append(P.value)
            self.n_rows.append(n.value)

    def _create(self, shards):
        keep = []
        arr = (Shard * len(shards))()
        for i, sh in enumerate(shards):
            if self.family == STK_SCHOOLS:
                y = np.ascontiguousarray(sh["y"], np.float64)
                sig = np.ascontiguousarray(sh["sigma"], np.float64)
                if y.shape != sig.shape or y.ndim != 1:
                    raise ValueError("schools shard: y and sigma must be equal-length vectors")
                keep += [y, sig]
                arr[i] = Shard(len(y), 0, None, y.ctypes.data, None, sig.ctypes.data)
            else:
                x = np.ascontiguousarray(sh["x"], np.float64)
                if x.ndim != 2:
                    raise ValueError("regression shard: x must be N x K")
                if self.family == STK_LOGREG:
                    y = np.ascontiguousarray(sh["y"], np.int32)
                    if np.any((y != 0) & (y != 1)):
                        raise ValueError("bernoulli_logit: y must be 0 or 1")
                    arr[i] = Shard(x.shape[0], x.shape[1], x.ctypes.data, None, y.ctypes.data, None)
                else:
                    y = np.ascontiguousarray(sh["y"], np.float64)
                    arr[i] = Shard(x.shape[0], x.shape[1], x.ctypes.data, y.ctypes.data, None, None)
                if y.shape[0] != x.shape[0]:
                    raise ValueError("x and y row counts differ")
                keep += [x, y]
        h = ctypes.c_void_p()
        check(_lib.load().stk_model_create(self.ctx._h, self.family, arr, len(shards), ctypes.byref(h)))
        return h

    @classmethod
    def synthetic(cls, ctx: Context, family, nshards: int, rows_per_shard: int, n_cols: int, data_seed: int = 20240,
                  row_offset: int = 0, alpha: float = 0.0, beta=None, noise_sigma: float = 1.0):
        """Shards generated in HBM by the Philox generator."""
        fam = FAMILIES.get(family, family)
        b = None
        if beta is not None:
            b = np.ascontiguousarray(beta, np.float64)
        h = ctypes.c_void_p()
        check(_lib.load().stk_model_create_synthetic(ctx._h, fam, nshards, int(rows_per_shard), int(row_offset),
                                                     int(n_cols), int(data_seed), float(alpha), _ptr(b),
                                                     float(noise_sigma), ctypes.byref(h)))
        obj = cls.__new__(cls)
        obj._nshards = nshards
        Model.__init__(obj, ctx, fam, None, _handle=h)
        return obj

    @staticmethod
    def gen_beta(data_seed: int, n_cols: int) -> np.ndarray:
        b = np.empty(n_cols, np.float64)
        check(_lib.load().stk_gen_beta(int(data_seed), int(n_cols), b.ctypes.data))
        return b

    def device_bytes(self) -> int:
        v = ctypes.c_int64()
        check(_lib.load().stk_model_device_bytes(self._h, ctypes.byref(v)))
        return v.value

    def copy_data(self, shard: int):
        n, D = self.n_rows[shard], self.D[shard]
        lib = _lib.load()
        if self.family == STK_SCHOOLS:
            y = np.empty(n)
            check(lib.stk_model_copy_data(self._h, shard, None, y.ctypes.data, None))
            return {"y": y}
        d = D - (1 if self.family == STK_LOGREG else 2)
        x = np.empty((n, d))
        if self.family == STK_LOGREG:
            y = np.empty(n, np.int32)
            check(lib.stk_model_copy_data(self._h, shard, x.ctypes.data, None, y.ctypes.data))
        else:
            y = np.empty(n)
            check(lib.stk_model_copy_data(self._h, shard, x.ctypes.data, y.ctypes.data, None))
        return {"x": x, "y": y}

    def log_density_grad(self, shard: int, q):
        """lp and grad lp (Stan log_prob, propto, jacobian) at C points (C x D)."""
        q = np.ascontiguousarray(np.atleast_2d(q), np.float64)
        C, D = q.shape
        if D != self.D[shard]:
            raise ValueError(f"q has {D} columns, shard {shard} has D = {self.D[shard]}")
        lp = np.empty(C)
        g = np.empty((C, D))
        check(_lib.load().stk_log_density_grad(self._h, shard, q.ctypes.data, C, lp.ctypes.data, g.ctypes.data))
        return lp, g

    def set_prior(self, alpha=None, beta=None):
        """normal(0, s) priors on alpha and beta (regressions); None or 0: flat."""
        check(_lib.load().stk_model_set_prior(self._h, float(alpha or 0.0), float(beta or 0.0)))
        self.prior = {"alpha": alpha, "beta": beta}
        return self

    def sampler(self, **cfg) -> "Sampler":
        return Sampler(self, make_config(**cfg))

    def sample(self, **cfg) -> SampleResult:
        s = self.sampler(**cfg)
        try:
            s.run()
            return s.result()
        finally:
            s.close()

    def transition(self, shard, q, *, seed, iteration, eps, inv_metric=None, max_depth=10):
        """One fixed-step NUTS transition per row of q (parity hook, see stk_transition)."""
        q = np.array(np.atleast_2d(q), np.float64, copy=True, order="C")
        C = q.shape[0]
        lp = np.empty(C)
        st = np.empty((C, N_STATS))
        im = None if inv_metric is None else np.ascontiguousarray(inv_metric, np.float64)
        check(_lib.load().stk_transition(self._h, shard, q.ctypes.data, C, int(seed), int(iteration), float(eps),
                                         _ptr(im), int(max_depth), lp.ctypes.data, st.ctypes.data))
        return q, lp, st

    def close(self):
        if getattr(self, "_h", None) and not _finalized:
            _lib.load().stk_model_destroy(self._h)
        self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Sampler:
    """Resumable NUTS run over every shard of a model (``stk_sampler``)."""

    def __init__(self, model: Model, cfg: Config):
        self.model = model
        self.cfg = cfg
        h = ctypes.c_void_p()
        check(_lib.load().stk_sampler_create(model._h, ctypes.byref(cfg), ctypes.byref(h)))
        self._h = h
        self.total = cfg.num_warmup + cfg.num_samples
        _live["sampler"].add(self)

    def run(self, target_iter: int | None = None, max_steps: int = 0):
        """Advance every chain to `target_iter` completed transitions (default: all)."""
        t = self.total if target_iter is None else int(target_iter)
        check(_lib.load().stk_sampler_run(self._h, t, int(max_steps)))
        return self

    def grad_block(self) -> int:
        """Doubles in the per-step [grad | lp] block that full-data mode sums over ranks."""
        n = ctypes.c_int64()
        check(_lib.load().stk_sampler_grad_block(self._h, ctypes.byref(n)))
        return int(n.value)

    def set_allreduce(self, fn, block_ptr: int | None = None):
        """Full-data mode: fn(block_ptr, count, stream) -> None is called after every step's
        local sweep + reduce and must leave the sum over ranks in the block (stk_sampler_set_allreduce)."""
        def _cb(user, ptr, count, stream):
            try:
                fn(ptr, count, stream)
                return 0
            except Exception as e:   # reported through the library's error path
                self._cb_error = e
                return -1
        self._cb = _lib.ALLREDUCE_FN(_cb)            # keep the trampoline alive with the sampler
        check(_lib.load().stk_sampler_set_allreduce(self._h, self._cb, None,
                                                    ctypes.c_void_p(block_ptr) if block_ptr else None))
        return self

    def save_state(self) -> np.ndarray:
        """The run so far as a byte blob (uint8 array): every chain's device state, the draws
        and the step counters (stk_sampler_save_state).  load_state() of the blob into a sampler
        of the same model geometry and config -- in another process, on another GPU --
        continues the run bit for bit as if it had never stopped."""
        n = ctypes.c_int64()
        lib = _lib.load()
        check(lib.stk_sampler_state_bytes(self._h, ctypes.byref(n)))
        buf = np.empty(n.value, np.uint8)
        check(lib.stk_sampler_save_state(self._h, buf.ctypes.data, n.value))
        return buf

    def load_state(self, blob) -> "Sampler":
        """Resume a run saved by save_state() (raises StarkHipError on another geometry / config)."""
        buf = np.ascontiguousarray(np.frombuffer(blob, np.uint8) if isinstance(blob, (bytes, bytearray)) else blob,
                                   np.uint8)
        check(_lib.load().stk_sampler_load_state(self._h, buf.ctypes.data, buf.size))
        return self

    def info(self) -> dict:
        ri = RunInfo()
        check(_lib.load().stk_sampler_info(self._h, ctypes.byref(ri)))
        return ri.as_dict()

    def draws(self, shard: int):
        S = self.cfg.chains * self.cfg.num_samples
        out = np.empty((self.model.P[shard], S))
        st = np.empty((S, N_STATS))
        check(_lib.load().stk_sampler_draws(self._h, shard, out.ctypes.data, st.ctypes.data))
        return out, st

    def draws_device(self, shard: int, out=None):
        """The draws of one shard, P x (chains * num_samples), copied device-to-device into a
        torch fp64 tensor on the context's GPU (allocated if `out` is None); no host copy."""
        import torch
        S = self.cfg.chains * self.cfg.num_samples
        if out is None:
            out = torch.empty((self.model.P[shard], S), dtype=torch.float64, device=f"cuda:{self.model.ctx.device}")
        if tuple(out.shape) != (self.model.P[shard], S) or out.dtype != torch.float64 or not out.is_cuda:
            raise ValueError(f"out must be a cuda fp64 tensor of shape {(self.model.P[shard], S)}")
        torch.cuda.current_stream(out.device).synchronize()
        check(_lib.load().stk_sampler_draws(self._h, shard, _ptr(out), None))
        return out

    def unconstrained(self, shard: int):
        n = self.cfg.num_samples + (self.cfg.num_warmup if self.cfg.save_warmup else 0)
        out = np.empty((self.cfg.chains, n, self.model.D[shard]))
        check(_lib.load().stk_sampler_draws_unconstrained(self._h, shard, out.ctypes.data))
        return out

    def iterations(self) -> np.ndarray:
        """Transitions completed by every chain (shard-major), warmup included."""
        n = self.model.nshards * self.cfg.chains
        out = np.empty(n, np.int32)
        check(_lib.load().stk_sampler_iterations(self._h, out.ctypes.data))
        return out

    def adaptation(self):
        n = self.model.nshards * self.cfg.chains
        eps = np.empty(n)
        im = np.zeros((n, max(self.model.D)))
        check(_lib.load().stk_sampler_adaptation(self._h, eps.ctypes.data, im.ctypes.data))
        return eps, im

    def result(self) -> SampleResult:
        info = self.info()
        if info["errors"]:
            raise StarkHipError(-5, f"{info['errors']} chain(s) stopped: step size left (0, 1e7] in init_stepsize")
        draws, stats = [], []
        for s in range(self.model.nshards):
            d, st = self.draws(s)
            draws.append(d)
            stats.append(st)
        return SampleResult(draws, stats, info, self.cfg.chains, self.cfg.num_samples)

    def close(self):
        if getattr(self, "_h", None) and not _finalized:
            _lib.load().stk_sampler_destroy(self._h)
        self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ---------------------------------------------------------------- combine
def _stack(draws):
    d = [np.ascontiguousarray(x, np.float64) for x in draws]
    shapes = {x.shape for x in d}
    if len(shapes) != 1:
        # stark/stark.py:20 broadcasts W0.f1 + W1.f2 and fails on unequal shapes
        raise ValueError(f"shards must share one (P, S) shape, got {sorted(shapes)}")
    return np.ascontiguousarray(np.stack(d)), d[0].shape


def _device_stack(draws):
    """draws as ONE contiguous [nshards, P, S] fp64 cuda tensor, or None for host input."""
    try:
        import torch
    except ImportError:          # pragma: no cover
        return None
    if isinstance(draws, torch.Tensor):
        t = draws
    elif isinstance(draws, (list, tuple)) and draws and all(isinstance(x, torch.Tensor) for x in draws):
        if len({tuple(x.shape) for x in draws}) != 1:
            raise ValueError(f"shards must share one (P, S) shape, got {sorted({tuple(x.shape) for x in draws})}")
        t = torch.stack(list(draws))
    else:
        return None
    if t.dim() != 3:
        raise ValueError("draws tensor must be [nshards, P, S]")
    if not t.is_cuda:
        return None
    return t.to(torch.float64).contiguous()


def consensus(draws, ctx: Context | None = None, separate_lp: bool = False):
    """(sum_s W_s)^-1 sum_s W_s theta_s, W_s = inv(cov(theta_s)): stark/stark.py:66-70 over
    the reducer stark/stark.py:7-21.  Returns (P x S, shard_used).

    draws: a list of P x S host arrays, or device-resident draws -- a [nshards, P, S] cuda
    tensor (e.g. dist.all_gather_partitions(..., as_tensor=True)) or a list of P x S cuda
    tensors.  Device draws are combined where they lie (no host round trip) and the result is
    a P x S cuda tensor on the same device.

    separate_lp: the last row (lp__, which fit.extract() hands the reference's combine,
    stark/stark.py:49-56) gets a 1 x 1 weight block of its own instead of joining the parameter
    rows' covariance.  Each shard's lp__ sits at its own offset, many of its sds apart; with a
    sample covariance, the noise in the lp__-parameter cross terms moves the parameter rows of
    the joint combine by a multiple of that offset.  Block weights are exact for a Gaussian
    posterior, where lp__ is uncorrelated with the parameters."""
    ctx = ctx or default_context()
    dev = _device_stack(draws)
    if dev is not None:
        import torch
        ns, P, S = (int(v) for v in dev.shape)
        if dev.device.index != ctx.device:
            raise ValueError(f"draws on {dev.device} but the context is on cuda:{ctx.device}: pass a context "
                             f"of the draws' device (engine.Context({dev.device.index}))")
        out_t = torch.empty((P, S), dtype=torch.float64, device=dev.device)
        used = np.empty(ns, np.int32)
        torch.cuda.current_stream(dev.device).synchronize()    # the library runs on its own stream
        if separate_lp:
            blk = np.zeros(P, np.int32)
            blk[-1] = 1
            check(_lib.load().stk_consensus_blocked(ctx._h, _ptr(dev), ns, P, S, blk.ctypes.data, _ptr(out_t),
                                                    used.ctypes.data))
        else:
            check(_lib.load().stk_consensus(ctx._h, _ptr(dev), ns, P, S, _ptr(out_t), used.ctypes.data))
        return out_t, used.astype(bool)
    if not isinstance(draws, (list, tuple)) and hasattr(draws, "numpy"):    # a host torch tensor
        draws = list(draws.numpy())
    X, (P, S) = _stack(draws)
    out = np.empty((P, S))
    used = np.empty(len(draws), np.int32)
    if separate_lp:
        # one call with block-diagonal weights: parameters in block 0, lp__ (last row) in block 1;
        # the NaN mask is per shard over all rows, so both blocks combine the same shard set
        blk = np.zeros(P, np.int32)
        blk[-1] = 1
        check(_lib.load().stk_consensus_blocked(ctx._h, X.ctypes.data, len(draws), P, S, blk.ctypes.data,
                                                out.ctypes.data, used.ctypes.data))
        return out, used.astype(bool)
    check(_lib.load().stk_consensus(ctx._h, X.ctypes.data, len(draws), P, S, out.ctypes.data, used.ctypes.data))
    return out, used.astype(bool)


def consensus_products(draws, ctx: Context | None = None):
    """[sum W_s, sum W_s theta_s] -- the value the reference reducer returns (stark/stark.py:19-20)."""
    ctx = ctx or default_context()
    X, (P, S) = _stack(draws)
    sw = np.empty((P, P))
    swt = np.empty((P, S))
    used = np.empty(len(draws), np.int32)
    check(_lib.load().stk_consensus_products(ctx._h, X.ctypes.data, len(draws), P, S, sw.ctypes.data,
                                             swt.ctypes.data, used.ctypes.data))
    return sw, swt, used.astype(bool)


def consensus_solve(sum_w, sum_wtheta, ctx: Context | None = None):
    """inv(sum W) . sum W theta (stark/stark.py:67-70)."""
    ctx = ctx or default_context()
    sw = np.ascontiguousarray(sum_w, np.float64)
    swt = np.ascontiguousarray(sum_wtheta, np.float64)
    P, S = swt.shape
    out = np.empty((P, S))
    check(_lib.load().stk_consensus_solve(ctx._h, sw.ctypes.data, swt.ctypes.data, P, S, out.ctypes.data))
    return out
