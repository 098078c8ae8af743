"""Drop-in for ``stark/stark.py`` (randommm/stark): same names, arguments, return layout.

    from stark_amd import *                 # binds the submodule `stark` (stark/__init__.py:1)
    st = stark.Stark(sc, rdd, prepare_data_callback)
    st.setStanModel(file="schools.stan")
    weighted = st.concensusWeight(iter=5000)   # P x S consensus draws
    naive = st.distribute(n=4)                 # stacked P x S blocks, one per run

What changed underneath:
  * ``setStanModel`` recognises the program as one of the GPU model families
    (``stark_amd.frontend``) instead of compiling it with pystan;
  * every partition is a shard resident on a GPU; all local shards sample in ONE batched
    NUTS run (``libstark_hip.so``), one process per GPU, partition p on rank p % world;
  * the only exchange is one all-gather of the P x S draw matrices (RCCL), then the
    consensus combine runs as gfx950 kernels in partition order.

Deliberate deviations from the reference code, each mirroring its evident intent
(DESIGN.md "Reference bugs"): the combine accepts any number of partitions (the reference
reducer only works for two); shards with NaN draws are left out of the combine; naive
mode runs ``n`` full-data replicas (the reference's non-accumulating ``union`` runs the
partitions plus one full copy -- available as ``distribute(..., reference_union=True)``).
Draws follow pystan's ``fit.extract()`` (``permuted=True``, stark/stark.py:49): each chain's
post-warmup draws in a seeded random order, chains concatenated; ``permuted=False`` keeps
chain order (what the sampler's diagnostics need).
"""
from __future__ import annotations

import inspect

import numpy as np

from . import dist, engine, frontend
from . import rdd as _rdd


def consensus_avg(J):
    """Pairwise reducer of stark/stark.py:7-21 on the GPU.

    ``c(f1, f2)`` returns ``[W1 + W2, W1 f1 + W2 f2]`` with ``W = inv(np.cov(f))``; if f1
    holds a NaN it returns f2 unchanged (:9-10).  Unlike the reference, f1 may also be the
    ``[sum W, sum W theta]`` pair of an earlier step, so ``functools.reduce`` works for any
    number of partitions.  ``J`` is ignored, as in the reference (:7)."""

    def c(f1, f2):
        if isinstance(f1, list):
            sw, swt = f1
            f2 = np.asarray(f2, np.float64)
            if np.isnan(f2).any():          # a NaN shard later in the reduce is left out
                return [sw, swt]
            w2, w2t, _ = engine.consensus_products([f2])
            return [sw + w2, swt + w2t]
        f1 = np.asarray(f1, np.float64)
        if np.isnan(f1).any():
            return f2
        sw, swt, _ = engine.consensus_products([f1, np.asarray(f2, np.float64)])
        return [sw, swt]

    return c


def concatenate_samples(a, b):
    """stark/stark.py:23-24."""
    return np.vstack((a, b))


def permute_draws(draws, chains: int, seed: int, partition: int):
    """pystan 2 ``extract(permuted=True)`` order for one partition's P x (chains * n) matrix
    (chain-major columns): every chain's n draws in a random order, chains concatenated.
    The permutation is a pure function of (seed, partition, chain) -- numpy's Philox
    counter-based generator keyed by the sampling seed -- so a run is reproducible on 1 or N
    GPUs.  (pystan draws its permutations from numpy's global RandomState; the order is
    arbitrary either way, what matters to the reference's combine is that draw i of every
    partition is paired after the shuffle, stark/stark.py:20.)"""
    draws = np.asarray(draws)
    P, S = draws.shape
    if S % chains:
        raise ValueError("draw columns must be chains x draws")
    n = S // chains
    cols = []
    for c in range(chains):
        g = np.random.Generator(np.random.Philox(key=[int(seed) & 0xFFFFFFFFFFFFFFFF,
                                                      (int(partition) << 32) | int(c)]))
        cols.append(c * n + g.permutation(n))
    return np.ascontiguousarray(draws[:, np.concatenate(cols)]) if cols else draws


def _extract_to_matrix(extract):
    """stark/stark.py:49-56: extract() values in key order, 1-D params as (S, 1) columns,
    hstack, transpose -> variables x samples."""
    h = [np.array(v) for v in extract.values()]
    for prm in h:
        if len(prm.shape) == 1:
            prm.shape = (prm.shape[0], 1)
    return np.transpose(np.hstack(h))


_CONTROL_KEYS = {"adapt_delta": "adapt_delta", "max_treedepth": "max_depth", "stepsize": "stepsize",
                 "adapt_gamma": "adapt_gamma", "adapt_kappa": "adapt_kappa", "adapt_t0": "adapt_t0",
                 "adapt_init_buffer": "adapt_init_buffer", "adapt_term_buffer": "adapt_term_buffer",
                 "adapt_window": "adapt_window", "adapt_engaged": "adapt_engaged", "inv_metric": "inv_metric",
                 "stepsize_jitter": "stepsize_jitter", "nuts_criterion": "nuts_criterion"}


def _unconstrain(family, data, init_dict):
    """Constrained parameter values (a pystan init dict) -> unconstrained vector."""
    if family == "schools":
        J = int(data["J"])
        eta = np.asarray(init_dict.get("eta", np.zeros(J)), np.float64).reshape(J)
        return np.concatenate([[float(init_dict.get("mu", 0.0)), np.log(float(init_dict.get("tau", 1.0)))], eta])
    K = int(data["K"])
    v = [float(init_dict.get("alpha", 0.0))] + list(np.asarray(init_dict.get("beta", np.zeros(K)), np.float64).reshape(K))
    if family == "linear":
        v.append(np.log(float(init_dict.get("sigma", 1.0))))
    return np.asarray(v)


def thin_draws(draws, chains, thin):
    """Stan's num_thin: of each chain's post-warmup iterations m = 0, 1, ... keep those with
    m % thin == 0 (ceil(S / thin) draws per chain; services/util/generate_transitions), columns
    chain-major as the sampler writes them."""
    if thin == 1:
        return draws
    P, n = draws.shape
    return np.ascontiguousarray(draws.reshape(P, chains, n // chains)[:, :, ::thin].reshape(P, -1))


def sampling_config(family, datas, **kw):
    """pystan 2 ``StanModel.sampling`` keywords -> engine config (stark/stark.py:48)."""
    kw = dict(kw)
    it = int(kw.pop("iter", 2000))
    warmup = int(kw.pop("warmup", it // 2))
    chains = int(kw.pop("chains", 4))
    kw.pop("n_jobs", None)
    thin = int(kw.pop("thin", 1))
    if thin < 1:
        raise ValueError("thin must be a positive integer")
    seed = kw.pop("seed", None)
    if seed is None:
        seed = int(np.random.SeedSequence().entropy) & 0x7FFFFFFF
    control = dict(kw.pop("control", None) or {})
    if control.pop("metric", "diag_e") != "diag_e":
        raise NotImplementedError("only metric='diag_e' (Stan's default) is supported")
    cfg = dict(num_warmup=warmup, num_samples=it - warmup, chains=chains, seed=seed, thin=thin)
    for k, v in control.items():
        if k not in _CONTROL_KEYS:
            raise ValueError(f"unknown control key {k!r}")
        cfg[_CONTROL_KEYS[k]] = v
    init = kw.pop("init", "random")
    init_r = float(kw.pop("init_r", 2.0))
    cfg["init_radius"] = init_r
    if isinstance(init, (int, float)) or (isinstance(init, str) and init == "0"):
        if float(init) != 0.0:
            raise ValueError("numeric init must be 0")
        init = "0"
    if init == "0":
        D = [len(_unconstrain(family, d, {})) for d in datas]
        cfg["init"] = np.concatenate([np.zeros(Ds * chains) for Ds in D])
    elif callable(init):
        # pystan 2: init(chain_id=...) per chain when the function takes a chain_id, else init();
        # decided from the signature, so a TypeError raised inside the user's function propagates
        # (chain_id = 0 .. chains - 1: parity unpinned against pystan)
        try:
            params = inspect.signature(init).parameters
            takes_id = "chain_id" in params or any(p.kind == p.VAR_KEYWORD for p in params.values())
        except (TypeError, ValueError):          # no introspectable signature (some builtins)
            takes_id = False
        dicts = [init(chain_id=c) if takes_id else init() for c in range(chains)]
        cfg["init"] = np.concatenate([_unconstrain(family, d, dicts[c]) for d in datas for c in range(chains)])
    elif isinstance(init, (list, tuple)):
        if len(init) != chains:
            raise ValueError("init list must have one dict per chain")
        cfg["init"] = np.concatenate([_unconstrain(family, d, init[c]) for d in datas for c in range(chains)])
    elif init != "random":
        raise ValueError(f"unsupported init {init!r}")
    for k in ("sample_file", "diagnostic_file"):
        # pystan writes Stan CSV files here; this build returns draws only, so a caller who asks
        # for a file is told, not silently handed none
        if kw.pop(k, None) is not None:
            raise NotImplementedError(f"{k}= (pystan's CSV output) is not supported: the draws are returned in memory")
    for k in ("verbose", "refresh", "check_hmc_diagnostics", "algorithm"):
        v = kw.pop(k, None)
        if k == "algorithm" and v not in (None, "NUTS"):
            raise NotImplementedError("only algorithm='NUTS' is supported")
    if kw:
        raise TypeError(f"unsupported sampling arguments: {sorted(kw)}")
    return cfg


class Stark:
    """Driver of stark/stark.py:26-85 over GPU shards."""
    rdd = None
    n_partitions = None
    prepare_data_callback = None

    def __init__(self, context, rdd, prepare_data_callback):
        self.rdd = rdd
        self.context = context
        self.prepare_data_callback = prepare_data_callback
        self.n_partitions = self.rdd.getNumPartitions()
        self.family = None
        self.priors = {}
        self.last_run = None

    def setStanModel(self, **kwargs):
        """stark/stark.py:37-39; accepts pystan.StanModel's file= / model_code= (+ family=)."""
        self.family, self.priors = frontend.load_program_info(**kwargs)
        self.stan_kwargs = kwargs

    # ---- per-partition sampling (stark/stark.py:41-57), batched over partitions
    def _sample_partitions(self, datas, shard_ids=None, permuted=True, pars=None, include=True, **kwargs):
        """Run every data dict as one shard of a single GPU model; returns one P x S matrix
        per data dict, rows in extract() order (params, transformed params, lp__), columns in
        ``extract(permuted=True)`` order (``permute_draws``) unless permuted=False.
        shard_ids: global partition index of each data dict (keys the RNG streams, so a
        partition samples identically on 1 or N GPUs).  pars / include: pystan 2's parameter
        selection (``frontend.select_pars``): only those rows (+ lp__) reach the P x S matrix,
        and so the combine, as in the reference (stark/stark.py:48-56)."""
        if self.family is None:
            raise RuntimeError("call setStanModel() first")
        rows = [frontend.select_pars(self.family, d, pars, include) for d in datas]   # validates first
        draws = self._draw_partitions(datas, shard_ids=shard_ids, permuted=permuted, **kwargs)
        return [d if r is None else np.ascontiguousarray(d[r]) for d, r in zip(draws, rows)]

    def _draw_partitions(self, datas, shard_ids=None, permuted=True, **kwargs):
        """The GPU run behind _sample_partitions: every extract() row of every partition."""
        shards = [frontend.pack_data(self.family, d) for d in datas]
        cfg = sampling_config(self.family, datas, **kwargs)
        if shard_ids is not None:
            cfg["shard_ids"] = shard_ids
        thin = cfg.pop("thin", 1)
        model = engine.Model(engine.default_context(), self.family, shards)
        if getattr(self, "priors", None):
            model.set_prior(**self.priors)
        try:
            res = model.sample(**cfg)
        finally:
            model.close()
        draws = [thin_draws(d, cfg["chains"], thin) for d in res.draws]
        if thin > 1:   # last_run holds what the caller got: the thinned draws and their stats
            idx = thin_draws(np.arange(res.chains * res.num_samples)[None, :], res.chains, thin)[0]
            res = engine.SampleResult(draws, [st[idx] for st in res.stats], res.info, res.chains, len(idx) // res.chains)
        self.last_run = res
        if not permuted:
            return draws
        ids = shard_ids if shard_ids is not None else range(len(datas))
        return [permute_draws(d, cfg["chains"], cfg["seed"], p) for d, p in zip(draws, ids)]

    def _mcmc(self, callback, **kwargs):
        def w(sts):
            sts = list(sts)
            data = callback(sts)
            return [self._sample_partitions([data], **kwargs)[0]]
        return w

    @staticmethod
    def _defaults(kwargs):
        if "iter" not in kwargs:
            kwargs["iter"] = 2000
        if "chains" not in kwargs:
            kwargs["chains"] = 1
        kwargs["n_jobs"] = 1
        return kwargs

    def _run_distributed(self, parts, **kwargs):
        rank, ws = dist.world()
        mine = dist.local_partitions(len(parts), rank, ws)
        datas = [self.prepare_data_callback(list(parts[p])) for p in mine]
        local = dict(zip(mine, self._sample_partitions(datas, shard_ids=mine, **kwargs))) if datas else {}
        return dist.all_gather_partitions(local, len(parts))

    def concensusWeight(self, separate_lp=False, **kwargs):
        """stark/stark.py:59-71: subposterior per partition, consensus weighted average.

        The default reproduces the REFERENCE's combine, for parity: every extract() row is
        combined jointly, lp__ included.  That is not the accurate choice: each shard's lp__
        sits at its own offset, many lp__ sds from the others, and the sampled lp__-parameter
        cross-covariances turn that offset into an error of the parameter means (mean z^2 of
        4-7 at N = 1e8).  For accuracy pass separate_lp=True: lp__ gets a
        1 x 1 weight block of its own and the parameters are combined from their own
        covariance (engine.consensus).  permuted=False keeps chain order in the draws.

        Raises stark_amd._lib.LinAlgError when a shard holds too few draws for
        its covariance to be invertible: each shard needs more than P draws, i.e.
        ceil((iter - warmup) / thin) * chains > P (P = the model's parameters + lp__; with separate_lp the
        parameters alone).  The reference's np.linalg.inv returns rounding noise there instead
        (DESIGN.md section 9)."""
        kwargs = self._defaults(kwargs)
        parts = _rdd.partitions_of(self.rdd)
        subposteriors = self._run_distributed(parts, **kwargs)
        out, _ = engine.consensus(subposteriors, separate_lp=separate_lp)
        return out

    def distribute(self, n=2, reference_union=False, **kwargs):
        """stark/stark.py:73-85: naive parallel runs over the full data, draws stacked with
        ``concatenate_samples`` (row blocks of P x S)."""
        kwargs = self._defaults(kwargs)
        parts = _rdd.partitions_of(self.rdd)
        full = [row for p in parts for row in p]
        if reference_union and n >= 2:
            runs = parts + [full]
        else:
            runs = [full] * n
        posteriors = self._run_distributed(runs, **kwargs)
        out = posteriors[0]
        for b in posteriors[1:]:
            out = concatenate_samples(out, b)
        return out
