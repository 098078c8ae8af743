"""GPU NUTS (iterative per-chain state machine) vs the oracle's recursive Stan 2.19 twin,
exact posterior moments, and reproducibility across runs / shard placements."""
import os

import numpy as np
import pytest

from stark_amd.diagnostics import ess

pytestmark = pytest.mark.gpu


def _schools_model(ctx, orc):
    from stark_amd import engine
    shards = [{"y": orc.SCHOOLS_Y[:4], "sigma": orc.SCHOOLS_SIGMA[:4]},
              {"y": orc.SCHOOLS_Y, "sigma": orc.SCHOOLS_SIGMA}]
    return engine.Model(ctx, "schools", shards), shards


# ---------------------------------------------------------------- one transition, same RNG stream
@pytest.mark.parametrize("eps", [0.05, 0.3, 0.9, 2.5])
def test_transition_matches_oracle_schools(ctx, orc, eps):
    m, shards = _schools_model(ctx, orc)
    rng = np.random.default_rng(int(eps * 100))
    C = 8
    for shard in (0, 1):
        om = orc.Model(orc.FAM_SCHOOLS, y=shards[shard]["y"], sigma=shards[shard]["sigma"])
        q0 = rng.normal(0, 1, (C, om.D))
        im = rng.uniform(0.5, 2.0, om.D)
        q, lp, st = m.transition(shard, q0, seed=77, iteration=5, eps=eps, inv_metric=im)
        for c in range(C):
            oq, olp, ost, _ = om.transition(q0[c], seed=77, gid=shard * C + c, iteration=5, eps=eps, inv_metric=im)
            np.testing.assert_allclose(q[c], oq, rtol=1e-9, atol=1e-10)
            assert abs(lp[c] - olp) <= 1e-9 * max(1, abs(olp))
            assert st[c, 2] == ost[2] and st[c, 3] == ost[3] and st[c, 4] == ost[4], (c, st[c], ost)
            np.testing.assert_allclose(st[c, [0, 5]], ost[[0, 5]], rtol=1e-9, atol=1e-12)


def test_transition_matches_oracle_logistic(ctx, orc):
    from stark_amd import engine
    rng = np.random.default_rng(4)
    n, d = 400, 6
    X = rng.uniform(-1.7, 1.7, (n, d))
    y = (rng.uniform(size=n) < 1 / (1 + np.exp(-X @ rng.normal(0, 0.5, d)))).astype(np.int32)
    m = engine.Model(ctx, "logistic", [{"x": X, "y": y}])
    om = orc.Model(orc.FAM_LOGREG, X=X, y=y)
    C = 4
    q0 = rng.normal(0, 0.1, (C, d + 1))
    q, lp, st = m.transition(0, q0, seed=3, iteration=11, eps=0.08)
    for c in range(C):
        oq, olp, ost, _ = om.transition(q0[c], seed=3, gid=c, iteration=11, eps=0.08)
        np.testing.assert_allclose(q[c], oq, rtol=1e-8, atol=1e-10)
        assert st[c, 3] == ost[3]


# ---------------------------------------------------------------- adaptive run vs oracle twin
@pytest.mark.parametrize("nw,jitter", [(30, 0.0), (150, 0.0), (30, 0.5)])
def test_adaptive_run_tracks_oracle(ctx, orc, nw, jitter):
    """Full warmup (init_stepsize probes, dual averaging, Welford windows incl. the 15/75/10
    short-warmup split at nw=30) on the GPU and in the recursive oracle from the same seed:
    on a well-conditioned posterior (stable dynamics, so ulp-level differences between ocml
    and glibc / FMA contraction stay ulp-level) both follow the same path."""
    from stark_amd import engine
    rng = np.random.default_rng(31)
    n, d = 500, 3
    X = rng.uniform(-1.7, 1.7, (n, d))
    y = (rng.uniform(size=n) < 1 / (1 + np.exp(-(0.3 + X @ np.array([0.8, -0.4, 0.2]))))).astype(np.int32)
    m = engine.Model(ctx, "logistic", [{"x": X, "y": y}])
    om = orc.Model(orc.FAM_LOGREG, X=X, y=y)
    ns, C = 20, 2
    res = m.sampler(num_warmup=nw, num_samples=ns, chains=C, seed=2024, save_warmup=True,
                    stepsize_jitter=jitter)
    res.run()
    eps, im = res.adaptation()
    uq = res.unconstrained(0)
    _, st = res.draws(0)
    for c in range(C):
        o = om.run_chain(num_warmup=nw, num_samples=ns, seed=2024, gid=c, stepsize_jitter=jitter)
        err = np.abs(uq[c] - o["q"]).max(axis=1)
        if nw <= 30:     # whole run on the oracle path
            assert err.max() < 1e-8, err.max()
            # per-transition step size (jittered around the nominal one when jitter > 0)
            np.testing.assert_allclose(st[c * ns:(c + 1) * ns, 1], o["stats"][nw:, 1], rtol=1e-8)
            if jitter:
                assert np.ptp(st[c * ns:(c + 1) * ns, 1]) > 0
            np.testing.assert_allclose(eps[c], o["stepsize"], rtol=1e-8)
            np.testing.assert_allclose(im[c, :om.D], o["inv_metric"], rtol=1e-8)
        else:
            # the first 60 transitions (init buffer: init_stepsize, dual averaging) stay on the
            # oracle path; afterwards the reduction-order drift (GPU tile sums vs sequential CPU
            # sums, ~1e-16 per gradient) may grow, but only gradually (no jump from a logic
            # difference): the error never grows by more than 100x between transitions
            assert err[:60].max() < 1e-8, err[:60].max()
            e = np.maximum(err, 1e-13)
            stop = int(np.argmax(e > 1e-6)) if np.any(e > 1e-6) else len(e)
            growth = e[1:stop] / e[:stop - 1]
            assert growth.size == 0 or growth.max() < 100.0, growth.max()
    res.close()


def _packed_schools_run(ctx=None, chains_per_wave=0):
    """10 chains of 8 schools (D = 10): 3 waves of the fused kernel at 4 chains per wave (the
    last one partly empty; chains_per_wave caps the packing), warmup with adaptation + draws;
    returns unconstrained draws and stats."""
    from oracle import oracle as orc
    from stark_amd import engine
    ctx = ctx or engine.Context(0)
    m = engine.Model(ctx, "schools", [{"y": orc.SCHOOLS_Y, "sigma": orc.SCHOOLS_SIGMA}])
    s = m.sampler(num_warmup=30, num_samples=25, chains=10, seed=91, save_warmup=True,
                  chains_per_wave=chains_per_wave)
    s.run()
    uq, st = s.unconstrained(0), s.draws(0)[1]
    s.close()
    m.close()
    return uq, st


def test_packed_schools_chains_bitwise_equal_unpacked(ctx, orc):
    """Packing 4 chains per wave (16 lanes each; segmented DPP sums) changes no bit: the same
    run with one and with two chains per wave (stk_config.chains_per_wave) gives identical draws
    and stats; and every chain starts on the recursive Stan twin's path."""
    uq, st = _packed_schools_run(ctx)
    for cpw in (1, 2):
        u1, s1 = _packed_schools_run(ctx, chains_per_wave=cpw)
        np.testing.assert_array_equal(uq, u1)
        np.testing.assert_array_equal(st, s1)
    om = orc.Model(orc.FAM_SCHOOLS, y=orc.SCHOOLS_Y, sigma=orc.SCHOOLS_SIGMA)
    for c in range(uq.shape[0]):
        o = om.run_chain(num_warmup=30, num_samples=25, seed=91, gid=c)
        err = np.abs(uq[c] - o["q"]).max(axis=1)
        assert err[:10].max() < 1e-8, (c, err[:10])     # ulp-level drift may grow later in the funnel


# ---------------------------------------------------------------- statistics
def test_schools_4096_chains_exact_moments(ctx, orc):
    """BASELINE config 2: 8 schools with 4096 parallel chains on one GPU."""
    from stark_amd import engine
    m = engine.Model(ctx, "schools", [{"y": orc.SCHOOLS_Y, "sigma": orc.SCHOOLS_SIGMA}])
    C = 4096
    s = m.sampler(num_warmup=500, num_samples=200, chains=C, seed=7)
    s.run()
    info = s.info()
    assert info["errors"] == 0 and info["done"] == C
    uq = s.unconstrained(0)          # C x 200 x 10
    em, ev = orc.schools_exact_moments(orc.SCHOOLS_Y, orc.SCHOOLS_SIGMA)
    for k in range(10):
        x = uq[:, :, k]
        e = ess(x)
        mcse = x.std() / np.sqrt(e)
        assert abs(x.mean() - em[k]) < 5 * mcse, (k, x.mean(), em[k], mcse, e)
    np.testing.assert_allclose(uq[:, :, 2:].reshape(-1, 8).var(0), ev[2:], rtol=0.05)
    d, st = s.draws(0)
    assert d.shape == (19, C * 200)
    np.testing.assert_allclose(d[1], np.exp(uq[:, :, 1].reshape(-1)), rtol=1e-15)        # tau
    np.testing.assert_allclose(d[10], d[0] + d[1] * d[2], rtol=1e-12, atol=1e-12)        # theta[1]
    assert 0.7 < st[:, 0].mean() < 0.95
    s.close()


def test_schools_divergence_rate_matches_oracle_twin(ctx, orc):
    """Post-warmup divergences of non-centred 8 schools (Stan defaults: 1000 + 1000, adapt_delta
    0.8) on the GPU against the recursive Stan 2.19.1 twin run on the same seeds and chain ids
    (configs[1] reports 2,688 divergences in 4.1M transitions, 0.07 %).  The two
    machines agree transition for transition until their roundings part the trajectories, so the
    rates are compared statistically: per-chain divergence counts (chains, not transitions, are
    the independent units -- a chain that sits in the funnel diverges repeatedly), difference of
    the two means within 4 standard errors."""
    from stark_amd import engine
    C, W, S, seed = 512, 1000, 1000, 11
    m = engine.Model(ctx, "schools", [{"y": orc.SCHOOLS_Y, "sigma": orc.SCHOOLS_SIGMA}])
    s = m.sampler(num_warmup=W, num_samples=S, chains=C, seed=seed)
    s.run()
    assert s.info()["errors"] == 0
    _, st = s.draws(0)
    gpu = st[:, 4].reshape(C, S).sum(1)
    s.close()
    om = orc.Model(orc.FAM_SCHOOLS, y=orc.SCHOOLS_Y, sigma=orc.SCHOOLS_SIGMA)
    cpu = np.array([om.run_chain(num_warmup=W, num_samples=S, seed=seed, gid=c)["stats"][W:, 4].sum()
                    for c in range(C)])
    se = np.sqrt(gpu.var(ddof=1) / C + cpu.var(ddof=1) / C)
    assert gpu.sum() > 0 and cpu.sum() > 0
    assert abs(gpu.mean() - cpu.mean()) < 4 * se, (gpu.mean() / S, cpu.mean() / S, se / S)


@pytest.mark.parametrize("C", [8, 16, 64])      # 16: the fp64 MFMA sweep (v4); 64: two-pass GEMMs (v5)
def test_linear_regression_closed_form(ctx, orc, C):
    from stark_amd import engine
    rng = np.random.default_rng(8)
    n, d = 2000, 5
    X = rng.uniform(-1.7, 1.7, (n, d))
    y = 0.7 + X @ rng.normal(0, 0.5, d) + 1.3 * rng.normal(size=n)
    m = engine.Model(ctx, "linear", [{"x": X, "y": y}])
    s = m.sampler(num_warmup=500, num_samples=1000, chains=C, seed=21)
    s.run()
    uq = s.unconstrained(0)
    mean, cov = orc.linreg_exact_moments(X, y)
    sd = np.sqrt(np.diag(cov))
    for k in range(d + 1):
        x = uq[:, :, k]
        mcse = x.std() / np.sqrt(ess(x))
        assert abs(x.mean() - mean[k]) < 5 * mcse, (k, x.mean(), mean[k], mcse)
        assert abs(x.std() / sd[k] - 1) < 0.06
    s.close()


@pytest.mark.parametrize("C", [8, 16, 64])
def test_logistic_matches_oracle_moments(ctx, orc, C):
    from stark_amd import engine
    rng = np.random.default_rng(12)
    n, d = 3000, 4
    X = rng.uniform(-1.7, 1.7, (n, d))
    y = (rng.uniform(size=n) < 1 / (1 + np.exp(-(0.2 + X @ rng.normal(0, 0.6, d))))).astype(np.int32)
    m = engine.Model(ctx, "logistic", [{"x": X, "y": y}])
    s = m.sampler(num_warmup=500, num_samples=1000, chains=C, seed=5)
    s.run()
    g = s.unconstrained(0)
    om = orc.Model(orc.FAM_LOGREG, X=X, y=y)
    runs = [om.run_chain(num_warmup=500, num_samples=1000, seed=99, gid=c) for c in range(4)]
    o = np.stack([r["q"][500:] for r in runs])
    for k in range(d + 1):
        a, b = g[:, :, k], o[:, :, k]
        se = np.hypot(a.std() / np.sqrt(ess(a)), b.std() / np.sqrt(ess(b)))
        assert abs(a.mean() - b.mean()) < 5 * se, (k, a.mean(), b.mean(), se)
        assert abs(a.std() / b.std() - 1) < 0.1
    s.close()


# ---------------------------------------------------------------- reproducibility
@pytest.mark.parametrize("C", [2, 16])
def test_bitwise_reproducible_and_resumable(ctx, C):
    from stark_amd import engine
    m = engine.Model.synthetic(ctx, "logistic", 2, 5000, 8, data_seed=3)
    cfg = dict(num_warmup=60, num_samples=40, chains=C, seed=11)
    a = m.sampler(**cfg)
    a.run()
    b = m.sampler(**cfg)
    b.run(30)
    b.run(75)
    b.run()
    for s in range(2):
        np.testing.assert_array_equal(a.draws(s)[0], b.draws(s)[0])
    ia, ib = a.info(), b.info()
    assert ia["grad_evals"] == ib["grad_evals"] and ia["leapfrogs"] == ib["leapfrogs"]
    a.close()
    b.close()


_SAVE_SCRIPT = """
import sys
sys.path.insert(0, {root!r})
import numpy as np
from stark_amd import engine
ctx = engine.Context(0)
fam, C, stop, max_steps, out = {fam!r}, {C}, {stop}, {max_steps}, {out!r}
if fam == "schools":
    from oracle import oracle as O
    m = engine.Model(ctx, "schools", [{{"y": O.SCHOOLS_Y, "sigma": O.SCHOOLS_SIGMA}}])
else:
    m = engine.Model.synthetic(ctx, fam, 2, 5000, 8, data_seed=3)
s = m.sampler(num_warmup=60, num_samples=40, chains=C, seed=11, shard_ids={ids!r})
s.run(stop, max_steps=max_steps)
np.save(out, s.save_state())
print(int(s.iterations().min()), int(s.info()["steps"]))
"""


@pytest.mark.parametrize("fam,C,stop,max_steps", [("logistic", 16, 30, 0), ("logistic", 16, 200, 37),
                                                  ("linear", 64, 75, 0), ("logistic", 2, 61, 0),
                                                  ("schools", 8, 30, 0)])
def test_run_split_across_processes_is_bit_identical(ctx, tmp_path, fam, C, stop, max_steps):
    """Checkpoint / resume: a run saved by one PROCESS (mid-warmup, mid-trajectory after a step
    budget, at the warmup/sampling boundary) and loaded into a fresh sampler of another process
    continues bit for bit as the unsplit run: the same draws, stats, step sizes, metric and
    gradient counts (stk_sampler_save_state / stk_sampler_load_state)."""
    import subprocess
    import sys
    from conftest import ROOT
    from stark_amd import engine
    from oracle import oracle as O
    ids = [5, 2]
    if fam == "schools":
        m = engine.Model(ctx, "schools", [{"y": O.SCHOOLS_Y, "sigma": O.SCHOOLS_SIGMA}])
        ids = [5]
    else:
        m = engine.Model.synthetic(ctx, fam, 2, 5000, 8, data_seed=3)
    cfg = dict(num_warmup=60, num_samples=40, chains=C, seed=11, shard_ids=ids)
    out = str(tmp_path / "state.npy")
    r = subprocess.run([sys.executable, "-c", _SAVE_SCRIPT.format(root=ROOT, fam=fam, C=C, stop=stop,
                                                                   max_steps=max_steps, out=out, ids=ids)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    it_saved, steps_saved = (int(v) for v in r.stdout.split())
    assert 0 <= it_saved < 100
    a = m.sampler(**cfg)
    a.run()
    b = m.sampler(**cfg)
    b.load_state(np.load(out))
    assert int(b.iterations().min()) == it_saved and b.info()["steps"] == steps_saved
    b.run()
    for s in range(m.nshards):
        da, sa = a.draws(s)
        db, sb = b.draws(s)
        np.testing.assert_array_equal(da, db)
        np.testing.assert_array_equal(sa, sb)
    np.testing.assert_array_equal(a.adaptation()[0], b.adaptation()[0])
    np.testing.assert_array_equal(a.adaptation()[1], b.adaptation()[1])
    ia, ib = a.info(), b.info()
    # (not "steps": a run launches steps in batches and may overshoot its last transition by a
    # few idle ones, so an unsplit run counts a different number of launched steps)
    for k in ("grad_evals", "leapfrogs", "divergent", "done", "errors"):
        assert ia[k] == ib[k], k
    # a blob only loads into the run it came from: another seed / chain count is refused
    c = m.sampler(**{**cfg, "seed": 12})
    with pytest.raises(engine.StarkHipError, match="another model geometry or sampler config"):
        c.load_state(np.load(out))
    c.close()
    if C != 64:
        d_ = m.sampler(**{**cfg, "chains": 64 if fam != "schools" else 4})
        with pytest.raises(engine.StarkHipError):
            d_.load_state(np.load(out))
        d_.close()
    for x in (a, b):
        x.close()
    m.close()


@pytest.mark.parametrize("C", [4, 16, 64])
def test_shard_placement_independent(ctx, C):
    """1 GPU holding 4 shards == 4 GPUs holding one shard each (same global shard ids)."""
    from stark_amd import engine
    rows, d = 3000, 10
    cfg = dict(num_warmup=50, num_samples=30, chains=C, seed=5)
    full = engine.Model.synthetic(ctx, "logistic", 4, rows, d, data_seed=8)
    ref = full.sample(**cfg)
    for k in (1, 3):
        one = engine.Model.synthetic(ctx, "logistic", 1, rows, d, data_seed=8, row_offset=k * rows)
        r = one.sample(shard_ids=[k], **cfg)
        np.testing.assert_array_equal(r.draws[0], ref.draws[k])
        one.close()
    full.close()


def test_stark_api_schools_end_to_end(ctx):
    import os
    from conftest import ROOT
    from stark_amd import stark
    from stark_amd.rdd import LocalContext
    sc = LocalContext()
    school = list(zip([28, 8, -3, 7, -1, 1, 18, 12], [15, 10, 16, 11, 9, 11, 10, 18]))

    def prep(data):
        return {"J": len(data), "y": [d[0] for d in data], "sigma": [d[1] for d in data]}

    st = stark.Stark(sc, sc.parallelize(school, 2), prep)
    st.setStanModel(file=os.path.join(ROOT, "stark_amd", "models", "schools.stan"))
    w = st.concensusWeight(iter=1000, seed=3)
    assert w.shape == (11, 500) and np.all(np.isfinite(w))
    nv = st.distribute(n=2, iter=400, seed=4)
    assert nv.shape == (38, 200)


def test_driver_weighted_matches_reference(ctx, golden, monkeypatch):
    """concensusWeight orchestration + GPU combine vs the reference driver on the same fake fits."""
    import test_host
    st = test_host._fake_stark(monkeypatch)
    g = golden("driver_ref.npz")
    out = st.concensusWeight(iter=600)
    ref = g["weighted"]
    np.testing.assert_allclose(out, ref, rtol=1e-9, atol=1e-10 * np.abs(ref).max())
    # with pystan 2's pars= selection the combine runs on the selected rows only (stark/stark.py:48-56)
    out = st.concensusWeight(iter=600, pars=["eta", "mu"])
    ref = g["weighted_pars"]
    assert out.shape == ref.shape == (6, 300)
    np.testing.assert_allclose(out, ref, rtol=1e-9, atol=1e-10 * np.abs(ref).max())


# ---------------------------------------------------------------- full-data mode (configs[4])
@pytest.mark.parametrize("C,d", [(16, 12), (64, 300)])
def test_fulldata_exchange_single_rank(C, d):
    """The full-data path -- context on torch's stream, [grad | lp] block in a torch tensor,
    RCCL all-reduce after every step -- on a one-rank NCCL group reproduces the plain sampler
    bit for bit (the sum over one rank is the identity)."""
    import socket
    import torch
    import torch.distributed as dist
    from stark_amd import engine, fulldata
    s_ = socket.socket()
    s_.bind(("127.0.0.1", 0))
    port = s_.getsockname()[1]
    s_.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        fctx = fulldata.context_on_torch_stream(0)
        cfg = dict(num_warmup=40, num_samples=30, chains=C, seed=9)
        m = engine.Model.synthetic(fctx, "logistic", 1, 3000, d, data_seed=4)
        fs = fulldata.FullDataSampler(m, force_exchange=True, **cfg)
        fs.run()
        got = fs.draws(0)[0]
        fs.close()
        ref = m.sample(shard_ids=[0], **cfg)
        np.testing.assert_array_equal(got, ref.draws[0])
        with pytest.raises(ValueError):
            fulldata.FullDataSampler(engine.Model.synthetic(fctx, "linear", 1, 100, 3), **cfg)
        m.close()
        fctx.close()
    finally:
        dist.destroy_process_group()


def test_logistic_prior_moments_match_oracle(ctx, orc):
    """A prior that matters (n = 60 rows, beta ~ normal(0, 0.4)): GPU chains vs the oracle's
    recursive Stan twin with the same prior, moments within MCSE."""
    from stark_amd import engine
    rng = np.random.default_rng(31)
    n, d = 60, 3
    X = rng.uniform(-1.7, 1.7, (n, d))
    y = (rng.uniform(size=n) < 1 / (1 + np.exp(-(0.3 + X @ np.array([1.0, -0.8, 0.5]))))).astype(np.int32)
    m = engine.Model(ctx, "logistic", [{"x": X, "y": y}]).set_prior(alpha=2.5, beta=0.4)
    s = m.sampler(num_warmup=500, num_samples=1000, chains=16, seed=3)
    s.run()
    g = s.unconstrained(0)
    om = orc.Model(orc.FAM_LOGREG, X=X, y=y, prior_alpha=2.5, prior_beta=0.4)
    runs = [om.run_chain(num_warmup=500, num_samples=1000, seed=77, gid=c) for c in range(4)]
    o = np.stack([r["q"][500:] for r in runs])
    for k in range(d + 1):
        a, b = g[:, :, k], o[:, :, k]
        se = np.hypot(a.std() / np.sqrt(ess(a)), b.std() / np.sqrt(ess(b)))
        assert abs(a.mean() - b.mean()) < 5 * se, (k, a.mean(), b.mean(), se)
        assert abs(a.std() / b.std() - 1) < 0.1
    s.close()
    m.close()


def _fulldata_rank(rank, world, port, q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from stark_amd import engine, fulldata
        torch.cuda.set_device(0)
        n, d = 4001, 10
        off, cnt = fulldata.rank_rows(n, world, rank)
        ctx = fulldata.context_on_torch_stream(0)
        m = engine.Model.synthetic(ctx, "logistic", 1, cnt, d, data_seed=6, row_offset=off)
        fs = fulldata.FullDataSampler(m, num_warmup=40, num_samples=30, chains=16, seed=2)
        fs.run()
        dr = fs.draws(0)[0]
        allr = [None] * world
        dist.all_gather_object(allr, dr)
        q.put((rank, bool(all(np.array_equal(allr[0], a) for a in allr)), bool(np.isfinite(dr).all()),
               fs.info()["grad_evals"]))
        fs.close()
        m.close()
        ctx.close()
    finally:
        dist.destroy_process_group()


def test_fulldata_two_ranks_share_one_gpu():
    """The real N-rank exchange (2 processes, gloo on one GPU): every rank holds half of the rows,
    the [grad | lp] block is summed across processes after every step, and the chains of both
    ranks stay bit-identical for the whole run."""
    import socket
    import torch.multiprocessing as mp
    s_ = socket.socket()
    s_.bind(("127.0.0.1", 0))
    port = s_.getsockname()[1]
    s_.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_fulldata_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(r[1] and r[2] for r in res)
    assert res[0][3] == res[1][3] > 0


# ---------------------------------------------------------------- Stan >= 2.23 U-turn checks (nuts_criterion)
@pytest.mark.parametrize("jitter", [0.0, 0.5])
def test_extended_criterion_tracks_oracle(ctx, orc, jitter):
    """nuts_criterion='stan2.23' (the checks across subtree junctions, at every merge and at
    the top level) against the recursive twin with the same checks: a whole adaptive run."""
    from stark_amd import engine
    rng = np.random.default_rng(31)
    n, d = 500, 3
    X = rng.uniform(-1.7, 1.7, (n, d))
    y = (rng.uniform(size=n) < 1 / (1 + np.exp(-(0.3 + X @ np.array([0.8, -0.4, 0.2]))))).astype(np.int32)
    m = engine.Model(ctx, "logistic", [{"x": X, "y": y}])
    om = orc.Model(orc.FAM_LOGREG, X=X, y=y)
    nw, ns, C = 30, 30, 4
    s = m.sampler(num_warmup=nw, num_samples=ns, chains=C, seed=77, save_warmup=True, stepsize_jitter=jitter,
                  nuts_criterion="stan2.23")
    s.run()
    uq = s.unconstrained(0)
    _, st = s.draws(0)
    for c in range(C):
        o = om.run_chain(num_warmup=nw, num_samples=ns, seed=77, gid=c, stepsize_jitter=jitter, uturn_ext=True)
        err = np.abs(uq[c] - o["q"]).max()
        assert err < 1e-8, (c, err)
        np.testing.assert_array_equal(st[c * ns:(c + 1) * ns, 3], o["stats"][nw:, 3])
    s.close()


def test_extended_criterion_schools_packed(ctx, orc):
    """The same checks in the fused 8-schools kernel (4 chains per wave): every chain starts
    on the recursive twin's path."""
    from stark_amd import engine
    m = engine.Model(ctx, "schools", [{"y": orc.SCHOOLS_Y, "sigma": orc.SCHOOLS_SIGMA}])
    om = orc.Model(orc.FAM_SCHOOLS, y=orc.SCHOOLS_Y, sigma=orc.SCHOOLS_SIGMA)
    s = m.sampler(num_warmup=30, num_samples=20, chains=6, seed=5, save_warmup=True, nuts_criterion="stan2.23")
    s.run()
    uq = s.unconstrained(0)
    for c in range(6):
        o = om.run_chain(num_warmup=30, num_samples=20, seed=5, gid=c, uturn_ext=True)
        err = np.abs(uq[c] - o["q"]).max(axis=1)
        assert err[:10].max() < 1e-8, (c, err[:10])
    s.close()
    m.close()


def test_extended_criterion_stops_resonant_trajectories(ctx):
    """On a near-isotropic Gaussian posterior (logistic regression, 2e4 rows, d = 100, unit
    metric scaled to the posterior sd) at a step size where 8 leapfrogs span half an orbit,
    Stan 2.19's single test lets trajectories run (depth 5-9); the junction checks stop them."""
    from stark_amd import engine
    m = engine.Model.synthetic(ctx, "logistic", 1, 20000, 100, data_seed=5)
    beta = engine.Model.gen_beta(5, 100)
    sd = 1 / np.sqrt(20000 * 0.2)
    init = np.concatenate([[0.0], beta])
    lf = {}
    for crit in ("stan2.19", "stan2.23"):
        s = m.sampler(num_warmup=0, num_samples=40, chains=16, seed=3, stepsize=0.40, skip_init_stepsize=True,
                      adapt_engaged=False, inv_metric=np.full(101, sd * sd), init=np.tile(init, 16),
                      nuts_criterion=crit)
        s.run()
        lf[crit] = s.draws(0)[1][:, 3].mean()
        s.close()
    assert lf["stan2.19"] > 2.5 * lf["stan2.23"], lf
    assert lf["stan2.23"] < 20, lf
    m.close()


@pytest.mark.parametrize("C", [4, 16])
def test_extended_criterion_moments(ctx, orc, C):
    """Statistical check of the extended criterion: logistic moments vs the 2.19 twin."""
    from stark_amd import engine
    rng = np.random.default_rng(12)
    n, d = 3000, 4
    X = rng.uniform(-1.7, 1.7, (n, d))
    y = (rng.uniform(size=n) < 1 / (1 + np.exp(-(0.2 + X @ rng.normal(0, 0.6, d))))).astype(np.int32)
    m = engine.Model(ctx, "logistic", [{"x": X, "y": y}])
    s = m.sampler(num_warmup=500, num_samples=1000, chains=C, seed=8, nuts_criterion="stan2.23")
    s.run()
    g = s.unconstrained(0)
    om = orc.Model(orc.FAM_LOGREG, X=X, y=y)
    runs = [om.run_chain(num_warmup=500, num_samples=1000, seed=99, gid=c) for c in range(4)]
    o = np.stack([r["q"][500:] for r in runs])
    for k in range(d + 1):
        a, b = g[:, :, k], o[:, :, k]
        se = np.hypot(a.std() / np.sqrt(ess(a)), b.std() / np.sqrt(ess(b)))
        assert abs(a.mean() - b.mean()) < 5 * se, (k, a.mean(), b.mean(), se)
        assert abs(a.std() / b.std() - 1) < 0.1
    s.close()
