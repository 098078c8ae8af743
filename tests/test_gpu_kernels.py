"""GPU parity: densities, synthetic generator and combine through libstark_hip.so vs the
CPU oracle and the reference-generated fixtures."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

RTOL_LP = 1e-10   # north_star: log-density and gradient within 1e-10 relative (fp64)


def _rel(a, b):
    return np.abs(a - b) / np.maximum(np.abs(b), 1.0)


# ---------------------------------------------------------------- log density + gradient
def test_schools_lpgrad(ctx, orc):
    from stark_amd import engine
    rng = np.random.default_rng(1)
    shards = [{"y": orc.SCHOOLS_Y[:4], "sigma": orc.SCHOOLS_SIGMA[:4]},
              {"y": orc.SCHOOLS_Y, "sigma": orc.SCHOOLS_SIGMA},
              {"y": rng.normal(0, 10, 70), "sigma": rng.uniform(5, 20, 70)}]   # J=70: two lane chunks
    m = engine.Model(ctx, "schools", shards)
    for s, sh in enumerate(shards):
        om = orc.Model(orc.FAM_SCHOOLS, y=sh["y"], sigma=sh["sigma"])
        q = rng.normal(0, 1, (5, om.D))
        lp, g = m.log_density_grad(s, q)
        for c in range(5):
            olp, og = om.lpgrad(q[c])
            assert _rel(lp[c], olp) < RTOL_LP
            assert np.all(_rel(g[c], og) < RTOL_LP)


# shapes cover every sweep variant: v3 LDS-DMA ring (even d <= 104: partial last tile, one tile,
# many chunks, d = 2), v2 (even d <= 128 beyond v3), v1 (odd or wide d), v4 (C = 16, d <= 128), v5 (C = 64, any d)
@pytest.mark.parametrize("n,d,C", [(1, 1, 5), (7, 3, 5), (1000, 100, 5), (4097, 50, 5), (333, 129, 5),
                                   (257, 300, 5), (100, 700, 5), (5000, 2, 5), (64, 65, 5), (64, 100, 5),
                                   (65, 104, 3), (20000, 100, 4), (3000, 120, 5), (1000, 100, 1), (777, 100, 2),
                                   # v4 fp64 MFMA (16 chains per launch; 20 = two batches, the second padded)
                                   (1, 1, 16), (7, 3, 16), (1000, 100, 16), (4097, 50, 16), (333, 128, 16),
                                   (65, 104, 20), (20000, 100, 16), (64, 65, 16), (5000, 2, 16), (129, 17, 16),
                                   (333, 129, 16), (3, 100, 16), (9, 50, 16), (100003, 100, 16),
                                   # k_sweep16 over the d <= 128 table: odd d, the VALU last tile (d = 99, 113,
                                   # 116), beta in registers with the late slot release (d > 108), and chunks of
                                   # > 64 sub-tiles per wave (the in-loop log1p flush of residual v4: n > 2.1e6)
                                   (500, 99, 16), (300, 113, 16), (300, 116, 16), (200, 127, 16), (64, 110, 16),
                                   (1000, 33, 16), (3000000, 4, 16), (2200000, 17, 16),
                                   # a last MFMA tile of > 4 columns that passes d - 1 (the one clamped
                                   # backward column, d = 94, 29, 30) and the odd-d forward's clamped last steps
                                   (300, 94, 16), (300, 93, 16), (100, 29, 16), (100, 30, 16),
                                   # v5 two-pass fp64 MFMA GEMMs (64 chains; 70 = two batches)
                                   (1, 1, 64), (7, 3, 64), (4097, 50, 64), (333, 129, 64), (257, 300, 64),
                                   (1000, 1000, 64), (130, 1001, 70), (5000, 100, 64),
                                   # pass F's stage count per 128-row tile NKC = ceil(d / 16) at 1 and 2 (the
                                   # parked tile's 8 epilogue parts mostly left for the next tile's end)
                                   (300, 16, 64), (300, 17, 64),
                                   # the largest d the C-ABI takes (1024: 64 pass-F stages per tile, 4 full
                                   # pass-B column blocks) and one past a pass-B column block
                                   (200, 1024, 64), (150, 257, 64),
                                   # pass F chunks of > 32 tiles of 128 rows (512 chunks per shard: n > 2.1e6),
                                   # so its residual-v4 running product is flushed inside the loop too
                                   (2200000, 5, 64)])
@pytest.mark.parametrize("family", ["logistic", "linear"])
def test_regression_lpgrad(ctx, orc, family, n, d, C):
    """lp and gradient of every sweep variant vs the oracle.  Bars: lp within 1e-10 relative;
    each gradient component within 1e-10 of max(|g_j|, 1e-3 max_j |g_j|) -- i.e. 1e-10 relative
    for every component down to a thousandth of the largest, and 1e-13 of the largest below that.
    The floor is there because a component that is a sum of O(n) terms of both signs cancelling
    to near zero carries the rounding of its terms (~n eps |terms|), which no fp64 summation
    order removes; north_star's 1e-10 relative holds for the components that do not cancel."""
    from stark_amd import engine
    rng = np.random.default_rng(n * 1000 + d)
    X = rng.uniform(-1.7, 1.7, (n, d))
    beta = rng.normal(0, 1 / np.sqrt(d), d)
    if family == "logistic":
        eta = X @ beta
        eta[: max(1, n // 50)] *= 80.0     # exercise the +-20 cutoff branches
        y = (rng.uniform(size=n) < 1 / (1 + np.exp(-eta))).astype(np.int32)
        om = orc.Model(orc.FAM_LOGREG, X=X, y=y)
    else:
        y = 0.3 + X @ beta + rng.normal(size=n)
        om = orc.Model(orc.FAM_LINREG, X=X, y=y)
    m = engine.Model(ctx, family, [{"x": X[: max(1, n // 3)], "y": y[: max(1, n // 3)]}, {"x": X, "y": y}])
    q = rng.normal(0, 0.2, (C, om.D))
    if family == "logistic":
        q[0, 1:] = beta * 40     # large |eta| rows
    lp, g = m.log_density_grad(1, q)
    for c in range(C):
        olp, og = om.lpgrad(q[c])
        assert _rel(lp[c], olp) < RTOL_LP, (c, lp[c], olp)
        scale = np.abs(og).max() + 1.0
        assert np.all(np.abs(g[c] - og) <= RTOL_LP * np.maximum(np.abs(og), scale * 1e-3)), (c, np.abs(g[c] - og).max())


@pytest.mark.parametrize("scale", [30.0, 1e3, 1e8, 1e150])
@pytest.mark.parametrize("n,d,C", [(2000, 100, 16), (999, 50, 16), (300, 40, 16), (300, 99, 16), (300, 113, 16),
                                   (500, 100, 64), (400, 60, 4)])
def test_logistic_lpgrad_extreme_eta(ctx, orc, scale, n, d, C):
    """|eta| from ~1 to ~1e151 (NUTS step-size probes from a dispersed init reach such points):
    Stan's +-20 cutoffs -- lt = t, dv = +-1 below, lt ~ -exp(-t) ~ 0 above -- through the
    table-driven residual v4 of k_sweep16 and of the 64-chain pass F (k_gemm_fwd's tile epilogue;
    |t| is clamped at 700 before the exp) and the VALU sweeps, vs the oracle.  The in-loop log1p
    flushes of both v4 users are exercised by test_regression_lpgrad's long-chunk shapes."""
    from stark_amd import engine
    rng = np.random.default_rng(int(scale) % 1000 + n)
    X = rng.uniform(-1.7, 1.7, (n, d))
    y = (rng.uniform(size=n) < 0.5).astype(np.int32)
    om = orc.Model(orc.FAM_LOGREG, X=X, y=y)
    m = engine.Model(ctx, "logistic", [{"x": X, "y": y}])
    q = rng.normal(0, 1.0 / np.sqrt(d), (C, om.D))
    q[: C // 2] *= scale
    lp, g = m.log_density_grad(0, q)
    for c in range(C):
        olp, og = om.lpgrad(q[c])
        assert np.isfinite(lp[c]) and _rel(lp[c], olp) < RTOL_LP, (c, lp[c], olp)
        gs = np.abs(og).max() + 1.0
        assert np.all(np.abs(g[c] - og) <= RTOL_LP * np.maximum(np.abs(og), gs * 1e-3)), (c, np.abs(g[c] - og).max())


# ---------------------------------------------------------------- synthetic generator
@pytest.mark.parametrize("d", [1, 7, 100])
def test_synthetic_generator_matches_oracle(ctx, orc, d):
    from stark_amd import engine
    seed, rows, nsh = 99, 3001, 3
    m = engine.Model.synthetic(ctx, "logistic", nsh, rows, d, data_seed=seed, row_offset=17)
    beta = engine.Model.gen_beta(seed, d)
    np.testing.assert_array_equal(beta, orc.gen_beta(seed, d))
    for s in range(nsh):
        got = m.copy_data(s)
        X = orc.gen_x(seed, 17 + s * rows, rows, d)
        np.testing.assert_array_equal(got["x"], X)     # bit-exact
        y, margin = orc.gen_y_logistic(seed, 17 + s * rows, X, 0.0, beta)
        diff = got["y"] != y
        assert np.all(margin[diff] < 1e-12)             # flips only where u ~ p to the last ulp
    ml = engine.Model.synthetic(ctx, "linear", 1, 500, d, data_seed=seed)
    got = ml.copy_data(0)
    X = orc.gen_x(seed, 0, 500, d)
    np.testing.assert_array_equal(got["x"], X)
    np.testing.assert_allclose(got["y"], orc.gen_y_linear(seed, 0, X, 0.0, beta), rtol=1e-13, atol=1e-13)


# ---------------------------------------------------------------- combine
@pytest.mark.parametrize("P", [11, 53, 102])
def test_combine_matches_reference_fixture(ctx, golden, P):
    from stark_amd import engine
    from stark_amd.stark import consensus_avg
    g = golden("combine_ref.npz")
    f1, f2 = g[f"P{P}_f1"], g[f"P{P}_f2"]
    sw, swt = consensus_avg(2)(f1, f2)
    cond = np.linalg.cond(g[f"P{P}_sumW"])
    tol = 1e-12                         # north_star: 1e-12 flat (measured <= 7.4e-15 at cond <= 47,
                                        # profiles/r02zz10_combine_fixture_errors.json)
    assert np.abs(sw - g[f"P{P}_sumW"]).max() <= tol * np.abs(g[f"P{P}_sumW"]).max()
    assert np.abs(swt - g[f"P{P}_sumWtheta"]).max() <= tol * np.abs(g[f"P{P}_sumWtheta"]).max()
    out, used = engine.consensus([f1, f2], ctx)
    assert used.all()
    ref = g[f"P{P}_final"]
    assert np.abs(out - ref).max() <= tol * np.abs(ref).max(), (np.abs(out - ref).max(), cond)


def test_combine_nan_guard(ctx, golden):
    from stark_amd import engine
    from stark_amd.stark import consensus_avg
    g = golden("combine_ref.npz")
    out = consensus_avg(2)(g["nan_f1"], g["nan_f2"])
    np.testing.assert_array_equal(out, g["nan_f2"])        # reference: NaN in f1 returns f2
    comb, used = engine.consensus([g["nan_f1"], g["nan_f2"]], ctx)
    assert list(used) == [False, True]
    np.testing.assert_allclose(comb, g["nan_f2"], rtol=1e-9, atol=1e-9)   # only shard 2 left


def test_combine_public_solve_is_a_general_inverse(ctx):
    """stk_consensus_solve takes the caller's sum W: any invertible matrix, inverted as
    np.linalg.inv does (partial pivoting; stark/stark.py:67-70) -- also a non-symmetric one and a
    symmetric indefinite one; an exactly singular one raises LinAlgError as numpy does."""
    from stark_amd import engine
    from stark_amd._lib import LinAlgError
    rng = np.random.default_rng(5)
    for P in (11, 102, 140):
        swt = rng.normal(size=(P, 64))
        ns = rng.normal(size=(P, P)) + 3 * np.eye(P)                    # not symmetric
        ind = rng.normal(size=(P, P))
        ind = ind + ind.T                                              # symmetric indefinite
        for M in (ns, ind):
            ref = np.linalg.inv(M) @ swt
            out = engine.consensus_solve(M, swt, ctx)
            np.testing.assert_allclose(out, ref, rtol=1e-9, atol=1e-11 * np.abs(ref).max() * np.linalg.cond(M))
    sing = np.ones((5, 5))
    with pytest.raises(np.linalg.LinAlgError):
        np.linalg.inv(sing)
    with pytest.raises(LinAlgError):
        engine.consensus_solve(sing, rng.normal(size=(5, 8)), ctx)


@pytest.mark.parametrize("P", [11, 30])
def test_combine_rank_deficient_covariance(ctx, golden, P):
    """S - 1 < P draws: each sample covariance is singular.  The reference's np.linalg.inv does
    not raise on it (LAPACK LU meets no exactly zero pivot) and returns an 'inverse' made of
    rounding noise (tests/golden/make_golden.py records it); the GPU combine reports it as
    LinAlgError, decided by the rank bound S - 1 < p before any arithmetic (not by the sign of a
    rounded pivot) -- the documented deviation (include/stark_hip.h).  Also
    through the blocked call (p = the larger weight block) and the pairwise reducer."""
    from stark_amd import engine
    from stark_amd._lib import LinAlgError
    g = golden("combine_ref.npz")
    f1, f2 = g[f"rankdef_P{P}_f1"], g[f"rankdef_P{P}_f2"]
    assert f1.shape[1] - 1 < P and int(g[f"rankdef_P{P}_raised"]) == 0
    with pytest.raises(LinAlgError):
        engine.consensus([f1, f2], ctx)
    with pytest.raises(LinAlgError):
        engine.consensus([f1, f2], ctx, separate_lp=True)
    with pytest.raises(LinAlgError):
        engine.consensus_products([f1, f2], ctx)
    # one draw more than the largest block: full rank, combined
    rng = np.random.default_rng(P)
    ok = [rng.normal(size=(P, P + 1)) for _ in range(2)]
    out, used = engine.consensus(ok, ctx)
    assert used.all() and np.isfinite(out).all()
    blk, _ = engine.consensus([x[:, :P] for x in ok], ctx, separate_lp=True)   # blocks P - 1 and 1, S = P
    assert np.isfinite(blk).all()


def test_combine_correlated_full_rank_covariance(ctx, orc):
    """A full-rank covariance with a near-collinear parameter pair (1 - R^2 ~ 1e-12, condition
    number ~1e12) is inverted, not reported singular: numpy's inv (the reference's combine) returns
    a usable inverse there, so the GPU combine must too (the singular-pivot threshold
    is P eps on the unit-diagonal matrix, the rounding level of the elimination)."""
    from stark_amd import engine
    rng = np.random.default_rng(21)
    P, S = 6, 4000
    draws = []
    for s in range(3):
        x = rng.normal(size=(P, S))
        x[1] = x[0] + 1e-6 * rng.normal(size=S)       # corr(x0, x1) = 1 - 5e-13
        draws.append(x + rng.normal(size=(P, 1)))
    c = np.cov(draws[0])
    assert np.linalg.cond(c) > 1e11
    ref = orc.consensus_combine_ref(draws)
    out, used = engine.consensus(draws, ctx)
    assert used.all() and np.isfinite(out).all()
    # the weighted average of near-collinear rows is conditioned like W itself: agree to cond * eps
    np.testing.assert_allclose(out, ref, rtol=0, atol=1e-3 * np.abs(ref).max())


@pytest.mark.parametrize("P,i,j", [(6, 0, 1), (40, 3, 20), (102, 17, 101)])
def test_combine_duplicated_parameter_row_is_singular(ctx, P, i, j):
    """An exactly duplicated parameter row with S >> P draws: the sample covariance is
    singular although S > P, so the rank bound does not catch it; the unit-diagonal matrix then
    has a 2 x 2 block [[1, r], [r, 1]] with r within 2 ulp of 1, and the elimination's pivot for
    the second row, 1 - r^2, lies within 4.4e-16 of zero, below the P eps threshold: LinAlgError
    (include/stark_hip.h).  numpy's LU on the same matrix (the reference's np.linalg.inv) meets
    either an exactly zero pivot (LinAlgError) or a rounded one and returns an 'inverse' of
    ~1e34 entries -- which of the two depends on the rounding, so no fixture pins it."""
    from stark_amd import engine
    from stark_amd._lib import LinAlgError
    rng = np.random.default_rng(P)
    draws = []
    for s in range(3):
        x = rng.normal(size=(P, 4000))
        x[j] = x[i]
        draws.append(x + rng.normal(size=(P, 1)))
    with pytest.raises(LinAlgError):
        engine.consensus(draws, ctx)
    with pytest.raises(LinAlgError):
        engine.consensus_products(draws, ctx)


def test_combine_device_mismatch_is_refused(ctx):
    """Device draws on another device than the context's are refused in Python, before the
    library would dereference them without peer access; the C-ABI itself stages such
    pointers through hipMemcpyAsync(Default) (capi.hip is_device_ptr checks the device)."""
    import torch
    from stark_amd import engine

    class OtherDevice:              # a context on another device: the check fires before any call
        device = ctx.device + 1
        _h = None
    dev_in = torch.zeros((2, 3, 10), dtype=torch.float64, device=f"cuda:{ctx.device}")
    with pytest.raises(ValueError, match="context"):
        engine.consensus(dev_in, OtherDevice())


def test_combine_device_draws_match_host(ctx):
    """Device-resident draws (a [shards, P, S] cuda tensor, as dist.all_gather_partitions(...,
    as_tensor=True) returns them) combine where they lie, bit-identical to the host-buffer path."""
    import torch
    from stark_amd import engine
    rng = np.random.default_rng(9)
    P, S, ns = 40, 500, 8
    draws = []
    for _ in range(ns):
        A = rng.normal(size=(P, P)) / np.sqrt(P)
        draws.append(rng.normal(size=(P, 1)) + np.linalg.cholesky(A @ A.T + 0.5 * np.eye(P)) @ rng.normal(size=(P, S)))
    host, used_h = engine.consensus(draws, ctx, separate_lp=True)
    dev_in = torch.as_tensor(np.stack(draws), device=f"cuda:{ctx.device}")
    out, used = engine.consensus(dev_in, ctx, separate_lp=True)
    assert out.is_cuda and tuple(out.shape) == (P, S)
    np.testing.assert_array_equal(out.cpu().numpy(), host)
    assert list(used) == list(used_h)
    out2, _ = engine.consensus([t for t in dev_in], ctx)
    np.testing.assert_array_equal(out2.cpu().numpy(), engine.consensus(draws, ctx)[0])


@pytest.mark.parametrize("S", [1, 3, 8])
def test_combine_general_shards(ctx, orc, S):
    from stark_amd import engine
    from stark_amd.stark import consensus_avg
    import functools
    rng = np.random.default_rng(S)
    P, n = 13, 400
    draws = []
    for s in range(S):
        A = rng.normal(size=(P, P)) / np.sqrt(P)
        L = np.linalg.cholesky(A @ A.T + 0.5 * np.eye(P))
        draws.append(rng.normal(size=(P, 1)) + L @ rng.normal(size=(P, n)))
    ref = orc.consensus_combine_ref(draws)
    out, used = engine.consensus(draws, ctx)
    assert used.all()
    np.testing.assert_allclose(out, ref, rtol=1e-10, atol=1e-11 * np.abs(ref).max())
    if S > 1:   # reducer chaining (functools.reduce over partitions, the reference's rdd.reduce)
        red = functools.reduce(consensus_avg(S), draws)
        np.testing.assert_allclose(engine.consensus_solve(red[0], red[1], ctx), ref, rtol=1e-10,
                                   atol=1e-11 * np.abs(ref).max())


@pytest.mark.parametrize("P,S", [(2, 50), (16, 80), (17, 90), (40, 300), (113, 640), (128, 700), (150, 900)])
def test_combine_sizes_and_blocked_weights(ctx, orc, P, S):
    """Every inverse path (register block Gauss-Jordan on 16 x 16 tiles up to P = 128 -- one
    to eight tiles, full and ragged last tiles -- and the global-memory pivoted GJ above)
    vs the numpy restatement, and the blocked call (stk_consensus_blocked) equal to combining
    the two row blocks separately."""
    from stark_amd import engine
    rng = np.random.default_rng(P)
    draws = []
    for s in range(5):
        A = rng.normal(size=(P, P)) / np.sqrt(P)
        L = np.linalg.cholesky(A @ A.T + 0.3 * np.eye(P))
        draws.append(rng.normal(size=(P, 1)) * 3 + L @ rng.normal(size=(P, S)))
    ref = orc.consensus_combine_ref(draws)
    out, used = engine.consensus(draws, ctx)
    assert used.all()
    scale = np.abs(ref).max()
    assert np.abs(out - ref).max() <= 1e-11 * scale, np.abs(out - ref).max() / scale
    blk, _ = engine.consensus(draws, ctx, separate_lp=True)
    two = np.vstack([orc.consensus_combine_ref([d[:-1] for d in draws]) if P > 1 else np.empty((0, S)),
                     orc.consensus_combine_ref([d[-1:] for d in draws])])
    assert np.abs(blk - two).max() <= 1e-11 * scale, np.abs(blk - two).max() / scale


def test_combine_singular_raises(ctx):
    """A singular sample covariance (a constant row) raises LinAlgError, as np.linalg.inv does."""
    from stark_amd import engine
    from stark_amd._lib import LinAlgError
    rng = np.random.default_rng(2)
    d = [rng.normal(size=(4, 100)) for _ in range(2)]
    d[1][2] = 1.5
    with pytest.raises(LinAlgError):
        engine.consensus(d, ctx)


def test_combine_separate_lp(ctx, orc):
    """engine.consensus(separate_lp=True): parameter rows and the lp__ row are combined as two
    weight blocks (each = the oracle combine of that block alone); with shard lp__ offsets of
    300 lp-sds, the joint combine (the reference's, stark/stark.py:49-56) moves the parameter
    means by several posterior sds, the block combine does not.  Gaussian shards, so the exact
    full-data mean is the average of the shard means."""
    from stark_amd import engine
    rng = np.random.default_rng(11)
    P, n, S = 21, 1000, 8
    A = rng.normal(size=(P, P)) / np.sqrt(P)
    L = np.linalg.cholesky(8 * (A @ A.T + 0.5 * np.eye(P)))
    mus = [L @ rng.normal(size=P) for _ in range(S)]
    draws = []
    for s in range(S):
        w = rng.normal(size=(P, n))
        lp = -0.5 * (w ** 2).sum(0) + 300 * np.sqrt(P / 2) * rng.normal()
        draws.append(np.vstack([mus[s][:, None] + L @ w, lp]))
    out, used = engine.consensus(draws, ctx, separate_lp=True)
    assert used.all() and out.shape == (P + 1, n)
    ref_t = orc.consensus_combine_ref([d[:-1] for d in draws])
    wl = [1.0 / np.var(d[-1], ddof=1) for d in draws]     # 1 x 1 blocks: inverse variances
    ref_l = (sum(w * d[-1:] for w, d in zip(wl, draws)) / sum(wl))
    np.testing.assert_allclose(out[:-1], ref_t, rtol=1e-10, atol=1e-11 * np.abs(ref_t).max())
    np.testing.assert_allclose(out[-1:], ref_l, rtol=1e-10, atol=1e-11 * np.abs(ref_l).max())
    joint, _ = engine.consensus(draws, ctx)
    full = np.mean(mus, axis=0)
    z2 = lambda c: float((((c.mean(1) - full) / c.std(1)) ** 2).mean())
    assert z2(out[:-1]) < 0.2          # weight noise alone: ~P / n per shard (measured 0.009)
    assert z2(joint[:-1]) > 5.0        # lp__ offsets leak through the cross-covariances (measured 38.6)


def test_combine_singular_constant_shards(ctx):
    from stark_amd import engine
    from stark_amd._lib import LinAlgError
    x = np.ones((3, 50))
    with pytest.raises(LinAlgError):
        engine.consensus([x, x + 1], ctx)


# ---------------------------------------------------------------- normal(0, s) priors
@pytest.mark.parametrize("C", [4, 16, 64])
@pytest.mark.parametrize("family", ["logistic", "linear"])
def test_prior_lpgrad(ctx, orc, family, C):
    """alpha ~ normal(0, 2.5), beta ~ normal(0, 0.3) added once per chain in the chunk reduction."""
    from stark_amd import engine
    rng = np.random.default_rng(C)
    n, d = 700, 20
    X = rng.uniform(-1.7, 1.7, (n, d))
    beta = rng.normal(0, 1 / np.sqrt(d), d)
    if family == "logistic":
        y = (rng.uniform(size=n) < 1 / (1 + np.exp(-(X @ beta)))).astype(np.int32)
        om = orc.Model(orc.FAM_LOGREG, X=X, y=y, prior_alpha=2.5, prior_beta=0.3)
    else:
        y = 0.3 + X @ beta + rng.normal(size=n)
        om = orc.Model(orc.FAM_LINREG, X=X, y=y, prior_alpha=2.5, prior_beta=0.3)
    m = engine.Model(ctx, family, [{"x": X, "y": y}]).set_prior(alpha=2.5, beta=0.3)
    q = rng.normal(0, 0.5, (C, om.D))
    lp, g = m.log_density_grad(0, q)
    for c in range(C):
        olp, og = om.lpgrad(q[c])
        assert _rel(lp[c], olp) < RTOL_LP
        assert np.all(np.abs(g[c] - og) <= RTOL_LP * np.maximum(np.abs(og), np.abs(og).max() * 1e-3 + 1.0))
    m.set_prior()                      # back to flat: bit-for-bit the flat model
    lp0, g0 = m.log_density_grad(0, q)
    flat = engine.Model(ctx, family, [{"x": X, "y": y}])
    lp1, g1 = flat.log_density_grad(0, q)
    np.testing.assert_array_equal(lp0, lp1)
    np.testing.assert_array_equal(g0, g1)
    m.close()
    flat.close()


# ---------------------------------------------------------------- the headline shapes at full size
def test_fullsize_shards_sum_to_full_data(ctx):
    """BASELINE configs[3] at full size (N = 1e8, d = 100, 16 chains: the k_sweepe launch of the
    bench): the log density of a flat-prior logistic regression is a sum over rows, so the 8
    subposterior shards' lp and gradient must add up to those of ONE shard holding all 1e8 rows
    (the same Philox rows, generated by global row index).  The two sums run over different chunk
    structures, so they agree to rounding: 1e-12 relative on lp, the sweep tolerance on the
    gradient.  Size-independent property; the oracle covers the arithmetic at small n."""
    from stark_amd import engine
    n, S, d, C, seed = 100_000_000, 8, 100, 16, 20240
    truth = np.concatenate([[0.0], engine.Model.gen_beta(seed, d)])
    q = truth + np.random.default_rng(3).normal(0, 2e-3, (C, d + 1))
    m8 = engine.Model.synthetic(ctx, "logistic", S, n // S, d, data_seed=seed)
    lp8, g8 = np.zeros(C), np.zeros((C, d + 1))
    for s in range(S):
        lp, g = m8.log_density_grad(s, q)
        lp8 += lp
        g8 += g
    m8.close()
    m1 = engine.Model.synthetic(ctx, "logistic", 1, n, d, data_seed=seed)
    lp1, g1 = m1.log_density_grad(0, q)
    m1.close()
    assert np.all(np.abs(lp8 - lp1) <= 1e-12 * np.abs(lp1)), np.abs(lp8 - lp1) / np.abs(lp1)
    for c in range(C):
        scale = np.abs(g1[c]).max() + 1.0
        assert np.all(np.abs(g8[c] - g1[c]) <= RTOL_LP * np.maximum(np.abs(g1[c]), scale * 1e-3)), \
            (c, np.abs(g8[c] - g1[c]).max(), scale)


def test_c_abi_rejects_bad_bernoulli_y(ctx):
    """stk_model_create (the boundary a reference-side binding calls directly, without the
    Python wrapper's check) rejects a logistic y outside {0, 1}: the sweeps read y as a sign bit."""
    import ctypes
    from stark_amd import _lib, engine
    x = np.zeros((5, 3))
    y = np.array([0, 1, 2, 1, 0], np.int32)
    arr = (engine.Shard * 1)()
    arr[0] = engine.Shard(5, 3, x.ctypes.data, None, y.ctypes.data, None)
    h = ctypes.c_void_p()
    rc = _lib.load().stk_model_create(ctx._h, engine.STK_LOGREG, arr, 1, ctypes.byref(h))
    assert rc != 0 and "y_int[2] = 2" in _lib.load().stk_last_error().decode()
    y[2] = 1
    assert _lib.load().stk_model_create(ctx._h, engine.STK_LOGREG, arr, 1, ctypes.byref(h)) == 0
    _lib.load().stk_model_destroy(h)
