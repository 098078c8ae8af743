"""Pin the CPU oracle before trusting it (CPU only).

* Philox4x32-10 against Random123's published known-answer vectors.
* The numpy combine restatement against fixtures produced by the REFERENCE's own
  consensus_avg / driver solve (tests/golden/make_golden.py imports stark/stark.py).
* Densities against central finite differences; the NUTS twin against exact posterior
  moments (8 schools by quadrature, flat-prior linear regression in closed form).
"""
import numpy as np
import pytest

from stark_amd.stark import _extract_to_matrix


KAT = [  # Random123 kat_vectors, philox4x32_10
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


@pytest.mark.parametrize("ctr,key,want", KAT)
def test_philox_kat(orc, ctr, key, want):
    assert tuple(orc.philox(ctr, key)) == want


@pytest.mark.parametrize("P", [11, 53, 102])
def test_combine_restatement_matches_reference(golden, orc, P):
    g = golden("combine_ref.npz")
    f1, f2 = g[f"P{P}_f1"], g[f"P{P}_f2"]
    red = orc.consensus_avg_ref(f1, f2)
    np.testing.assert_allclose(red[0], g[f"P{P}_sumW"], rtol=1e-12, atol=0)
    np.testing.assert_allclose(red[1], g[f"P{P}_sumWtheta"], rtol=1e-10, atol=1e-12 * np.abs(red[1]).max())
    final = orc.consensus_combine_ref([f1, f2])
    np.testing.assert_allclose(final, g[f"P{P}_final"], rtol=1e-9, atol=1e-12 * np.abs(final).max())


def test_combine_lp_row_leak(orc):
    """The reference's joint combine (lp__ inside inv(cov), stark/stark.py:49-56) on Gaussian
    shards whose lp__ rows sit 300 lp-sds apart: the parameter means move by several posterior
    sds; combining the parameter rows alone (the separate_lp block) does not."""
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
    full = np.mean(mus, axis=0)
    z2 = lambda c: float((((c.mean(1) - full) / c.std(1)) ** 2).mean())
    assert z2(orc.consensus_combine_ref(draws)[:-1]) > 5.0
    assert z2(orc.consensus_combine_ref([d[:-1] for d in draws])) < 0.2


def test_combine_nan_guard_reference(golden, orc):
    g = golden("combine_ref.npz")
    out = orc.consensus_avg_ref(g["nan_f1"], g["nan_f2"])
    np.testing.assert_array_equal(out, g["nan_out"])
    np.testing.assert_array_equal(out, g["nan_f2"])


def test_concat_reference(golden):
    from stark_amd.stark import concatenate_samples
    g = golden("concat_ref.npz")
    np.testing.assert_array_equal(concatenate_samples(g["a"], g["b"]), g["out"])


def test_extract_to_matrix_reference(golden):
    """stark/stark.py:49-56 contract (key order, (S,1) reshape, transpose) vs the reference's
    own closure output on the same fake fit."""
    import collections
    g = golden("driver_ref.npz")
    # rebuild partition 0's fake fit at iter=600 from the fixture and compare layouts
    od = collections.OrderedDict((k, g[f"w600_part0_{k}"]) for k in ("mu", "tau", "eta", "theta", "lp__"))
    m = _extract_to_matrix(od)
    assert m.shape == (11, 300)
    np.testing.assert_array_equal(m[0], od["mu"])
    np.testing.assert_array_equal(m[2:6], od["eta"].T)
    np.testing.assert_array_equal(m[-1], od["lp__"])
    assert g["part0"].shape == (11, 1000)


@pytest.mark.parametrize("family", ["schools", "logistic", "linear"])
def test_oracle_density_fd(orc, family):
    rng = np.random.default_rng(3)
    if family == "schools":
        m = orc.Model(orc.FAM_SCHOOLS, y=orc.SCHOOLS_Y, sigma=orc.SCHOOLS_SIGMA)
    else:
        X = rng.uniform(-1.7, 1.7, (300, 5))
        beta = rng.normal(0, 0.5, 5)
        if family == "logistic":
            y = (rng.uniform(size=300) < 1 / (1 + np.exp(-X @ beta))).astype(np.int32)
            m = orc.Model(orc.FAM_LOGREG, X=X, y=y)
        else:
            y = X @ beta + rng.normal(size=300)
            m = orc.Model(orc.FAM_LINREG, X=X, y=y)
    q = rng.normal(0, 0.3, m.D)
    lp, g = m.lpgrad(q)
    h = 1e-6
    fd = np.array([(m.lpgrad(q + h * e)[0] - m.lpgrad(q - h * e)[0]) / (2 * h) for e in np.eye(m.D)])
    np.testing.assert_allclose(g, fd, rtol=1e-6, atol=1e-6 * max(1.0, np.abs(g).max()))


def test_oracle_generator_shapes(orc):
    X = orc.gen_x(7, 0, 50, 9)
    assert X.shape == (50, 9) and np.all(np.abs(X) < np.sqrt(3))
    assert abs(X.var() - 1.0) < 0.2
    b = orc.gen_beta(7, 9)
    y, margin = orc.gen_y_logistic(7, 0, X, 0.0, b)
    assert set(np.unique(y)) <= {0, 1} and np.all(margin >= 0)
    # sharding invariance: rows carry their global index
    np.testing.assert_array_equal(orc.gen_x(7, 20, 10, 9), X[20:30])


def test_oracle_nuts_schools_exact_moments(orc):
    m = orc.Model(orc.FAM_SCHOOLS, y=orc.SCHOOLS_Y, sigma=orc.SCHOOLS_SIGMA)
    em, ev = orc.schools_exact_moments(orc.SCHOOLS_Y, orc.SCHOOLS_SIGMA)
    runs = [m.run_chain(num_warmup=1000, num_samples=5000, seed=11, gid=c) for c in range(8)]
    Q = np.concatenate([r["q"][1000:] for r in runs])
    from stark_amd.diagnostics import ess
    for k in range(m.D):
        x = np.stack([r["q"][1000:, k] for r in runs])
        mcse = x.std() / np.sqrt(ess(x))
        assert abs(Q[:, k].mean() - em[k]) < 5 * mcse + 1e-3, (k, Q[:, k].mean(), em[k], mcse)
    # variances of eta within 10%
    np.testing.assert_allclose(Q[:, 2:].var(0), ev[2:], rtol=0.1)


def test_oracle_nuts_linreg_closed_form(orc):
    rng = np.random.default_rng(5)
    X = rng.uniform(-1.7, 1.7, (200, 3))
    y = 0.5 + X @ np.array([1.0, -0.5, 0.25]) + rng.normal(size=200)
    m = orc.Model(orc.FAM_LINREG, X=X, y=y)
    mean, cov = orc.linreg_exact_moments(X, y)
    runs = [m.run_chain(num_warmup=500, num_samples=2000, seed=3, gid=c) for c in range(4)]
    Q = np.concatenate([r["q"][500:, :4] for r in runs])
    sd = np.sqrt(np.diag(cov))
    assert np.all(np.abs(Q.mean(0) - mean) < 0.1 * sd + 4 * sd / np.sqrt(len(Q) / 3))
    np.testing.assert_allclose(Q.std(0), sd, rtol=0.08)


def test_oracle_transition_deterministic(orc):
    m = orc.Model(orc.FAM_SCHOOLS, y=orc.SCHOOLS_Y, sigma=orc.SCHOOLS_SIGMA)
    q0 = np.linspace(-0.5, 0.5, m.D)
    a = m.transition(q0, seed=5, gid=3, iteration=7, eps=0.3)
    b = m.transition(q0, seed=5, gid=3, iteration=7, eps=0.3)
    np.testing.assert_array_equal(a[0], b[0])
    assert a[2][3] == 2 ** a[2][2] - 1 or a[2][4] == 1 or a[2][2] >= 0


def test_residual_v3_emulation_accuracy():
    """The design of k_sweepe's logistic residual v3 (tables, polynomial degrees, Stan's +-20
    cutoffs by clamping, one Newton step on a 2^-24 reciprocal seed), emulated in numpy by
    tools/residual_v3_accuracy.py, against Stan's bernoulli_logit term in long double: lt within
    4e-15 absolute and dv within 1e-15 relative away from the cutoff bands, exactly Stan's (t, 1)
    below -20, NaN kept.  (The GPU kernel is checked against the oracle in test_gpu_kernels.py.)"""
    import numpy as np
    from tools import residual_v3_accuracy as R
    t = np.concatenate([np.random.default_rng(3).uniform(-25, 25, 100_000), np.linspace(-21, -19, 2001)])
    lt, dv = R.resid3(t)
    lr, dr = R.stan(t)
    inner = np.abs(t) < 20
    assert np.abs(lt - lr.astype(np.float64))[inner].max() < 4e-15
    assert (np.abs(dv - dr.astype(np.float64)) / dr.astype(np.float64))[inner].max() < 1e-15
    low = t < -20
    assert np.array_equal(lt[low], t[low]) and np.all(dv[low] == 1.0)
    assert np.isnan(R.resid3(np.array([np.nan]))[0][0])


def test_residual_v4_emulation_accuracy():
    """The design of k_sweep16's logistic residual v4 (sweep16.hip: logit_resid4 -- 1024-entry exp
    table, fitted degree-3 polynomial, ln2/1024 rounded once, Stan's lower cutoff by a -1100 ldexp
    exponent, and the log terms summed as log1p of a per-lane running product flushed every 256
    elements), emulated in numpy by tools/residual_v3_accuracy.py, against Stan's bernoulli_logit
    term in long double: the lp sum of 2e5 uniform t in [-25, 25] and of a stretch where every e is
    below eps (t > 37: the product must still add them) within 1e-14 relative, dv within 4e-15
    relative away from the cutoff bands, exactly 1 below -20, a NaN kept in the sum."""
    import numpy as np
    from tools import residual_v3_accuracy as R
    rng = np.random.default_rng(4)
    for t in (rng.uniform(-25, 25, 200_000), rng.uniform(37, 45, 50_000), rng.uniform(-0.5, 3, 70_001)):
        lp, dv = R.resid4(t)
        lr, dr = R.stan(t)
        ref = float(lr.sum())
        assert abs(lp - ref) <= 1e-14 * abs(ref), (lp, ref)
        inner = np.abs(t) < 20
        if inner.any():
            assert (np.abs(dv - dr.astype(np.float64)) / dr.astype(np.float64))[inner].max() < 4e-15
    t = np.linspace(-30, -20.000001, 999)
    lp, dv = R.resid4(t)
    assert np.all(dv == 1.0) and abs(lp - float(t.sum())) <= 1e-15 * abs(float(t.sum()))   # lt = t exactly
    assert np.isnan(R.resid4(np.array([0.5, np.nan, -3.0]))[0])


def test_nuts_table_math_emulation_accuracy():
    """The fused NUTS kernel's table-driven exp / log1p (nuts.hip exp_mt, log1p01_mt), emulated in
    numpy by tools/nuts_math_accuracy.py: within 3 ulp of long-double references over the ranges
    the state machine feeds them, with exp's special values (0, inf, NaN) kept."""
    import numpy as np
    from tools import nuts_math_accuracy as M
    rng = np.random.default_rng(5)
    x = np.concatenate([rng.uniform(-40, 0, 100_000), rng.uniform(-700, 700, 100_000)])
    assert M.ulps(M.exp_mt(x), np.exp(x.astype(np.longdouble))).max() < 3
    e = np.concatenate([rng.uniform(0, 1, 100_000), 10.0 ** rng.uniform(-300, 0, 50_000), [0.0, 1.0]])
    assert M.ulps(M.log1p01_mt(e), np.log1p(e.astype(np.longdouble))).max() < 3
    sp = M.exp_mt(np.array([-np.inf, np.inf, np.nan, -1000.0, 1000.0]))
    assert sp[0] == 0 and sp[1] == np.inf and np.isnan(sp[2]) and sp[3] == 0 and sp[4] == np.inf
