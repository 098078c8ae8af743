"""CPU oracle for the stark hot path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module, and only as the checker / CPU baseline.  The product path
(``stark_amd`` + ``libstark_hip.so``) never imports it and fails loudly without its HIP
library instead of falling back here.

Contents
  * ctypes bindings to ``oracle/_build/liboracle.so`` (``stark_oracle.c``): Philox, the
    synthetic generator, the three log densities + gradients, the Stan 2.19 NUTS twin.
  * ``consensus_avg_ref`` / ``consensus_combine_ref``: numpy restatement of the
    reference's combine (``stark/stark.py:7-21`` pairwise reducer and the driver solve
    ``stark/stark.py:66-70``), pinned against golden fixtures produced by importing the
    reference itself (``tests/golden/make_golden.py``).
  * exact posterior moments used to pin the sampler:
    8-schools by quadrature over (mu, tau) with eta/theta marginalised analytically, and
    flat-prior linear regression in closed form.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")

FAM_SCHOOLS, FAM_LINREG, FAM_LOGREG = 1, 2, 3
TAG_INIT, TAG_MOM, TAG_UNI, TAG_SSMOM, TAG_JIT, TAG_X, TAG_Y, TAG_BETA = 0x1, 0x2, 0x3, 0x4, 0x5, 0x10, 0x11, 0x12


def build() -> str:
    """Compile the C restatement (gcc; no GPU needed)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        dp = ctypes.POINTER(ctypes.c_double)
        i32p = ctypes.POINTER(ctypes.c_int32)
        u64, i64, u32, ci = ctypes.c_uint64, ctypes.c_int64, ctypes.c_uint32, ctypes.c_int
        L.orc_philox4x32_10.argtypes = [ctypes.POINTER(u32), ctypes.POINTER(u32), ctypes.POINTER(u32)]
        L.orc_uniform.argtypes = [u64, u32, u32, u32, u32]
        L.orc_uniform.restype = ctypes.c_double
        L.orc_normal.argtypes = [u64, u32, u32, u32, u32, u32]
        L.orc_normal.restype = ctypes.c_double
        L.orc_gen_x.argtypes = [u64, i64, i64, ci, dp]
        L.orc_gen_beta.argtypes = [u64, ci, dp]
        L.orc_gen_y_logistic.argtypes = [u64, i64, i64, ci, dp, ctypes.c_double, dp, i32p, dp]
        L.orc_gen_y_linear.argtypes = [u64, i64, i64, ci, dp, ctypes.c_double, dp, ctypes.c_double, dp]
        L.orc_schools_lpgrad.argtypes = [ci, dp, dp, dp, dp]
        L.orc_schools_lpgrad.restype = ctypes.c_double
        L.orc_logreg_lpgrad.argtypes = [i64, ci, dp, i32p, dp, dp]
        L.orc_logreg_lpgrad.restype = ctypes.c_double
        L.orc_linreg_lpgrad.argtypes = [i64, ci, dp, dp, dp, dp]
        L.orc_linreg_lpgrad.restype = ctypes.c_double
        L.orc_prior_lpgrad.argtypes = [ctypes.c_double, ctypes.c_double, ci, dp, dp]
        L.orc_prior_lpgrad.restype = ctypes.c_double
        L.orc_run_chain.argtypes = [ctypes.c_void_p, ctypes.c_void_p, u32, dp, dp, dp, dp, dp]
        L.orc_run_chain.restype = ctypes.c_long
        L.orc_transition.argtypes = [ctypes.c_void_p, u64, u32, u32, ci, ctypes.c_double, dp, dp, dp, dp, ci]
        L.orc_transition.restype = ctypes.c_long
        L.orc_logreg_grad_loop.argtypes = [i64, ci, dp, i32p, dp, dp, ci]
        L.orc_logreg_grad_loop.restype = ctypes.c_double
        _lib = L
    return _lib


def _dp(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double)) if a is not None else None


def _ip(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)) if a is not None else None


# ------------------------------------------------------------------- RNG / generator
def philox(ctr, key):
    u32 = ctypes.c_uint32
    o = (u32 * 4)()
    lib().orc_philox4x32_10((u32 * 4)(*ctr), (u32 * 2)(*key), o)
    return list(o)


def gen_x(seed, row0, nrows, d):
    X = np.empty((nrows, d), np.float64)
    lib().orc_gen_x(seed, row0, nrows, d, _dp(X))
    return X


def gen_beta(seed, d):
    b = np.empty(d, np.float64)
    lib().orc_gen_beta(seed, d, _dp(b))
    return b


def gen_y_logistic(seed, row0, X, alpha, beta):
    X = np.ascontiguousarray(X, np.float64)
    n, d = X.shape
    y = np.empty(n, np.int32)
    margin = np.empty(n, np.float64)
    beta = np.ascontiguousarray(beta, np.float64)
    lib().orc_gen_y_logistic(seed, row0, n, d, _dp(X), float(alpha), _dp(beta), _ip(y), _dp(margin))
    return y, margin


def gen_y_linear(seed, row0, X, alpha, beta, sigma=1.0):
    X = np.ascontiguousarray(X, np.float64)
    n, d = X.shape
    y = np.empty(n, np.float64)
    beta = np.ascontiguousarray(beta, np.float64)
    lib().orc_gen_y_linear(seed, row0, n, d, _dp(X), float(alpha), _dp(beta), float(sigma), _dp(y))
    return y


# --------------------------------------------------------------------- densities
class _Data(ctypes.Structure):
    _fields_ = [("family", ctypes.c_int), ("n", ctypes.c_int64), ("d", ctypes.c_int),
                ("x", ctypes.c_void_p), ("y", ctypes.c_void_p), ("yi", ctypes.c_void_p),
                ("sigma", ctypes.c_void_p), ("pa", ctypes.c_double), ("pb", ctypes.c_double)]


class _Cfg(ctypes.Structure):
    _fields_ = [("num_warmup", ctypes.c_int), ("num_samples", ctypes.c_int), ("max_depth", ctypes.c_int),
                ("adapt_delta", ctypes.c_double), ("gamma", ctypes.c_double), ("kappa", ctypes.c_double),
                ("t0", ctypes.c_double), ("stepsize", ctypes.c_double), ("init_radius", ctypes.c_double),
                ("init_buffer", ctypes.c_int), ("term_buffer", ctypes.c_int), ("window", ctypes.c_int),
                ("adapt_engaged", ctypes.c_int), ("seed", ctypes.c_uint64), ("stepsize_jitter", ctypes.c_double),
                ("uturn_ext", ctypes.c_int)]


class Model:
    """Holds host arrays for one shard and exposes lp/grad and the NUTS twin."""

    def __init__(self, family, *, y=None, sigma=None, X=None, prior_alpha=0.0, prior_beta=0.0):
        """prior_alpha / prior_beta: scales s of normal(0, s) priors on alpha / beta (0: flat)."""
        self.family = family
        if family == FAM_SCHOOLS:
            self.y = np.ascontiguousarray(y, np.float64)
            self.sigma = np.ascontiguousarray(sigma, np.float64)
            self.X = None
            self.n, self.d = len(self.y), 0
            self.D = self.n + 2
        else:
            self.X = np.ascontiguousarray(X, np.float64)
            self.n, self.d = self.X.shape
            if family == FAM_LOGREG:
                self.y = np.ascontiguousarray(y, np.int32)
                self.D = self.d + 1
            else:
                self.y = np.ascontiguousarray(y, np.float64)
                self.D = self.d + 2
            self.sigma = None
        self._s = _Data(family, self.n, self.d,
                        self.X.ctypes.data if self.X is not None else None,
                        self.y.ctypes.data if family != FAM_LOGREG else None,
                        self.y.ctypes.data if family == FAM_LOGREG else None,
                        self.sigma.ctypes.data if self.sigma is not None else None,
                        1.0 / prior_alpha ** 2 if prior_alpha else 0.0, 1.0 / prior_beta ** 2 if prior_beta else 0.0)

    def lpgrad(self, q):
        q = np.ascontiguousarray(q, np.float64)
        g = np.empty(self.D, np.float64)
        L = lib()
        if self.family == FAM_SCHOOLS:
            lp = L.orc_schools_lpgrad(self.n, _dp(self.y), _dp(self.sigma), _dp(q), _dp(g))
        elif self.family == FAM_LOGREG:
            lp = L.orc_logreg_lpgrad(self.n, self.d, _dp(self.X), _ip(self.y), _dp(q), _dp(g))
        else:
            lp = L.orc_linreg_lpgrad(self.n, self.d, _dp(self.X), _dp(self.y), _dp(q), _dp(g))
        if self.family != FAM_SCHOOLS and (self._s.pa or self._s.pb):
            lp += L.orc_prior_lpgrad(self._s.pa, self._s.pb, self.d, _dp(q), _dp(g))
        return lp, g

    def run_chain(self, *, num_warmup=1000, num_samples=1000, max_depth=10, adapt_delta=0.8,
                  gamma=0.05, kappa=0.75, t0=10.0, stepsize=1.0, init_radius=2.0,
                  init_buffer=75, term_buffer=50, window=25, adapt_engaged=True, seed=1234,
                  gid=0, init=None, stepsize_jitter=0.0, uturn_ext=False):
        """uturn_ext: Stan >= 2.23's extra U-turn checks between subtrees (default: Stan 2.19)."""
        cfg = _Cfg(num_warmup, num_samples, max_depth, adapt_delta, gamma, kappa, t0, stepsize,
                   init_radius, init_buffer, term_buffer, window, int(adapt_engaged), seed, stepsize_jitter,
                   int(bool(uturn_ext)))
        T = num_warmup + num_samples
        q = np.empty((T, self.D))
        lp = np.empty(T)
        st = np.empty((T, 6))
        fin = np.empty(self.D + 1)
        init_a = None if init is None else np.ascontiguousarray(init, np.float64)
        ng = lib().orc_run_chain(ctypes.byref(self._s), ctypes.byref(cfg), gid, _dp(init_a),
                                 _dp(q), _dp(lp), _dp(st), _dp(fin))
        if ng < 0:
            raise RuntimeError("oracle: step size left (0, 1e7]")
        return dict(q=q, lp=lp, stats=st, stepsize=fin[0], inv_metric=fin[1:], n_grad=ng)

    def transition(self, q, *, seed, gid, iteration, eps, inv_metric=None, max_depth=10, uturn_ext=False):
        q = np.array(q, np.float64, copy=True)
        im = np.ones(self.D) if inv_metric is None else np.ascontiguousarray(inv_metric, np.float64)
        lp = ctypes.c_double()
        st = np.empty(6)
        ng = lib().orc_transition(ctypes.byref(self._s), seed, gid, iteration, max_depth, eps,
                                  _dp(im), _dp(q), ctypes.byref(lp), _dp(st), int(bool(uturn_ext)))
        return q, lp.value, st, ng


# ---------------------------------------------------------------- combine (numpy)
def consensus_avg_ref(f1, f2):
    """Restates stark/stark.py:8-20 (``consensus_avg(J).c``): NaN guard on f1 (:9-10),
    W_j = inv(np.cov(f_j)) (:17), returns [W0 + W1, W0 f1 + W1 f2] (:19-20)."""
    if np.isnan(f1).any():
        return f2
    w = [np.linalg.inv(np.cov(f)) for f in (f1, f2)]
    return [w[0] + w[1], np.dot(w[0], f1) + np.dot(w[1], f2)]


def consensus_combine_ref(draws):
    """General-S consensus: (sum_s W_s)^-1 sum_s W_s theta_s with W_s = inv(cov(theta_s)),
    the evident intent of stark/stark.py:59-71 (the reference reducer only works for two
    partitions).  Shards holding any NaN are left out, as the guard
    at stark/stark.py:9-10 intends.  draws: (S, P, n) -> (P, n)."""
    sw = None
    swt = None
    for f in draws:
        if np.isnan(f).any():
            continue
        w = np.linalg.inv(np.atleast_2d(np.cov(f)))       # a 1-row block (lp__ alone): 1 x 1
        sw = w if sw is None else sw + w
        wt = np.dot(w, f)
        swt = wt if swt is None else swt + wt
    if sw is None:
        raise ValueError("every shard holds NaN draws")
    return np.dot(np.linalg.inv(sw), swt)


# ------------------------------------------------------------- exact moments
SCHOOLS_Y = np.array([28, 8, -3, 7, -1, 1, 18, 12], np.float64)        # example/stark_ex.py:5
SCHOOLS_SIGMA = np.array([15, 10, 16, 11, 9, 11, 10, 18], np.float64)  # example/stark_ex.py:6


def schools_exact_moments(y, sigma, n_mu=1601, n_logtau=1601):
    """Posterior means / variances of (mu, log tau, eta_j) for the non-centred 8 schools
    model with flat priors on mu and tau (example/schools.stan).  Given (mu, tau),
    theta_j ~ N(m_j, v_j) with v_j = 1/(1/tau^2 + 1/s_j^2), m_j = v_j (mu/tau^2 + y_j/s_j^2);
    the (mu, tau) marginal is prod_j N(y_j | mu, s_j^2 + tau^2) (flat in tau, measure dtau).
    Integrated on a (mu, u=log tau) grid with density * tau.  Returns dict of means/vars
    over the unconstrained coordinates (mu, u, eta_1..J)."""
    y = np.asarray(y, np.float64)
    s2 = np.asarray(sigma, np.float64) ** 2
    mus = np.linspace(-60, 80, n_mu)
    us = np.linspace(-12, 6.5, n_logtau)
    MU, U = np.meshgrid(mus, us, indexing="ij")
    T2 = np.exp(2 * U)
    logp = U.copy()   # Jacobian dtau = tau du
    for yj, sj2 in zip(y, s2):
        var = sj2 + T2
        logp += -0.5 * np.log(var) - 0.5 * (yj - MU) ** 2 / var
    w = np.exp(logp - logp.max())
    w /= w.sum()
    out_mean, out_var = [], []

    def mom(f):
        m = (w * f).sum()
        return m, (w * f * f).sum() - m * m

    for f in (MU, U):
        m, v = mom(f)
        out_mean.append(m)
        out_var.append(v)
    tau = np.exp(U)
    for yj, sj2 in zip(y, s2):
        vj = 1.0 / (1.0 / T2 + 1.0 / sj2)
        mj = vj * (MU / T2 + yj / sj2)
        # eta = (theta - mu)/tau: conditional mean/var
        em = (mj - MU) / tau
        ev = vj / T2
        m = (w * em).sum()
        v = (w * (ev + em * em)).sum() - m * m
        out_mean.append(m)
        out_var.append(v)
    return np.array(out_mean), np.array(out_var)


def schools_exact_extract_means(y, sigma, n_mu=1601, n_logtau=1601):
    """Posterior means of the 2J+3 rows fit.extract() gives for example/schools.stan, in
    order: mu, tau, eta[1..J], theta[1..J], lp__ (the 19 "targets" of test/stark_test.py:26
    for J = 8).  Same quadrature as schools_exact_moments; given (mu, tau) eta_j is normal
    with mean em_j and variance ev_j, so theta_j = mu + tau eta_j and
    lp__ = -sum eta^2 / 2 - sum ((y - theta) / sigma)^2 / 2 + log tau (Stan's log_prob,
    propto, Jacobian of tau > 0) have closed-form conditional means."""
    y = np.asarray(y, np.float64)
    s2 = np.asarray(sigma, np.float64) ** 2
    mus = np.linspace(-60, 80, n_mu)
    us = np.linspace(-12, 6.5, n_logtau)
    MU, U = np.meshgrid(mus, us, indexing="ij")
    T2 = np.exp(2 * U)
    tau = np.exp(U)
    logp = U.copy()
    for yj, sj2 in zip(y, s2):
        var = sj2 + T2
        logp += -0.5 * np.log(var) - 0.5 * (yj - MU) ** 2 / var
    w = np.exp(logp - logp.max())
    w /= w.sum()
    mean_eta, mean_theta = [], []
    lp = U.copy()
    for yj, sj2 in zip(y, s2):
        vj = 1.0 / (1.0 / T2 + 1.0 / sj2)
        mj = vj * (MU / T2 + yj / sj2)
        em, ev = (mj - MU) / tau, vj / T2
        mean_eta.append((w * em).sum())
        mean_theta.append((w * mj).sum())
        lp += -0.5 * (ev + em * em) - 0.5 * ((yj - mj) ** 2 + vj) / sj2
    return np.array([(w * MU).sum(), (w * tau).sum()] + mean_eta + mean_theta + [(w * lp).sum()])


def linreg_exact_moments(X, y):
    """Flat-prior linear regression with sigma = exp(u), Jacobian u, i.e. p(sigma) flat:
    the marginal posterior of (alpha, beta) is multivariate t with nu = N - k - 1 dof
    (k = number of coefficients), location = OLS, scale s^2 (X'X)^-1 with
    s^2 = RSS/(N - k - 1); its covariance is nu/(nu-2) s^2 (X'X)^-1.
    (p(beta, sigma | y) prop sigma^-N exp(-RSS(beta)/2sigma^2); integrating sigma gives
    [RSS(beta)]^-(N-1)/2, a t with N - k - 1 dof.)  Returns (mean, cov) of (alpha, beta)."""
    n = X.shape[0]
    A = np.hstack([np.ones((n, 1)), X])
    k = A.shape[1]
    xtx = A.T @ A
    mean = np.linalg.solve(xtx, A.T @ y)
    rss = float(((y - A @ mean) ** 2).sum())
    nu = n - k - 1
    s2 = rss / nu
    cov = (nu / (nu - 2.0)) * s2 * np.linalg.inv(xtx)
    return mean, cov
