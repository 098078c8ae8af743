"""Full-data posterior reference for the consensus check at scale (measurement infrastructure).

At the headline size (logistic regression, N = 1e8 rows, d = 100, flat priors) the full-data
posterior is Gaussian to O(d / sqrt(N)) ~ 1e-2 posterior sds (Bernstein-von Mises), so its
mean and covariance are the MAP and the inverse negative Hessian there.  Both come from the
GPU's own log-density gradient (``stk_log_density_grad`` through ``engine.Model``):

  * the full-data gradient is the sum of the shards' gradients (flat priors: every shard's
    log density is a pure sum over its rows, so the sum is the full-data log density);
  * the Hessian is the central difference of the gradient, column j from the two points
    q +- h_j e_j (2 D points per Hessian, in batches of 16 chains = one fp64-MFMA sweep of
    each shard per batch);
  * Newton's method from the pooled draw mean converges in 2-3 steps.

The same on each shard alone gives every subposterior's Laplace mean and precision: the
"exact" consensus weights W_s = -H_s, which separate the combine's weight noise (sampled
covariances) from the subposteriors' own Monte Carlo error.

Used by tools/consensus_check.py, bench.py and the -m gpu consensus tests; not on the
product path.
"""
from __future__ import annotations

import numpy as np


def _grad(model, shards, Q, batch=16, reduce=None):
    """lp and gradient at the rows of Q, summed over `shards` (and over ranks by `reduce`,
    a function that sums a float64 array over the process group in place, when the shards
    are spread over several processes)."""
    Q = np.atleast_2d(np.asarray(Q, np.float64))
    lp = np.zeros(Q.shape[0])
    g = np.zeros(Q.shape)
    for b0 in range(0, Q.shape[0], batch):
        qb = np.ascontiguousarray(Q[b0:b0 + batch])
        for s in shards:
            l_, g_ = model.log_density_grad(s, qb)
            lp[b0:b0 + len(qb)] += l_
            g[b0:b0 + len(qb)] += g_
    if reduce is not None:
        both = np.concatenate([lp, g.reshape(-1)])
        reduce(both)
        lp, g = both[:lp.size], both[lp.size:].reshape(g.shape)
    return lp, g


def hessian(model, shards, q, h, reduce=None):
    """Central-difference Hessian of the summed log density at q (steps h, one per coordinate)."""
    D = q.shape[0]
    pts = np.empty((2 * D, D))
    for j in range(D):
        pts[2 * j] = q
        pts[2 * j + 1] = q
        pts[2 * j, j] += h[j]
        pts[2 * j + 1, j] -= h[j]
    _, g = _grad(model, shards, pts, reduce=reduce)
    H = np.empty((D, D))
    for j in range(D):
        H[:, j] = (g[2 * j] - g[2 * j + 1]) / (2.0 * h[j])
    return 0.5 * (H + H.T)


def laplace(model, shards, q0, sd0, iters=6, tol=1e-7, reduce=None):
    """MAP and covariance (-H)^-1 of the posterior formed by `shards`, from q0 (sd0: a rough
    posterior sd per coordinate, sets the difference steps 0.1 sd).  Returns (mean, cov, info).
    With shards on several ranks every rank calls this with its own shards, the same q0/sd0
    and a `reduce` that sums over ranks; all ranks then take identical Newton steps."""
    q = np.asarray(q0, np.float64).copy()
    h = 0.1 * np.asarray(sd0, np.float64)
    steps = []
    for _ in range(iters):
        _, g = _grad(model, shards, q[None], reduce=reduce)
        H = hessian(model, shards, q, h, reduce=reduce)
        cov = np.linalg.inv(-H)
        dq = cov @ g[0]
        q = q + dq
        sd = np.sqrt(np.diag(cov))
        h = 0.1 * sd
        steps.append(float(np.abs(dq / sd).max()))
        if steps[-1] < tol:
            break
    H = hessian(model, shards, q, h, reduce=reduce)
    cov = np.linalg.inv(-H)
    cov = 0.5 * (cov + cov.T)
    return q, cov, {"newton_steps_in_sd": steps}


def consensus_fixed_weights(draws, precisions):
    """(sum W_s)^-1 sum W_s theta_s with given weights (P x P each) on P x S draw matrices."""
    sw = sum(precisions)
    swt = sum(W @ x for W, x in zip(precisions, draws))
    return np.linalg.solve(sw, swt)
