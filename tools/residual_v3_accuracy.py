#!/usr/bin/env python3
"""Accuracy of the logistic residuals emulated in numpy -- v3 (sweep.hip: logit_resid3, the 64-chain
pass F epilogue) and v4 (sweep16.hip: logit_resid4, the 16-chain sweep, with its per-lane
product accumulation of the log terms) -- the same operation sequences in float64 with every fma
evaluated in long double and rounded once, against Stan 2.19's bernoulli_logit term and
derivative (+-20 cutoffs) in long double.  Prints the worst errors by t-range, the relative error
of an lp sum over 2e6 uniform t in [-25, 25], and the NaN / +-inf cases.  (The GPU kernels
themselves are checked against the C oracle within 1e-10 by tests/test_gpu_kernels.py.)"""
import numpy as np

mp = np.longdouble
Q1, Q2, Q3, Q4 = -0.4999999999996968, 0.33333333333269194, -0.25000063579045223, 0.2000006787837857
MAGIC = 6755399441055744.0
INV_L = 369.3299304675746
L_HI, L_LO = 0.0027076061742263846, -1.6409824498184568e-13
TE = np.array([np.float64(mp(2) ** (mp(i) / 256)) for i in range(256)])
CJ = np.array([np.float64(mp(256) / (256 + j)) for j in range(257)])
DJ = np.array([np.float64(mp(j) / (256 + j)) for j in range(257)])
LJ = np.array([np.float64(np.log1p(mp(j) / 256)) for j in range(257)])


def fma(a, b, c):
    return (mp(a) * mp(b) + mp(c)).astype(np.float64)


def resid3(t, newton=True):
    t = np.asarray(t, np.float64)
    with np.errstate(invalid="ignore", over="ignore"):
        a = np.fmin(fma(np.fmax(-20.0 - t, 0.0), 2.0 ** 60, np.abs(t)), 700.0)
        sn = fma(-a, INV_L, MAGIC)
        ni = (sn.view(np.uint64) & 0xFFFFFFFF).astype(np.uint32).view(np.int32).astype(np.int64)
        n = sn - MAGIC
        r = fma(-n, L_LO, fma(-n, L_HI, -a))
        p = fma(fma(fma(fma(1.0 / 24.0, r, 1.0 / 6.0), r, 0.5), r, 1.0), r, 1.0)
        e = np.ldexp(TE[ni & 255] * p, (ni >> 8).astype(np.int32))
        j = np.trunc(fma(e, 256.0, 0.5)).astype(np.int64)
        rl = fma(e, CJ[j], -DJ[j])
        q = fma(fma(fma(fma(Q4, rl, Q3), rl, Q2), rl, Q1), rl, 1.0)
        lg = fma(rl, q, LJ[j])
        u = 1.0 + e
        ri = (1.0 / u) * (1 + 2.2e-16)           # an rcp seed one ulp off
        if newton:
            ri = fma(ri, fma(-u, ri, 1.0), ri)
        w = e * ri
        dvp = np.where(np.signbit(t), ri, w)
        lt = fma(0.5, t, fma(-0.5, np.abs(t), -lg))
    return lt, dvp


# ---- v4 (sweep16.hip: logit_resid4)
INV_L4, L4 = 1477.3197218702985, 0.0006769015435155716
C2, C3 = 0.5000000039583942, 0.16666666713444417
TE4 = np.array([np.float64(mp(2) ** (mp(i) / 1024)) for i in range(1024)])


def resid4(t, lanes=64, flush=256):
    """v4 on t = (2y - 1) eta: returns (lp sum as the kernel forms it, dv/sgn per element).
    The elements are dealt to `lanes` lanes in order (lane l takes t[l::lanes]); each lane keeps
    lm = sum(t - |t|) and sp = prod(1 + e) - 1, adding log1p(sp) every `flush` elements."""
    t = np.asarray(t, np.float64)
    with np.errstate(invalid="ignore", over="ignore"):
        a = np.fmin(np.abs(t), 700.0)
        sn = fma(-a, INV_L4, MAGIC)
        ni = (sn.view(np.uint64) & 0xFFFFFFFF).astype(np.uint32).view(np.int32).astype(np.int64)
        n = sn - MAGIC
        r = fma(-n, L4, -a)
        p = fma(fma(fma(C3, r, C2), r, 1.0), r, 1.0)
        ke = np.where(t < -20.0, -1100, ni >> 10).astype(np.int32)
        e = np.ldexp(TE4[ni & 1023] * p, ke)
        u = 1.0 + e
        ri = (1.0 / u) * (1 + 2.2e-16)           # an rcp seed one ulp off
        ri = fma(ri, fma(-u, ri, 1.0), ri)
        w = e * ri
        dvp = np.where(t > 0, w, ri)
        m = t - np.abs(t)
    k = -(-len(t) // lanes) * lanes
    E = np.zeros(k)
    U = np.ones(k)
    M = np.zeros(k)
    E[:len(t)], U[:len(t)], M[:len(t)] = e, u, m
    E, U, M = E.reshape(-1, lanes), U.reshape(-1, lanes), M.reshape(-1, lanes)
    lm = M.sum(0)
    sp = np.zeros(lanes)
    ll = np.zeros(lanes)
    for i in range(E.shape[0]):
        sp = fma(sp, U[i], E[i])
        if i % flush == flush - 1:
            ll = ll + np.log1p(sp)
            sp = np.zeros(lanes)
    ll = ll + np.log1p(sp)
    return float((0.5 * lm - ll).sum()), dvp


def stan(t):
    t = t.astype(mp)
    with np.errstate(over="ignore"):
        lt = np.where(t > 20, -np.exp(-t), np.where(t < -20, t, -np.log1p(np.exp(-t))))
        dv = np.where(t > 20, np.exp(-t), np.where(t < -20, mp(1), 1 / (1 + np.exp(t))))
    return lt, dv


def main():
    rng = np.random.default_rng(0)
    t = np.concatenate([rng.uniform(-25, 25, 2_000_000), rng.uniform(-1, 1, 200_000),
                        np.linspace(-21, -19, 20001), np.linspace(19, 21, 20001)])
    lt, dv = resid3(t)
    lr, dr = stan(t)
    ea = np.abs(lt - lr.astype(np.float64))
    er = np.abs(dv - dr.astype(np.float64)) / dr.astype(np.float64)
    for lo, hi in [(-25, -20), (-20, -5), (-5, 0), (0, 5), (5, 20), (20, 25)]:
        m = (t >= lo) & (t < hi)
        print(f"t in [{lo:4d}, {hi:4d}): lt abs err max {ea[m].max():.2e}, dv rel err max {er[m].max():.2e}")
    n = 2_000_000
    print("lp sum over uniform t in [-25, 25]: relative error %.2e" %
          (abs((lt[:n] - lr[:n].astype(np.float64)).sum()) / abs(lr[:n].astype(np.float64).sum())))
    print("t = NaN, +inf, -inf ->", resid3(np.array([np.nan, np.inf, -np.inf])))
    lp4, dv4 = resid4(t[:n])
    er4 = np.abs(dv4 - dr[:n].astype(np.float64)) / dr[:n].astype(np.float64)
    print("v4: lp sum over uniform t in [-25, 25]: relative error %.2e; dv rel err max %.2e" %
          (abs(lp4 - float(lr[:n].sum())) / abs(float(lr[:n].sum())), er4.max()))
    lt0, dv0 = resid3(t[:n], newton=False)
    print("without the Newton step (rcp seed 1 ulp off): dv rel err max %.2e" %
          (np.abs(dv0 - dr[:n].astype(np.float64)) / dr[:n].astype(np.float64)).max())


if __name__ == "__main__":
    main()
