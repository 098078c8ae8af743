#!/usr/bin/env python3
"""Accuracy of the fused NUTS kernel's table-driven exp / log1p (nuts.hip: exp_mt, log1p01_mt,
log_sum_exp_mt) emulated in numpy: the same operation sequence in float64 with every fma
evaluated in long double and rounded once, against long-double references.  Prints the worst
relative errors in ulps over the argument ranges the state machine feeds them (energy differences,
log weights)."""
import numpy as np

mp = np.longdouble
MAGIC = 6755399441055744.0
INV_L, L_HI, L_LO = 184.6649652337873, 0.005415212348452769, -3.2819649005320973e-13
TE = np.array([np.float64(mp(2) ** (mp(i) / 128)) for i in range(128)])
CJ = np.array([np.float64(mp(128) / (128 + j)) for j in range(129)])
DJ = np.array([np.float64(mp(j) / (128 + j)) for j in range(129)])
LJ = np.array([np.float64(np.log1p(mp(j) / 128)) for j in range(129)])


def fma(a, b, c):
    return (mp(a) * mp(b) + mp(c)).astype(np.float64)


def exp_mt(x):
    x = np.asarray(x, np.float64)
    with np.errstate(invalid="ignore", over="ignore"):
        xc = np.fmin(np.fmax(x, -800.0), 800.0)
        sn = fma(xc, INV_L, MAGIC)
        ni = (sn.view(np.uint64) & 0xFFFFFFFF).astype(np.uint32).view(np.int32).astype(np.int64)
        n = sn - MAGIC
        r = fma(-n, L_LO, fma(-n, L_HI, xc))
        p = fma(fma(fma(fma(fma(1.0 / 120.0, r, 1.0 / 24.0), r, 1.0 / 6.0), r, 0.5), r, 1.0), r, 1.0)
        e = np.ldexp(TE[ni & 127] * p, (ni >> 7).astype(np.int32))
    return np.where(np.isnan(x), x, e)


def log1p01_mt(e):
    e = np.asarray(e, np.float64)
    j = np.trunc(fma(e, 128.0, 0.5)).astype(np.int64)
    rl = fma(e, CJ[j], -DJ[j])
    q = fma(fma(fma(fma(fma(fma(1.0 / 7.0, rl, -1.0 / 6.0), rl, 0.2), rl, -0.25), rl, 1.0 / 3.0), rl, -0.5), rl, 1.0)
    return fma(rl, q, LJ[j])


def ulps(got, ref):
    ref = np.asarray(ref, mp)
    return np.abs(np.asarray(got, mp) - ref) / np.spacing(np.abs(ref.astype(np.float64)))


def main():
    rng = np.random.default_rng(0)
    x = np.concatenate([rng.uniform(-40, 0, 500_000), rng.uniform(-700, 700, 500_000), rng.uniform(-1e-3, 1e-3, 100_000)])
    print("exp_mt: max %.2f ulp over [-700, 700]" % ulps(exp_mt(x), np.exp(x.astype(mp))).max())
    e = np.concatenate([rng.uniform(0, 1, 500_000), 10.0 ** rng.uniform(-300, 0, 200_000)])
    print("log1p01_mt: max %.2f ulp over [0, 1]" % ulps(log1p01_mt(e), np.log1p(e.astype(mp))).max())
    print("exp_mt(-inf, inf, nan, -1000, 1000) =", exp_mt(np.array([-np.inf, np.inf, np.nan, -1000.0, 1000.0])))


if __name__ == "__main__":
    main()
