"""Sampler diagnostics: effective sample size and split R-hat.

Restates Stan 2.19.1's ``stan::analyze::compute_effective_sample_size`` (Geyer initial
positive + initial monotone sequence on the multi-chain autocovariance, with the
improved-tail term ``rho_hat_s(max_s + 1)`` that 2.19 already has) and
``compute_split_potential_scale_reduction`` -- the numbers pystan 2.19 / ``stansummary``
report.  Stan 2.19 has no lower bound on tau_hat; the
``tau_hat >= 1 / log10(total draws)`` floor of later releases is available as
``ess(..., floor=True)`` and is off by default.  Host-side reporting only; not on the hot
path.
"""
from __future__ import annotations

import numpy as np


def _autocovariance(x: np.ndarray) -> np.ndarray:
    n = x.shape[0]
    m = 1
    while m < 2 * n:
        m *= 2
    f = np.fft.rfft(x - x.mean(), m)
    ac = np.fft.irfft(f * np.conj(f), m)[:n]
    return ac / n


def ess(chains, floor: bool = False) -> float:
    """ESS of one scalar quantity; `chains` is (num_chains, num_draws).
    floor: apply the later releases' tau_hat >= 1/log10(N) bound (not in Stan 2.19)."""
    chains = np.atleast_2d(np.asarray(chains, np.float64))
    nc, n = chains.shape
    if n < 4:
        return float("nan")
    if np.all(chains == chains.flat[0]) or not np.all(np.isfinite(chains)):
        return float("nan")
    acov = np.stack([_autocovariance(c) for c in chains])
    chain_mean = chains.mean(axis=1)
    chain_var = acov[:, 0] * n / (n - 1.0)
    mean_var = chain_var.mean()
    var_plus = mean_var * (n - 1.0) / n
    if nc > 1:
        var_plus += chain_mean.var(ddof=1)
    rho = np.zeros(n)
    rho_even = 1.0
    rho[0] = rho_even
    rho_odd = 1.0 - (mean_var - acov[:, 1].mean()) / var_plus
    rho[1] = rho_odd
    s = 1
    while s < n - 4 and (rho_even + rho_odd) > 0:
        rho_even = 1.0 - (mean_var - acov[:, s + 1].mean()) / var_plus
        rho_odd = 1.0 - (mean_var - acov[:, s + 2].mean()) / var_plus
        if rho_even + rho_odd >= 0:
            rho[s + 1] = rho_even
            rho[s + 2] = rho_odd
        s += 2
    max_s = s
    if rho_even > 0:
        rho[max_s + 1] = rho_even
    for t in range(1, max_s - 2, 2):
        if rho[t + 1] + rho[t + 2] > rho[t - 1] + rho[t]:
            rho[t + 1] = (rho[t - 1] + rho[t]) / 2.0
            rho[t + 2] = rho[t + 1]
    tau = -1.0 + 2.0 * rho[:max_s].sum() + rho[max_s + 1]
    if floor:
        tau = max(tau, 1.0 / np.log10(nc * n))
    return float(nc * n / tau)


def split_rhat(chains) -> float:
    chains = np.atleast_2d(np.asarray(chains, np.float64))
    nc, n = chains.shape
    h = n // 2
    sp = np.concatenate([chains[:, :h], chains[:, n - h:]], axis=0)
    m, k = sp.shape
    means = sp.mean(axis=1)
    W = sp.var(axis=1, ddof=1).mean()
    B = k * means.var(ddof=1)
    var_plus = (k - 1.0) / k * W + B / k
    return float(np.sqrt(var_plus / W))


def ess_matrix(draws: np.ndarray, chains: int) -> np.ndarray:
    """ESS per row of a P x (chains*n) chain-major draw matrix."""
    P, S = draws.shape
    n = S // chains
    return np.array([ess(draws[p, : chains * n].reshape(chains, n)) for p in range(P)])


def summary(draws: np.ndarray, chains: int, names=None) -> list:
    P, S = draws.shape
    n = S // chains
    out = []
    for p in range(P):
        x = draws[p, : chains * n].reshape(chains, n)
        e = ess(x)
        sd = x.std(ddof=1)
        out.append({"name": names[p] if names else p, "mean": float(x.mean()), "sd": float(sd),
                    "mcse": float(sd / np.sqrt(e)) if e and e > 0 else float("nan"), "n_eff": e,
                    "rhat": split_rhat(x)})
    return out
