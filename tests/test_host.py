"""Host-side logic (CPU only): the C-ABI library, Stan front end, RDD shim, driver
orchestration against the reference's own driver outputs, diagnostics."""
import collections
import os
import re

import numpy as np
import pytest

from conftest import ROOT


# ---------------------------------------------------------------- C ABI
def _header_symbols():
    src = open(os.path.join(ROOT, "include", "stark_hip.h")).read()
    return sorted(set(re.findall(r"STK_API\s+[\w\s\*]+?\b(stk_\w+)\s*\(", src)))


def test_library_exports_every_header_symbol():
    import ctypes
    from stark_amd import _lib
    lib = _lib.load()
    names = _header_symbols()
    assert len(names) >= 25
    for n in names:
        assert hasattr(lib, n), n
    bound = {s[0] for s in _lib.SIGNATURES}
    assert set(names) == bound, set(names) ^ bound
    assert lib.stk_version() == 1
    c = _lib.default_config()
    assert (c.num_warmup, c.num_samples, c.chains, c.max_depth) == (1000, 1000, 1, 10)
    assert c.adapt_delta == 0.8 and c.stepsize == 1.0 and c.adapt_init_buffer == 75
    # struct layouts must match the C header: compile a probe with gcc
    import subprocess, tempfile
    src = ('#include <stdio.h>\n#include <stddef.h>\n#include "stark_hip.h"\n'
           'int main(){printf("%zu %zu %zu %zu %zu %zu", sizeof(stk_config), sizeof(stk_shard), sizeof(stk_run_info),'
           ' offsetof(stk_config, seed), offsetof(stk_config, shard_ids), offsetof(stk_config, chains_per_wave));return 0;}')
    with tempfile.TemporaryDirectory() as d:
        open(os.path.join(d, "p.c"), "w").write(src)
        subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), "-o", os.path.join(d, "p"), os.path.join(d, "p.c")],
                       check=True)
        got = [int(v) for v in subprocess.run([os.path.join(d, "p")], capture_output=True, text=True).stdout.split()]
    assert got == [ctypes.sizeof(_lib.Config), ctypes.sizeof(_lib.Shard), ctypes.sizeof(_lib.RunInfo),
                   _lib.Config.seed.offset, _lib.Config.shard_ids.offset, _lib.Config.chains_per_wave.offset]


def test_no_device_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from stark_amd import engine
    from stark_amd._lib import StarkHipError
    with pytest.raises(StarkHipError):
        engine.Context(0)


# ---------------------------------------------------------------- front end
def test_recognise_programs():
    from stark_amd import frontend
    for fam in ("schools", "logistic", "linear"):
        code = open(os.path.join(ROOT, "stark_amd", "models", f"{fam}.stan")).read()
        assert frontend.recognise(code) == fam
    newsyntax = """
    data { int<lower=0> J; array[J] real y; array[J] real<lower=0> sigma; }
    parameters { real mu; real<lower=0> tau; vector[J] eta; }
    transformed parameters { vector[J] theta = mu + tau * eta; }
    model { eta ~ std_normal(); y ~ normal(theta, sigma); }"""
    assert frontend.recognise(newsyntax) == "schools"
    with pytest.raises(NotImplementedError):
        frontend.recognise(newsyntax.replace("std_normal()", "normal(0, 2)"))
    prior = open(os.path.join(ROOT, "stark_amd", "models", "logistic.stan")).read().replace(
        "model {", "model {\n beta ~ normal(0, 1);")
    assert frontend.program_info(prior) == ("logistic", {"beta": 1.0})   # normal(0, s) priors: supported
    with pytest.raises(NotImplementedError):
        frontend.recognise(prior.replace("normal(0, 1)", "cauchy(0, 1)"))


def test_pack_data_validation():
    from stark_amd import frontend
    d = frontend.pack_data("schools", {"J": 2, "y": [1, 2], "sigma": [3, 4]})
    assert d["y"].dtype == np.float64
    with pytest.raises(ValueError):
        frontend.pack_data("schools", {"J": 3, "y": [1, 2], "sigma": [3, 4]})
    with pytest.raises(ValueError):
        frontend.pack_data("schools", {"J": 2, "y": [1, 2], "sigma": [3, 0]})
    r = frontend.pack_data("logistic", {"N": 2, "K": 1, "x": [[1.0], [2.0]], "y": [0, 1]})
    assert r["y"].dtype == np.int32 and r["x"].shape == (2, 1)
    assert frontend.column_names("schools", {"J": 2}) == ["mu", "tau", "eta[1]", "eta[2]", "theta[1]", "theta[2]",
                                                          "lp__"]


def test_sampling_config_mapping():
    from stark_amd.stark import sampling_config
    datas = [{"J": 4, "y": [1, 2, 3, 4], "sigma": [1, 1, 1, 1]}]
    c = sampling_config("schools", datas, iter=5000, chains=1, n_jobs=1, seed=9,
                        control={"adapt_delta": 0.9, "max_treedepth": 12, "stepsize_jitter": 0.3})
    assert c["num_warmup"] == 2500 and c["num_samples"] == 2500
    assert c["adapt_delta"] == 0.9 and c["max_depth"] == 12 and c["seed"] == 9
    assert c["stepsize_jitter"] == 0.3
    c0 = sampling_config("schools", datas, iter=20, chains=2, init=0, seed=1)
    assert c0["init"].shape == (12,) and not c0["init"].any()
    ci = sampling_config("schools", datas, iter=20, chains=1, seed=1, init=[{"mu": 1.0, "tau": np.e}])
    assert ci["init"][0] == 1.0 and abs(ci["init"][1] - 1.0) < 1e-15
    with pytest.raises(ValueError):
        sampling_config("schools", datas, thin=0)
    assert sampling_config("schools", datas, iter=20, thin=3, seed=1)["thin"] == 3
    # callable init, pystan 2: init(chain_id=c), or init() when it takes no chain_id
    cf = sampling_config("schools", datas, iter=20, chains=2, seed=1, init=lambda chain_id: {"mu": chain_id + 0.5})
    assert cf["init"][0] == 0.5 and cf["init"][6] == 1.5
    cg = sampling_config("schools", datas, iter=20, chains=2, seed=1, init=lambda: {"tau": 2.0})
    assert abs(cg["init"][1] - np.log(2.0)) < 1e-15 and abs(cg["init"][7] - np.log(2.0)) < 1e-15
    # the call form comes from the signature: a TypeError raised INSIDE the user's function is
    # the user's error, not a cue to retry without chain_id
    def bad(chain_id):
        raise TypeError("user bug")
    with pytest.raises(TypeError, match="user bug"):
        sampling_config("schools", datas, iter=20, chains=2, seed=1, init=bad)
    ck = sampling_config("schools", datas, iter=20, chains=2, seed=1, init=lambda **kw: {"mu": kw["chain_id"] + 2.0})
    assert ck["init"][0] == 2.0 and ck["init"][6] == 3.0
    with pytest.raises(TypeError):
        sampling_config("schools", datas, bogus=1)


def test_thin_draws_keeps_every_thin_th_iteration_per_chain():
    """Stan's num_thin (services/util/generate_transitions: save when m % num_thin == 0):
    ceil(S / thin) draws per chain, chain-major columns as the sampler writes them."""
    from stark_amd.stark import thin_draws
    P, chains, S = 3, 2, 7
    d = np.arange(P * chains * S, dtype=float).reshape(P, chains * S)
    t = thin_draws(d, chains, 3)
    assert t.shape == (P, chains * 3)
    np.testing.assert_array_equal(t[0], [0, 3, 6, 7, 10, 13])
    assert thin_draws(d, chains, 1) is d


# ---------------------------------------------------------------- RDD shim

def test_sampling_config_refuses_csv_output():
    """pystan's sample_file / diagnostic_file write Stan CSV; this build returns draws in memory
    and says so instead of silently dropping the keyword (missing item 4)."""
    from stark_amd.stark import sampling_config
    datas = [{"J": 2, "y": [1.0, 2.0], "sigma": [1.0, 1.0]}]
    for k in ("sample_file", "diagnostic_file"):
        with pytest.raises(NotImplementedError, match=k):
            sampling_config("schools", datas, iter=20, chains=1, seed=1, **{k: "/tmp/x.csv"})
    assert sampling_config("schools", datas, iter=20, chains=1, seed=1, sample_file=None)["num_samples"] == 10

def test_local_rdd_semantics():
    from stark_amd.rdd import LocalContext
    sc = LocalContext()
    school = list(zip([28, 8, -3, 7, -1, 1, 18, 12], [15, 10, 16, 11, 9, 11, 10, 18]))
    rdd = sc.parallelize(school, 2)
    assert rdd.getNumPartitions() == 2
    assert rdd.partitions()[0] == school[:4] and rdd.partitions()[1] == school[4:]
    assert [len(p) for p in sc.parallelize(range(8), 3).partitions()] == [2, 3, 3]   # Spark slicing
    assert rdd.coalesce(1).partitions() == [school]
    assert rdd.union(rdd.coalesce(1)).getNumPartitions() == 3
    assert sc.parallelize(range(5), 2).reduce(lambda a, b: a * 10 + b) == 1234


# ---------------------------------------------------------------- driver vs reference driver (fake sampler)
def _fake_extract(data, it, chains=1):
    """Same fake fit as tests/golden/make_golden.py's FakeStanModel."""
    J = data["J"]
    S = it // 2 * chains
    seed = int(abs(sum(data["y"]) * 1000 + sum(data["sigma"]))) % (2 ** 32)
    rng = np.random.default_rng(seed)
    mu = rng.normal(8, 5, S)
    tau = np.exp(rng.normal(1.5, 1.0, S))
    eta = rng.normal(0, 1, (S, J))
    theta = mu[:, None] + tau[:, None] * eta
    lp = rng.normal(-40, 3, S)
    return collections.OrderedDict([("mu", mu), ("tau", tau), ("eta", eta), ("theta", theta), ("lp__", lp)])


def prepare_school_data(data):
    return {"J": len(data), "y": [d[0] for d in data], "sigma": [d[1] for d in data]}


def _fake_stark(monkeypatch):
    from stark_amd import stark as S
    from stark_amd.rdd import LocalContext

    def fake(self, datas, **kw):
        return [S._extract_to_matrix(_fake_extract(d, kw["iter"], kw.get("chains", 1))) for d in datas]

    # below the pars / include row selection of _sample_partitions, which runs for real
    monkeypatch.setattr(S.Stark, "_draw_partitions", fake)
    sc = LocalContext()
    school = list(zip([28, 8, -3, 7, -1, 1, 18, 12], [15, 10, 16, 11, 9, 11, 10, 18]))
    st = S.Stark(sc, sc.parallelize(school, 2), prepare_school_data)
    st.setStanModel(file=os.path.join(ROOT, "stark_amd", "models", "schools.stan"))
    return st


def test_driver_mcmc_closure_matches_reference(golden, monkeypatch):
    st = _fake_stark(monkeypatch)
    g = golden("driver_ref.npz")
    school = list(zip([28, 8, -3, 7, -1, 1, 18, 12], [15, 10, 16, 11, 9, 11, 10, 18]))
    w = st._mcmc(prepare_school_data, iter=2000, chains=1, n_jobs=1)
    np.testing.assert_array_equal(w(iter(school[:4]))[0], g["part0"])


def test_driver_distribute_reference_union(golden, monkeypatch):
    st = _fake_stark(monkeypatch)
    g = golden("driver_ref.npz")
    out = st.distribute(n=4, iter=200, reference_union=True)
    assert out.shape == (41, 100)
    np.testing.assert_array_equal(out, g["naive"])
    intent = st.distribute(n=4, iter=200)
    assert intent.shape == (4 * 19, 100)


def test_driver_pars_include_matches_reference(golden, monkeypatch):
    """pystan 2 sampling(pars=, include=) forwarded through the driver's **kwargs
    (stark/stark.py:48): only the selected parameters (+ lp__, last) reach the P x S matrix --
    against the reference driver run with a fake StanModel that honours them
    (tests/golden/make_golden.py)."""
    st = _fake_stark(monkeypatch)
    g = golden("driver_ref.npz")
    out = st.distribute(n=4, iter=200, reference_union=True, pars=["theta", "tau"], include=False)
    np.testing.assert_array_equal(out, g["naive_exclude"])
    w = st._mcmc(prepare_school_data, iter=600, chains=1, n_jobs=1, pars=["eta", "mu"])
    part0 = w(iter(list(zip([28, 8, -3, 7], [15, 10, 16, 11]))))[0]
    assert part0.shape == (6, 300)          # eta[1..4], mu, lp__
    with pytest.raises(ValueError, match="No parameter"):
        st.distribute(n=2, iter=200, pars=["nope"])
    from stark_amd import frontend
    assert frontend.select_pars("logistic", {"K": 3}, ["beta"]) == [1, 2, 3, 4]
    assert frontend.select_pars("linear", {"K": 2}, ["beta"], include=False) == [0, 3, 4]


# ---------------------------------------------------------------- diagnostics
def test_ess_ar1():
    from stark_amd.diagnostics import ess, split_rhat
    rng = np.random.default_rng(0)
    rho, n, nc = 0.6, 20000, 4
    x = np.zeros((nc, n))
    e = rng.normal(size=(nc, n))
    for t in range(1, n):
        x[:, t] = rho * x[:, t - 1] + e[:, t]
    want = nc * n * (1 - rho) / (1 + rho)
    assert abs(ess(x) / want - 1) < 0.1
    assert abs(split_rhat(x) - 1) < 0.01
    iid = rng.normal(size=(4, 5000))
    assert abs(ess(iid) / 20000 - 1) < 0.1


def test_recognise_priors():
    from stark_amd import frontend
    m = os.path.join(ROOT, "stark_amd", "models")
    assert frontend.load_program_info(file=os.path.join(m, "logistic_prior.stan")) == (
        "logistic", {"alpha": 2.5, "beta": 1.0})
    lin = open(os.path.join(m, "linear.stan")).read().replace("model {", "model {\n beta ~ normal(0, .5);")
    assert frontend.program_info(lin) == ("linear", {"beta": 0.5})
    with pytest.raises(NotImplementedError):       # non-zero prior mean: not one of the families
        frontend.program_info(lin.replace("normal(0, .5)", "normal(1, .5)"))
    sch = open(os.path.join(m, "schools.stan")).read().replace("model {", "model {\n alpha ~ normal(0, 1);")
    with pytest.raises(NotImplementedError):
        frontend.program_info(sch)
    assert frontend.load_program_info(family="logistic", priors={"beta": 2.0}) == ("logistic", {"beta": 2.0})


def test_permute_draws_is_pystan_extract_order():
    """extract(permuted=True) (stark/stark.py:49): each chain's draws shuffled, chains
    concatenated; a pure function of (seed, partition, chain)."""
    from stark_amd.stark import permute_draws
    chains, n = 3, 50
    d = np.vstack([np.arange(chains * n, dtype=np.float64), -np.arange(chains * n, dtype=np.float64)])
    p = permute_draws(d, chains, seed=7, partition=2)
    for c in range(chains):
        blk = p[0, c * n:(c + 1) * n]
        assert sorted(blk) == list(range(c * n, (c + 1) * n))     # chain c's draws stay in block c
        assert not np.array_equal(blk, np.arange(c * n, (c + 1) * n))
    np.testing.assert_array_equal(p[1], -p[0])                    # columns move whole (every row)
    np.testing.assert_array_equal(p, permute_draws(d, chains, seed=7, partition=2))
    assert not np.array_equal(p, permute_draws(d, chains, seed=7, partition=3))
    with pytest.raises(ValueError):
        permute_draws(d[:, :-1], chains, seed=1, partition=0)


def test_logistic_y_must_be_binary_integers():
    from stark_amd import frontend
    ok = frontend.pack_data("logistic", {"N": 3, "K": 1, "x": [[1.0], [2.0], [3.0]], "y": [0.0, 1.0, 1]})
    assert ok["y"].tolist() == [0, 1, 1]
    for bad in ([0, 0.5, 1], [0, 1.9, 1], [0, 2, 1], [-1, 0, 1]):
        with pytest.raises(ValueError):
            frontend.pack_data("logistic", {"N": 3, "K": 1, "x": [[1.0], [2.0], [3.0]], "y": bad})


def test_ess_stan219_has_no_floor():
    """Stan 2.19's estimator has no tau_hat floor; the later releases' one is opt-in."""
    from stark_amd.diagnostics import ess
    rng = np.random.default_rng(1)
    x = np.zeros(4000)
    e = rng.normal(size=4000)
    for t in range(1, 4000):
        x[t] = -0.9 * x[t - 1] + e[t]                     # antithetic AR(1): tau = 1/19
    assert ess(x) > ess(x, floor=True)
    assert abs(ess(x, floor=True) - 4000 * np.log10(4000)) < 1e-6 * 4000


def test_laplace_reference_matches_closed_form_gaussian():
    """tools/laplace.py on a model with an exactly quadratic log density: MAP and covariance
    exact (the Newton step and the difference Hessian are exact for a quadratic)."""
    from tools import laplace as L
    rng = np.random.default_rng(3)
    D = 7
    A = rng.normal(size=(D, D))
    prec = A @ A.T + D * np.eye(D)
    mu = rng.normal(size=D)

    class Quad:
        def log_density_grad(self, s, Q):
            Q = np.atleast_2d(Q)
            r = Q - mu
            part = prec / 2.0                       # two "shards" of half the precision each
            return -0.5 * np.einsum("ij,jk,ik->i", r, part, r), -(r @ part)

    m, c, info = L.laplace(Quad(), [0, 1], mu + 0.3, np.ones(D))
    np.testing.assert_allclose(m, mu, rtol=0, atol=1e-9)
    np.testing.assert_allclose(c, np.linalg.inv(prec), rtol=1e-7, atol=1e-10)


def test_rocpd_window_selects_the_timed_dispatches(tmp_path):
    """tools/rocpd_summary.py window: the kernel dispatches inside the bench line's timed window
    (timed_window_monotonic_ns) and nothing else -- the figure the line's roofline.avg_launch_ms
    is checked against."""
    import json
    import sqlite3
    import subprocess
    import sys
    db = tmp_path / "run_results.db"
    con = sqlite3.connect(db)
    con.execute("create table kernels (name text, start integer, end integer)")
    rows = [("void stk::k_sweepe<3, 25, 7, 0>(stk::SweepArgs)", t, t + d) for t, d in
            [(100, 5_000_000), (20_000_000, 17_000_000), (40_000_000, 17_200_000), (60_000_000, 16_800_000),
             (90_000_000, 9_000_000)]] + [("stk::k_nuts_step", 38_000_000, 38_100_000)]
    con.executemany("insert into kernels values (?, ?, ?)", rows)
    con.commit()
    con.close()
    line = tmp_path / "bench.json"
    line.write_text(json.dumps({"timed_window_monotonic_ns": [19_000_000, 80_000_000], "steps": 3,
                                "roofline": {"avg_launch_ms": 17.0}}) + "\n")
    out = subprocess.run([sys.executable, "tools/rocpd_summary.py", "window", str(db), "--kernel", "k_sweepe",
                          "--bench-json", str(line)], capture_output=True, text=True, check=True,
                         cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    rec = json.loads(out.stdout.strip().splitlines()[-1])
    assert rec["window_dispatches"] == 3 and rec["dispatches_total"] == 5
    assert abs(rec["window_avg_ms"] - 17.0) < 1e-9


def test_last_run_is_thinned_like_the_returned_draws(monkeypatch):
    """thin > 1: Stark.last_run holds the draws the caller got and their per-draw stats (ADVICE
    r4), ceil(num_samples / thin) per chain."""
    from stark_amd import engine
    from stark_amd import stark as S
    from stark_amd.rdd import LocalContext

    class FakeModel:
        def __init__(self, ctx, family, shards):
            self.n = len(shards)

        def set_prior(self, **kw):
            pass

        def sample(self, **cfg):
            C, S_ = cfg["chains"], cfg["num_samples"]
            draws = [np.arange(19 * C * S_, dtype=float).reshape(19, C * S_) + 1000 * k for k in range(self.n)]
            stats = [np.arange(C * S_, dtype=float)[:, None].repeat(6, 1) for _ in range(self.n)]
            return engine.SampleResult(draws, stats, {"errors": 0}, C, S_)

        def close(self):
            pass

    monkeypatch.setattr(S.engine, "Model", FakeModel)
    monkeypatch.setattr(S.engine, "default_context", lambda *a: None)
    sc = LocalContext()
    school = list(zip([28, 8, -3, 7, -1, 1, 18, 12], [15, 10, 16, 11, 9, 11, 10, 18]))
    st = S.Stark(sc, sc.parallelize(school, 2), prepare_school_data)
    st.setStanModel(file=os.path.join(ROOT, "stark_amd", "models", "schools.stan"))
    out = st._draw_partitions([prepare_school_data(school[:4])], iter=10, warmup=5, chains=2, thin=2, seed=3,
                              permuted=False)
    lr = st.last_run
    assert out[0].shape == (19, 6) and lr.draws[0].shape == (19, 6) and lr.num_samples == 3
    np.testing.assert_array_equal(lr.draws[0], out[0])
    np.testing.assert_array_equal(lr.stats[0][:, 0], [0, 2, 4, 5, 7, 9])
