"""Generate golden fixtures by running the REFERENCE's own code (not a restatement).

Run in the build container (where /root/reference exists):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

``stark/stark.py`` imports pyspark and pystan at module top (stark/stark.py:1-4); neither
is installed, so both are stubbed in ``sys.modules`` before ``from stark import stark``
(SURVEY.md section 8c).  Only the pure-numpy parts run: ``consensus_avg`` (:7-21), the
driver solve of ``concensusWeight`` (:66-70, driven through a stub RDD), and the
per-partition closure ``_mcmc.w`` (:43-56, driven through a stub StanModel whose fit
returns fixed draws).  Outputs are plain arrays in ``tests/golden/*.npz``; the reference
source never leaves /root/reference.
"""
import collections
import os
import pickle
import sys
import types

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def _import_reference():
    for name in ("pyspark", "pystan"):
        sys.modules[name] = types.ModuleType(name)
    sys.modules["pyspark"].SparkContext = object
    sys.modules["pyspark"].SparkConf = object
    sys.modules["pyspark"].SparkFiles = object
    sys.modules["pystan"].StanModel = FakeStanModel
    sys.path.insert(0, REF)
    from stark import stark  # noqa: E402
    stark.StanModel = FakeStanModel
    return stark


class FakeFit:
    def __init__(self, od):
        self._od = od

    def extract(self):
        return self._od


class FakeStanModel:
    """Stands in for pystan.StanModel: sampling() returns draws that depend only on the
    data dict and the seed, shaped like pystan 2's extract(): mu (S,), tau (S,),
    eta (S,J), theta (S,J), lp__ (S,)."""

    def __init__(self, **kwargs):
        self.kwargs = kwargs

    def sampling(self, data, pars=None, include=True, **kw):
        """pars / include as pystan 2 applies them to extract(): the named parameters in the
        given order (include=True) or all others in model order (include=False), lp__ last."""
        fit = self._sampling(data, **kw)
        if pars is None:
            return fit
        od = fit.extract()
        pars = [pars] if isinstance(pars, str) else list(pars)
        keep = [p for p in pars if p != "lp__"] if include else [k for k in od if k not in pars and k != "lp__"]
        return FakeFit(collections.OrderedDict([(k, od[k]) for k in keep] + [("lp__", od["lp__"])]))

    def _sampling(self, data, **kw):
        J = data["J"]
        S = kw["iter"] // 2 * kw.get("chains", 1)
        seed = int(abs(sum(data["y"]) * 1000 + sum(data["sigma"]))) % (2**32)
        rng = np.random.default_rng(seed)
        mu = rng.normal(8, 5, S)
        tau = np.exp(rng.normal(1.5, 1.0, S))
        eta = rng.normal(0, 1, (S, J))
        theta = mu[:, None] + tau[:, None] * eta
        lp = rng.normal(-40, 3, S)
        return FakeFit(collections.OrderedDict(
            [("mu", mu), ("tau", tau), ("eta", eta), ("theta", theta), ("lp__", lp)]))


class StubRDD:
    """Spark RDD semantics the reference relies on (PySpark, third-party): contiguous
    parallelize slicing, mapPartitions, reduce in partition order, coalesce, union."""

    def __init__(self, parts):
        self.parts = [list(p) for p in parts]

    @classmethod
    def parallelize(cls, data, k):
        data = list(data)
        n = len(data)
        return cls([data[i * n // k:(i + 1) * n // k] for i in range(k)])

    def getNumPartitions(self):
        return len(self.parts)

    def mapPartitions(self, f):
        return StubRDD([list(f(iter(p))) for p in self.parts])

    def reduce(self, f):
        import functools
        vals = [v for p in self.parts for v in p]
        return functools.reduce(f, vals)

    def coalesce(self, n):
        assert n == 1
        return StubRDD([[v for p in self.parts for v in p]])

    def union(self, other):
        return StubRDD(self.parts + other.parts)


def spd_draws(rng, P, S, cond_scale=1.0):
    A = rng.normal(size=(P, P)) / np.sqrt(P)
    L = np.linalg.cholesky(A @ A.T + 0.5 * np.eye(P)) * cond_scale
    mean = rng.normal(size=(P, 1))
    return mean + L @ rng.normal(size=(P, S))


def main():
    stark = _import_reference()
    rng = np.random.default_rng(20240601)

    # ---- consensus_avg (stark/stark.py:7-21) + driver solve (:66-70), two shards
    combine = {}
    for P, S in ((11, 400), (53, 200), (102, 160)):
        f1 = spd_draws(rng, P, S)
        f2 = spd_draws(rng, P, S, 1.3)
        red = stark.consensus_avg(2)(f1, f2)
        final = np.dot(np.linalg.inv(red[0]), red[1])
        combine[f"P{P}_f1"] = f1
        combine[f"P{P}_f2"] = f2
        combine[f"P{P}_sumW"] = red[0]
        combine[f"P{P}_sumWtheta"] = red[1]
        combine[f"P{P}_final"] = final
    # NaN guard (:9-10): NaN in f1 returns f2 unchanged
    f1 = spd_draws(rng, 11, 50)
    f1[3, 7] = np.nan
    f2 = spd_draws(rng, 11, 50)
    combine["nan_f1"] = f1
    combine["nan_f2"] = f2
    combine["nan_out"] = stark.consensus_avg(2)(f1, f2)
    # rank-deficient sample covariances (S - 1 < P): what the reference's np.linalg.inv does
    # with them (LAPACK LU: it raises only on an exactly zero pivot)
    for P, S in ((11, 6), (30, 12)):
        f1 = spd_draws(rng, P, S)
        f2 = spd_draws(rng, P, S, 1.3)
        combine[f"rankdef_P{P}_f1"] = f1
        combine[f"rankdef_P{P}_f2"] = f2
        try:
            red = stark.consensus_avg(2)(f1, f2)
            final = np.dot(np.linalg.inv(red[0]), red[1])
            combine[f"rankdef_P{P}_raised"] = np.array(0)
            combine[f"rankdef_P{P}_final"] = final
            combine[f"rankdef_P{P}_cond_sumW"] = np.array(np.linalg.cond(red[0]))
        except np.linalg.LinAlgError:
            combine[f"rankdef_P{P}_raised"] = np.array(1)
    np.savez_compressed(os.path.join(OUT, "combine_ref.npz"), **combine)

    # ---- concatenate_samples (:23-24)
    a = rng.normal(size=(11, 30))
    b = rng.normal(size=(19, 30))
    np.savez_compressed(os.path.join(OUT, "concat_ref.npz"), a=a, b=b, out=stark.concatenate_samples(a, b))

    # ---- Stark driver through stubs: _mcmc.w (:43-56), concensusWeight (:59-71), distribute (:73-85)
    school = list(zip([28, 8, -3, 7, -1, 1, 18, 12], [15, 10, 16, 11, 9, 11, 10, 18]))  # example/stark_ex.py:4-6

    def prepare(data):          # example/stark_ex.py:8-11
        return {"J": len(data), "y": [d[0] for d in data], "sigma": [d[1] for d in data]}

    rdd = StubRDD.parallelize(school, 2)
    st = stark.Stark(None, rdd, prepare)
    st.setStanModel(model_code="fake")
    w = st._mcmc(prepare, iter=2000, chains=1, n_jobs=1)
    part0 = w(iter(rdd.parts[0]))[0]
    weighted = st.concensusWeight(iter=600)
    naive = st.distribute(n=4, iter=200)
    driver = dict(part0=part0, weighted=weighted, naive=naive)
    # pystan 2 parameter selection forwarded through **kwargs (stark/stark.py:48): fewer rows reach
    # the P x S matrix, and so the combine
    driver["weighted_pars"] = st.concensusWeight(iter=600, pars=["eta", "mu"])
    driver["naive_exclude"] = st.distribute(n=4, iter=200, pars=["theta", "tau"], include=False)
    # the inputs the fake sampler saw, so tests can rebuild them without the reference
    for k, part in enumerate(rdd.parts):
        fit = FakeStanModel().sampling(prepare(part), iter=600, chains=1)
        for name, arr in fit.extract().items():
            driver[f"w600_part{k}_{name}"] = arr
    np.savez_compressed(os.path.join(OUT, "driver_ref.npz"), **driver)
    print("wrote", sorted(os.listdir(OUT)))


if __name__ == "__main__":
    main()
