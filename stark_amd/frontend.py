"""Stan-program front end for ``Stark.setStanModel`` (stark/stark.py:37-39).

The reference compiles any Stan program with pystan (``StanModel(**kwargs)``).  This build
has no Stan compiler: it recognises the program as one of the fixed model families whose
log density and gradient are hand-written gfx950 kernels, and raises
``NotImplementedError`` for anything else.  Recognition works on a normalised token
stream (comments and whitespace removed, old ``real y[J]`` and new ``array[J] real y``
declarations both accepted), so formatting does not matter; an explicit ``family=``
keyword overrides it.
"""
from __future__ import annotations

import re

import numpy as np


def _strip(code: str) -> str:
    code = re.sub(r"/\*.*?\*/", " ", code, flags=re.S)
    code = re.sub(r"//[^\n]*", " ", code)
    code = re.sub(r"#[^\n]*", " ", code)
    code = re.sub(r"\s+", " ", code)
    code = re.sub(r"\s*([{}()\[\];,<>=~*+\-:/])\s*", r"\1", code)
    return code.strip()


def _blocks(code: str) -> dict:
    out = {}
    i = 0
    while i < len(code):
        m = re.compile(r"(functions|transformed data|data|transformed parameters|parameters|model|generated quantities)\{").match(code, i)
        if not m:
            i += 1
            continue
        depth, j = 1, m.end()
        while j < len(code) and depth:
            depth += {"{": 1, "}": -1}.get(code[j], 0)
            j += 1
        out[m.group(1)] = code[m.end():j - 1]
        i = j
    return out


def _decl(block: str, pattern: str) -> bool:
    return re.search(pattern, block) is not None


def _stmts(block: str) -> list:
    return [s for s in block.split(";") if s]


_NUM = r"([0-9]+(?:\.[0-9]*)?(?:[eE][-+]?[0-9]+)?|\.[0-9]+(?:[eE][-+]?[0-9]+)?)"
_PRIOR = re.compile(r"(alpha|beta)~normal\(0(?:\.0*)?," + _NUM + r"\)$")


def _split_priors(stmts):
    """Separate `alpha ~ normal(0, s)` / `beta ~ normal(0, s)` statements (s > 0) from the rest."""
    priors, rest = {}, []
    for st in stmts:
        m = _PRIOR.match(st)
        if m and float(m.group(2)) > 0 and m.group(1) not in priors:
            priors[m.group(1)] = float(m.group(2))
        else:
            rest.append(st)
    return priors, rest


def program_info(model_code: str):
    """(family, priors) of a supported Stan program; priors = {'alpha': s, 'beta': s} for the
    regressions' optional `alpha ~ normal(0, s)` / `beta ~ normal(0, s)` statements (absent: flat)."""
    code = _strip(model_code)
    b = _blocks(code)
    priors, rest = _split_priors(_stmts(b.get("model", "")))
    fam = _recognise_blocks(b, sorted(rest))
    if fam == "schools" and priors:
        fam = None
    if fam is None:
        raise NotImplementedError(
            "stark_amd runs a fixed set of model families on the GPU (8 schools, Bayesian linear and logistic "
            "regression with flat or normal(0, s) priors on alpha and beta; see stark_amd/models/*.stan).  This "
            "Stan program is not one of them; pass family='schools'|'linear'|'logistic' if it is an equivalent "
            "program.")
    return fam, priors


def recognise(model_code: str) -> str:
    """Return 'schools', 'linear' or 'logistic' for a supported Stan program."""
    return program_info(model_code)[0]


def _recognise_blocks(b: dict, stm: list):
    params = b.get("parameters", "")
    tp = b.get("transformed parameters", "")
    # 8 schools, non-centred (example/schools.stan:1-18)
    if (_decl(params, r"(^|;)real mu(;|$)") and _decl(params, r"real<lower=0>tau") and
            _decl(params, r"(real eta\[J\]|vector\[J\]eta|array\[J\]real eta)")):
        theta_ok = (re.search(r"theta\[j\]=mu\+tau\*eta\[j\]", tp) or re.search(r"theta=mu\+tau\*eta", tp))
        want = sorted(["eta~normal(0,1)", "y~normal(theta,sigma)"])
        want2 = sorted(["eta~std_normal()", "y~normal(theta,sigma)"])
        if theta_ok and stm in (want, want2):
            return "schools"
    if _decl(params, r"(^|;)real alpha(;|$)") and _decl(params, r"vector\[K\]beta"):
        if stm in (["y~bernoulli_logit(alpha+x*beta)"], ["y~bernoulli_logit(x*beta+alpha)"]):
            if not _decl(params, r"sigma"):
                return "logistic"
        if stm in (["y~normal(alpha+x*beta,sigma)"], ["y~normal(x*beta+alpha,sigma)"]):
            if _decl(params, r"real<lower=0>sigma"):
                return "linear"
    return None


def load_program_info(file=None, model_code=None, family=None, priors=None, **_ignored):
    """Mirror of pystan.StanModel(file=..., model_code=...) argument handling -> (family, priors).
    family= (and priors={'alpha': s, 'beta': s}) override recognition."""
    if family is not None:
        if family not in ("schools", "linear", "logistic"):
            raise ValueError(f"unknown family {family!r}")
        return family, dict(priors or {})
    if model_code is None:
        if file is None:
            raise ValueError("Either file or model_code must be given (pystan.StanModel)")
        with open(file) as f:
            model_code = f.read()
    return program_info(model_code)


def load_program(file=None, model_code=None, family=None, **kw):
    """The family of the program (stark/stark.py:37-39 setStanModel)."""
    return load_program_info(file=file, model_code=model_code, family=family, **kw)[0]


def pack_data(family: str, data: dict) -> dict:
    """Validate a Stan data dict (the prepare_data_callback output, example/stark_ex.py:8-11)
    and turn it into a shard for stk_model_create."""
    if family == "schools":
        J = int(data["J"])
        y = np.asarray(data["y"], np.float64).reshape(-1)
        s = np.asarray(data["sigma"], np.float64).reshape(-1)
        if y.shape[0] != J or s.shape[0] != J:
            raise ValueError(f"schools data: J = {J} but len(y) = {y.shape[0]}, len(sigma) = {s.shape[0]}")
        if np.any(s <= 0):
            raise ValueError("schools data: sigma must be positive (real<lower=0> sigma[J])")
        return {"y": y, "sigma": s}
    N, K = int(data["N"]), int(data["K"])
    x = np.asarray(data["x"], np.float64).reshape(N, K)
    if family == "logistic":
        y = np.asarray(data["y"]).reshape(-1)
        if y.shape[0] != N:
            raise ValueError("y must have N entries")
        # int<lower=0, upper=1> y[N]: pystan rejects non-integer or out-of-range values
        yf = y.astype(np.float64)
        if not np.all(yf == np.round(yf)) or np.any((yf != 0) & (yf != 1)):
            raise ValueError("bernoulli_logit data: y must hold the integers 0 and 1")
        return {"x": x, "y": yf.astype(np.int32)}
    y = np.asarray(data["y"], np.float64).reshape(-1)
    if y.shape[0] != N:
        raise ValueError("y must have N entries")
    return {"x": x, "y": y}


def column_names(family: str, data: dict) -> list:
    """extract() key order flattened to rows of the P x S draw matrix (stark/stark.py:49-56)."""
    if family == "schools":
        J = int(data["J"])
        return (["mu", "tau"] + [f"eta[{j}]" for j in range(1, J + 1)] + [f"theta[{j}]" for j in range(1, J + 1)]
                + ["lp__"])
    K = int(data["K"])
    cols = ["alpha"] + [f"beta[{k}]" for k in range(1, K + 1)]
    if family == "linear":
        cols.append("sigma")
    return cols + ["lp__"]


def param_rows(family: str, data: dict) -> "dict[str, list[int]]":
    """extract() keys in model order (parameters, transformed parameters, lp__) -> their rows
    in the P x S draw matrix (stark/stark.py:49-56 flattens each key to consecutive rows)."""
    groups, row = {}, 0
    for name in column_names(family, data):
        key = name.split("[")[0]
        groups.setdefault(key, []).append(row)
        row += 1
    return groups


def select_pars(family: str, data: dict, pars=None, include: bool = True) -> "list[int] | None":
    """pystan 2 ``sampling(pars=..., include=...)`` (forwarded by stark/stark.py:48 **kwargs):
    the rows that ``fit.extract()`` then returns, in its key order.  pars names the parameters
    to keep (include=True, in the given order) or to drop (include=False, model order kept);
    lp__ is always returned, last, once (an explicit 'lp__' in pars is that same row).  Unknown
    names raise ValueError as pystan does.  None: all rows (no selection).
    Parity UNPINNED against pystan itself: pystan is not importable here, and the golden fixture
    (tests/golden/make_golden.py, FakeStanModel) encodes this same reading of pystan 2's
    extract() order, so the driver test pins the reshape, not the selection order."""
    if pars is None:
        return None
    if isinstance(pars, str):
        pars = [pars]
    pars = list(pars)
    groups = param_rows(family, data)
    for p in pars:
        if p not in groups:
            raise ValueError(f"No parameter {p}")
    if include:
        keep = list(dict.fromkeys(p for p in pars if p != "lp__"))
    else:
        keep = [k for k in groups if k not in pars and k != "lp__"]
    keep.append("lp__")
    return [r for k in keep for r in groups[k]]

