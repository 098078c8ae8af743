"""Multi-process path on CPU (gloo, world_size 2): partition placement p % world, the single
all-gather of draw matrices, and the driver's result equal to the 1-process run."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from stark_amd import dist as sdist
        # ragged shapes, 5 partitions over 2 ranks
        shapes = [(3, 4), (5, 4), (2, 4), (3, 6), (1, 1)]
        mine = sdist.local_partitions(len(shapes), rank, world)
        local = {p: np.full(shapes[p], float(p) + 0.5) + np.arange(np.prod(shapes[p])).reshape(shapes[p])
                 for p in mine}
        allp = sdist.all_gather_partitions(local, len(shapes))
        ok = all(a.shape == shapes[p] and np.array_equal(
            a, np.full(shapes[p], float(p) + 0.5) + np.arange(np.prod(shapes[p])).reshape(shapes[p]))
            for p, a in enumerate(allp))
        # as_tensor: equal shapes, ONE [partitions, rows, cols] tensor (the bench's device combine input);
        # local values may be tensors; ragged shapes are refused
        import torch
        eq = {p: torch.full((3, 4), float(p)) + torch.arange(12.).reshape(3, 4) for p in mine}
        t = sdist.all_gather_partitions(eq, len(shapes), as_tensor=True)
        ok = ok and tuple(t.shape) == (5, 3, 4) and t.dtype == torch.float64 and all(
            torch.equal(t[p], torch.full((3, 4), float(p), dtype=torch.float64) + torch.arange(12.).reshape(3, 4))
            for p in range(5))
        try:
            sdist.all_gather_partitions(local, len(shapes), as_tensor=True)
            ok = False
        except ValueError:
            pass
        # driver with a fake sampler: naive mode across ranks
        import pytest as _pt  # noqa: F401
        from test_host import _fake_stark
        mp_ = _pt.MonkeyPatch()
        st = _fake_stark(mp_)
        out = st.distribute(n=3, iter=100, reference_union=True)
        q.put((rank, ok, mine, out))
        mp_.undo()
    finally:
        dist.destroy_process_group()


def test_gloo_world2_gather_and_driver(golden):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort(key=lambda r: r[0])
    assert res[0][2] == [0, 2, 4] and res[1][2] == [1, 3]
    assert all(r[1] for r in res)
    # both ranks hold the same stacked result, equal to the single-process driver
    np.testing.assert_array_equal(res[0][3], res[1][3])
    mpatch = pytest.MonkeyPatch()
    from test_host import _fake_stark
    st = _fake_stark(mpatch)
    np.testing.assert_array_equal(st.distribute(n=3, iter=100, reference_union=True), res[0][3])
    mpatch.undo()


# ---------------------------------------------------------------- full-data mode exchange
def _fulldata_worker(rank, world, port, q):
    """Each rank: oracle lp/grad of ITS rows (fulldata.rank_rows) in the library's block layout
    ([C][Dp] gradients, then [C] log densities), summed by fulldata.sum_over_ranks -- the
    exchange the GPU path runs after every step -- must equal the full-data oracle."""
    import sys
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle as O
        from stark_amd import fulldata
        O.build()
        n, d, C = 1001, 7, 3
        Dp = (d + 1 + 7) // 8 * 8
        X = O.gen_x(5, 0, n, d)
        beta = O.gen_beta(5, d)
        y, _ = O.gen_y_logistic(5, 0, X, 0.0, beta)
        q_ = np.random.default_rng(3).normal(0, 0.3, (C, d + 1))
        off, cnt = fulldata.rank_rows(n, world, rank)
        om = O.Model(O.FAM_LOGREG, X=X[off:off + cnt], y=y[off:off + cnt])
        block = torch.zeros(C * Dp + C, dtype=torch.float64)
        for c in range(C):
            lp, g = om.lpgrad(q_[c])
            block[c * Dp:c * Dp + d + 1] = torch.from_numpy(g)
            block[C * Dp + c] = lp
        fulldata.sum_over_ranks(block)
        full = O.Model(O.FAM_LOGREG, X=X, y=y)
        ok = True
        for c in range(C):
            lp, g = full.lpgrad(q_[c])
            ok &= abs(block[C * Dp + c].item() - lp) <= 1e-12 * abs(lp)
            ok &= bool(np.allclose(block[c * Dp:c * Dp + d + 1].numpy(), g, rtol=1e-12, atol=1e-12 * np.abs(g).max()))
        q.put((rank, ok, (off, cnt)))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_fulldata_exchange():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fulldata_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in procs])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(r[1] for r in res)
    assert res[0][2] == (0, 500) and res[1][2] == (500, 501)


# ---------------------------------------------------------------- bench exchange (ESS / accuracy phase)
def _bench_exchange_worker(rank, world, port, q):
    """bench.py's N-rank tail on gloo: each rank holds 2 of 4 logistic shards (oracle models
    stand in for the GPU gradient), the draw matrices are all-gathered in partition order, and
    the full-data Laplace reference is formed from per-rank gradient sums all-reduced over the
    group -- every rank must take the same Newton steps and end at the single-process MAP."""
    import sys
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle as O
        from stark_amd import dist as sdist
        from tools import laplace as L
        O.build()
        n, d, S = 3000, 5, 4
        X = O.gen_x(9, 0, n * S, d)
        beta = O.gen_beta(9, d)
        y, _ = O.gen_y_logistic(9, 0, X, 0.2, beta)
        mine = list(range(rank * S // world, (rank + 1) * S // world))

        class Shards:
            def __init__(self, ids):
                self.m = [O.Model(O.FAM_LOGREG, X=X[k * n:(k + 1) * n], y=y[k * n:(k + 1) * n]) for k in ids]

            def log_density_grad(self, s, Q):
                out = [self.m[s].lpgrad(qq) for qq in np.atleast_2d(Q)]
                return np.array([o[0] for o in out]), np.array([o[1] for o in out])

        def allreduce(arr):
            t = torch.from_numpy(np.ascontiguousarray(arr))
            dist.all_reduce(t)
            arr[...] = t.numpy()

        local = {k: np.full((3, 8), float(k)) + rank * 0 for k in mine}
        allp = sdist.all_gather_partitions(local, S)
        gathered_ok = all(np.array_equal(allp[k], np.full((3, 8), float(k))) for k in range(S))
        q0 = np.zeros(d + 1)
        sd0 = np.full(d + 1, 0.02)
        m_, c_, info = L.laplace(Shards(mine), list(range(len(mine))), q0, sd0, reduce=allreduce)
        q.put((rank, gathered_ok, m_, c_, info["newton_steps_in_sd"]))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_bench_exchange():
    import sys
    sys.path.insert(0, ROOT)
    from oracle import oracle as O
    from tools import laplace as L
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_exchange_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=180) for _ in procs], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0][1] and res[1][1]
    np.testing.assert_array_equal(res[0][2], res[1][2])           # identical Newton paths on both ranks
    assert res[0][4] == res[1][4]
    # single process, all 4 shards: the same MAP (sums differ only in association order)
    O.build()
    n, d, S = 3000, 5, 4
    X = O.gen_x(9, 0, n * S, d)
    beta = O.gen_beta(9, d)
    y, _ = O.gen_y_logistic(9, 0, X, 0.2, beta)
    full = O.Model(O.FAM_LOGREG, X=X, y=y)

    class One:
        def log_density_grad(self, s, Q):
            out = [full.lpgrad(qq) for qq in np.atleast_2d(Q)]
            return np.array([o[0] for o in out]), np.array([o[1] for o in out])

    m1, c1, _ = L.laplace(One(), [0], np.zeros(d + 1), np.full(d + 1, 0.02))
    sd = np.sqrt(np.diag(c1))
    assert np.abs((res[0][2] - m1) / sd).max() < 1e-6
    np.testing.assert_allclose(res[0][3], c1, rtol=1e-5)
