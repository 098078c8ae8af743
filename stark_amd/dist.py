"""One process per GPU: shard placement and the single exchange of the hot path.

Replaces Spark's executor placement and collect-to-driver (stark/stark.py:65-66, 85).
Partition p runs on rank p % world_size (device LOCAL_RANK); sampling needs no
communication, and at the end every rank's P x S draw matrices are all-gathered in one
collective (torch.distributed: RCCL over xGMI on GPUs, gloo on CPU) so that every rank
holds all shards in partition order and the combine runs in a fixed shard order --
results are bitwise identical on 1 or N GPUs.
"""
from __future__ import annotations

import numpy as np


def world():
    try:
        import torch.distributed as dist
    except Exception:  # pragma: no cover
        return 0, 1
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def local_partitions(n_partitions: int, rank: int, world_size: int):
    return [p for p in range(n_partitions) if p % world_size == rank]


def _device_for_backend():
    """RCCL ('nccl') collectives run on this rank's GPU (LOCAL_RANK); the object collectives
    use torch's CURRENT device, so it is set here too -- otherwise every rank would send on
    cuda:0."""
    import torch
    import torch.distributed as dist
    if dist.get_backend() == "nccl":
        import os
        dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count()))
        torch.cuda.set_device(dev)
        return dev
    return torch.device("cpu")


def all_gather_partitions(local: dict, n_partitions: int, as_tensor: bool = False):
    """local: {partition index: 2-D float64 array or device tensor} -- whatever partitions
    this rank holds (round-robin p % world for the driver, contiguous blocks for bench.py).
    Returns the list over all partitions: one all_gather of a padded [slots, rows, cols] fp64
    tensor per rank, after a tiny object collective that tells every rank who holds which
    partition.

    as_tensor: return ONE [n_partitions, rows, cols] fp64 tensor on this rank's device instead
    (all partitions must share one shape, as the combine requires, stark/stark.py:20): the
    gathered draws stay in HBM and go straight into the device combine (engine.consensus)."""
    rank, ws = world()
    import torch.distributed as _d
    if not (_d.is_available() and _d.is_initialized()):
        if as_tensor:
            import torch
            parts = [torch.as_tensor(local[p], dtype=torch.float64) for p in range(n_partitions)]
            dev = next((t.device for t in parts if t.is_cuda), None)
            if dev is None and torch.cuda.is_available():
                dev = torch.device("cuda", torch.cuda.current_device())
            return torch.stack([t.to(dev) for t in parts]).contiguous()
        return [local[p] for p in range(n_partitions)]
    # an initialised group runs the collective even at world size 1 (same code path as N > 1)
    import torch
    import torch.distributed as dist
    dev = _device_for_backend()      # before the object collective: it sends on the current device
    held = [None] * ws
    dist.all_gather_object(held, {int(p): tuple(int(v) for v in a.shape) for p, a in local.items()})
    where, shapes = {}, {}
    for r, dct in enumerate(held):
        for k, p in enumerate(sorted(dct)):
            where[p] = (r, k)
            shapes[p] = tuple(dct[p])
    missing = [p for p in range(n_partitions) if p not in where]
    if missing:
        raise ValueError(f"partitions {missing} are held by no rank")
    rmax = max(sh[0] for sh in shapes.values())
    cmax = max(sh[1] for sh in shapes.values())
    slots = max(1, max(len(dct) for dct in held))
    buf = torch.zeros((slots, rmax, cmax), dtype=torch.float64, device=dev)
    for k, p in enumerate(sorted(local)):
        a = local[p] if isinstance(local[p], torch.Tensor) else torch.as_tensor(np.ascontiguousarray(local[p]))
        buf[k, : a.shape[0], : a.shape[1]] = a.to(dev, torch.float64)
    out = [torch.empty_like(buf) for _ in range(ws)]
    dist.all_gather(out, buf)
    if as_tensor:
        if len(set(shapes.values())) != 1:
            raise ValueError(f"as_tensor: partitions must share one shape, got {sorted(set(shapes.values()))}")
        rr, cc = shapes[0]
        return torch.stack([out[where[p][0]][where[p][1], :rr, :cc] for p in range(n_partitions)]).contiguous()
    res = []
    for p in range(n_partitions):
        r, k = where[p]
        rr, cc = shapes[p]
        res.append(out[r][k, :rr, :cc].cpu().numpy().copy())
    return res
