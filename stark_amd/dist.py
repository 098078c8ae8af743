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
    import torch
    import torch.distributed as dist
    if dist.get_backend() == "nccl":
        import os
        return torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
    return torch.device("cpu")


def all_gather_partitions(local: dict, n_partitions: int):
    """local: {partition index: 2-D float64 array}.  Returns the list over all partitions
    (one all_gather of a padded [slots, rows, cols] fp64 tensor per rank)."""
    rank, ws = world()
    if ws == 1:
        return [local[p] for p in range(n_partitions)]
    import torch
    import torch.distributed as dist
    dev = _device_for_backend()
    shapes = [None] * n_partitions
    for p, a in local.items():
        shapes[p] = a.shape
    # every rank learns every shape (tiny object collective)
    all_shapes = [None] * ws
    dist.all_gather_object(all_shapes, {p: a.shape for p, a in local.items()})
    for d in all_shapes:
        for p, sh in d.items():
            shapes[p] = tuple(sh)
    rmax = max(s[0] for s in shapes)
    cmax = max(s[1] for s in shapes)
    slots = (n_partitions + ws - 1) // ws
    buf = torch.zeros((slots, rmax, cmax), dtype=torch.float64, device=dev)
    for k, p in enumerate(local_partitions(n_partitions, rank, ws)):
        a = torch.as_tensor(np.ascontiguousarray(local[p]), dtype=torch.float64)
        buf[k, : a.shape[0], : a.shape[1]] = a.to(dev)
    out = [torch.empty_like(buf) for _ in range(ws)]
    dist.all_gather(out, buf)
    res = []
    for p in range(n_partitions):
        r, k = p % ws, p // ws
        rr, cc = shapes[p]
        res.append(out[r][k, :rr, :cc].cpu().numpy().copy())
    return res
