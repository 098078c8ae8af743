"""Full-data mode: ONE posterior whose rows are split over the GPUs of a node, with the
per-leapfrog gradient summed over ranks (BASELINE.json configs[4]; SURVEY.md 8e "full-data
extension").  The reference has no counterpart -- stark always samples subposteriors
(stark/stark.py:43-56) -- so this mode sits next to the consensus path, not inside it.

Every rank holds rows [offset, offset + count) of the N-row data set as a one-shard model and
runs the SAME chains (same config, same global shard id 0, so the same RNG streams).  After
each state-machine step's local sweep + chunk reduction, the [nchains][Dp] gradient block and
the [nchains] log densities (one contiguous block) are summed over ranks by
``torch.distributed.all_reduce`` -- RCCL over xGMI -- on the library's own HIP stream (the
context is created on torch's current stream, so the kernels and the collective are ordered
without a host sync).  All ranks then run the NUTS step on bitwise-identical inputs, so their
chain states never diverge and no other exchange is needed.

The log density must be a pure sum over rows: the logistic family (flat priors, no Jacobian).
"""
from __future__ import annotations

from . import engine


def rank_rows(n_total: int, world: int, rank: int):
    """Contiguous row range of `rank`: (offset, count), sizes differing by at most one."""
    lo = n_total * rank // world
    hi = n_total * (rank + 1) // world
    return lo, hi - lo


def sum_over_ranks(block, group=None):
    """The per-step exchange: in-place sum of a [grad | lp] block over the ranks of `group`."""
    import torch.distributed as dist
    dist.all_reduce(block, op=dist.ReduceOp.SUM, group=group)
    return block


def context_on_torch_stream(device: int) -> engine.Context:
    """A library context on torch's current stream of `device` (required for the exchange)."""
    import torch
    return engine.Context(device, stream=torch.cuda.current_stream(device).cuda_stream)


class FullDataSampler:
    """NUTS over the full data set, rows split over ranks.

    model: this rank's one-shard logistic model (e.g. Model.synthetic(..., nshards=1,
    rows_per_shard=count, row_offset=offset)); ctx of the model must be on torch's current
    stream when the exchange is active.  group: torch.distributed group (default: WORLD).
    force_exchange: run the all-reduce even with one rank (tests the path on one GPU).
    """

    def __init__(self, model: engine.Model, group=None, force_exchange: bool = False, **cfg):
        if model.family != engine.FAMILIES["logistic"]:
            raise ValueError("full-data mode needs the logistic family (a log density that is a pure sum over rows)")
        if model.nshards != 1:
            raise ValueError("full-data mode: one shard (this rank's rows) per model")
        cfg = dict(cfg)
        cfg["shard_ids"] = [0]          # identical RNG streams on every rank
        self.model = model
        self.sampler = model.sampler(**cfg)
        self.block = None
        import torch.distributed as dist
        world = dist.get_world_size(group) if (dist.is_available() and dist.is_initialized()) else 1
        self.world = world
        if world > 1 or force_exchange:
            import torch
            dev = torch.device("cuda", model.ctx.device)
            if model.ctx.stream != torch.cuda.current_stream(dev).cuda_stream:
                raise ValueError("full-data exchange: create the context with fulldata.context_on_torch_stream()")
            self.block = torch.zeros(self.sampler.grad_block(), dtype=torch.float64, device=dev)
            blk = self.block
            self.sampler.set_allreduce(lambda ptr, count, stream: sum_over_ranks(blk, group), blk.data_ptr())

    def run(self, target_iter=None, max_steps: int = 0):
        self.sampler.run(target_iter, max_steps)
        return self

    def __getattr__(self, name):        # info(), draws(), iterations(), adaptation(), result(), close()
        return getattr(self.sampler, name)
