"""Multi-GPU plumbing for the relay: one process per GPU, sessions sharded by
FNV-1a-64 of the stream ID, no collective on the data path.  torch.distributed (RCCL on the
GPU box, gloo in CPU tests) only brackets the timed region and reduces the results."""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

from .workload import fnv1a64, stream_id


def owner(global_session: int, world: int) -> int:
    return fnv1a64(stream_id(global_session)) % world


def env_world():
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def reduce_run(elapsed_s: float, counts: list, device=None):
    """max of elapsed over ranks, sum of counts over ranks (whole-node throughput)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return elapsed_s, list(counts)
    t = torch.tensor([elapsed_s], dtype=torch.float64, device=device)
    c = torch.tensor([float(x) for x in counts], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dist.all_reduce(c, op=dist.ReduceOp.SUM)
    return float(t.item()), [int(round(x)) for x in c.tolist()]
