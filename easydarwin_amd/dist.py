"""Multi-GPU plumbing for the relay: one process per GPU, sessions sharded by
FNV-1a-64 of the stream ID, no collective on the steady-state data path.  torch.distributed
(RCCL on the GPU box, gloo in CPU tests) brackets the timed region, reduces the results, and
carries the joins of subscribers whose egress GPU is not the stream's owner (BASELINE config
C4): their bucket places (route_places) and the peer-mailbox handles (replica.DistReplicaLink.
connect).  The session images themselves then flow owner -> replica through the mailboxes
(easydarwin_amd/mailbox.py) with no collective."""
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


def reduce_run(elapsed_s: float, counts: list, device=None, force: bool = False):
    """max of elapsed over ranks, sum of counts over ranks (whole-node throughput).  force: run
    the collectives even at world size 1 (exercises the RCCL path on one GPU)."""
    if not (dist.is_available() and dist.is_initialized()) or (dist.get_world_size() == 1 and not force):
        return elapsed_s, list(counts)
    t = torch.tensor([elapsed_s], dtype=torch.float64, device=device)
    c = torch.tensor([float(x) for x in counts], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dist.all_reduce(c, op=dist.ReduceOp.SUM)
    return float(t.item()), [int(round(x)) for x in c.tolist()]


def subscriber_rank(sub_id: int, world: int) -> int:
    """Egress GPU of a subscriber (BASELINE config C4: hash(subID) % nGPU)."""
    return fnv1a64(f"sub{int(sub_id)}") % world


def route_places(events, join_fn, leave_fn, world: int, rank: int):
    """Bucket places of replica subscribers, taken in their owners' bucket arrays
    (ReflectorStream::AddOutput / RemoveOutput, ReflectorStream.cpp:281-336), so that a session's
    subscribers on every GPU are numbered in one array as the reference's one process numbers
    them (edgpu_session_remote_join / _leave).

    events    this rank's replica joins and leaves since the last round, in order:
              ("join", t_ms, global session, key) / ("leave", t_ms, global session, place)
    join_fn   (global session owned here) -> place
    leave_fn  (global session owned here, place) -> None

    Every owner applies all ranks' events on its sessions in (time, rank, order) -- the order a
    single server would have seen them in.  Collective (two all_gather_object rounds of a few
    integers).  Returns {key: place} for this rank's joins."""
    lists = [None] * world
    dist.all_gather_object(lists, [tuple(e) for e in events])
    merged = sorted((e[1], r, i, e) for r, lst in enumerate(lists) for i, e in enumerate(lst)
                    if owner(e[2], world) == rank)
    given = {}
    for _t, r, _i, e in merged:
        if e[0] == "join":
            given.setdefault(r, {})[e[3]] = int(join_fn(e[2]))
        else:
            leave_fn(e[2], int(e[3]))
    answers = [None] * world
    dist.all_gather_object(answers, given)
    out = {}
    for a in answers:
        out.update(a.get(rank, {}))
    return out
