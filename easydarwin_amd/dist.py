"""Multi-GPU plumbing for the relay: one process per GPU, sessions sharded by
FNV-1a-64 of the stream ID, no collective on the steady-state data path.  torch.distributed
(RCCL on the GPU box, gloo in CPU tests) brackets the timed region, reduces the results, and
carries the one real exchange: session images for subscribers whose egress GPU is not the
stream's owner (exchange_images, BASELINE config C4)."""
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


def exchange_images(requests, export_fn, import_fn, make_buf, world: int, rank: int):
    """One round of the only cross-GPU exchange on the path: session images
    from their owners to the ranks that serve replicas of them.

    requests   global sessions this rank needs images of this round (owned elsewhere)
    export_fn  (sessions, dst_rank) -> (uint8 tensor, offsets[n+1]); images of `sessions`,
               owned here, for `dst_rank` (full the first time, deltas afterwards)
    import_fn  (tensor, offsets, sessions, src_rank) -> None
    make_buf   nbytes -> uint8 tensor on the communication device

    Control metadata (which sessions, image offsets) goes through all_gather_object; the
    image bytes go point-to-point in one batch_isend_irecv group (ncclGroupStart/End with
    ncclSend/ncclRecv pairs under RCCL).  Returns (bytes sent, bytes received)."""
    reqs = [None] * world
    dist.all_gather_object(reqs, sorted(int(g) for g in requests))
    outgoing = {}
    for r in range(world):
        if r == rank:
            continue
        mine = [g for g in reqs[r] if owner(g, world) == rank]
        if mine:
            buf, offs = export_fn(mine, r)
            outgoing[r] = (mine, buf, [int(x) for x in offs])
    meta = [None] * world
    dist.all_gather_object(meta, {r: (m, offs) for r, (m, _, offs) in outgoing.items()})
    incoming = {}
    for src in range(world):
        if src != rank and rank in meta[src]:
            sess, offs = meta[src][rank]
            incoming[src] = (sess, offs, make_buf(max(offs[-1], 1)))
    ops = []
    for r, (_, buf, offs) in sorted(outgoing.items()):
        if offs[-1]:
            ops.append(dist.P2POp(dist.isend, buf[:offs[-1]], r))
    for src, (_, offs, buf) in sorted(incoming.items()):
        if offs[-1]:
            ops.append(dist.P2POp(dist.irecv, buf[:offs[-1]], src))
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()
    for src, (sess, offs, buf) in sorted(incoming.items()):
        import_fn(buf, offs, sess, src)
    sent = sum(o[-1] for _, _, o in outgoing.values())
    recv = sum(o[-1] for _, o, _ in incoming.values())
    return sent, recv


def route_relocations(relocated, key_update_fn, world: int, rank: int):
    """The replicas' feedback to the owners: a relocation on a replica (Q9,
    ReflectorSender::NeedRelocateBookMark -> ReflectorSession::SetHasVideoKeyFrameUpdate,
    ReflectorStream.cpp:1311-1317) must set the owner's flag before the owner's next keyframe
    index, so the session's next audio packet becomes its audio key pointer (:1913-1930).

    relocated      global sessions this rank's replicas relocated an output of (since the last call)
    key_update_fn  (global sessions owned here) -> None; sets their flag (edgpu_session_key_update)

    Collective (all_gather_object of a few integers).  Returns the owned sessions updated."""
    lists = [None] * world
    dist.all_gather_object(lists, sorted(int(g) for g in relocated))
    mine = sorted({g for lst in lists for g in lst if owner(g, world) == rank})
    if mine:
        key_update_fn(mine)
    return mine


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
