"""GPU, two engine processes (torch.distributed over gloo, world size 2, one MI355X): the
multi-GPU path of SURVEY.md §8.e executed by libedgpu in separate processes, as the driver's
8-GPU run executes it -- one process per GPU, each with its own engine context.

* Sharding: each process owns the sessions whose FNV-1a-64 stream-ID hash names its rank
  (dist.owner), replays its shard of a multi-session trace through the engine, and the union of
  the two captures is the reference capture (relay_model, pinned to the reference).
* Exchange: one process owns every session (ingest + owner ticks), the other serves every
  subscriber from replica sessions kept in step by session images (DistReplicaLink: full image
  first, deltas after) that the owner exports into peer mailboxes in its HBM and the replica's
  GPU imports straight out of them through IPC mappings -- the only collectives are the join
  rounds (mailbox handles, bucket places); the subscribers' bytes equal the reference
  reflector's capture.  With two or more GPUs visible the processes take GPUs 0 and 1 (the
  images cross over xGMI, the control plane over RCCL); on a one-GPU box both share GPU 0 (the
  same IPC mappings within one device, the control plane over gloo).
"""
import hashlib
import json
import os
import socket
import subprocess
import tempfile

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port, backend="gloo"):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if backend == "nccl":
        torch.cuda.set_device(rank)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", rank))
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    return dist


def _gpus():
    import torch
    return torch.cuda.device_count()          # counts devices without initialising the GPU


def _shard_worker(rank, world, port, n_sess, out_q):
    try:
        dist = _init(rank, world, port)
        from easydarwin_amd.dist import owner
        from easydarwin_amd.replay import replay
        from easydarwin_amd.trace import capture_summary, read_capture
        from test_multi_rank import _trace
        mine = [g for g in range(n_sess) if owner(g, world) == rank]
        cap, _ = replay(_trace(mine), device=0)
        summ = capture_summary(read_capture(cap))
        got = [None] * world
        dist.all_gather_object(got, (mine, summ))
        if rank == 0:
            out_q.put(got)
        dist.destroy_process_group()
    except Exception as e:          # noqa: BLE001 -- reported to the parent
        out_q.put(("error", rank, repr(e)))
        raise


@pytest.mark.gpu
def test_two_engine_processes_shard_sessions(oracle_bins):
    from test_multi_rank import N_SESS, _capture
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_shard_worker, args=(r, 2, port, N_SESS, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
    assert got[0] != "error", got
    assert all(p.exitcode == 0 for p in procs)
    owned = [set(m) for m, _ in got]
    assert owned[0] and owned[1] and not (owned[0] & owned[1]) and owned[0] | owned[1] == set(range(N_SESS))
    merged = {}
    for _, part in got:
        assert not (merged.keys() & part.keys())
        merged.update(part)
    assert merged == _capture(list(range(N_SESS)), oracle_bins["port"])


def _exchange_worker(rank, world, port, name, pull, out_q):
    """rank 0: owner of every session of the scenario; rank 1: every subscriber, on replicas.
    Two GPUs: rank r on GPU r, images over RCCL; one GPU: both on GPU 0, images over gloo."""
    try:
        cross = _gpus() >= world
        dist = _init(rank, world, port, "nccl" if cross else "gloo")
        import numpy as np
        from easydarwin_amd import edgpu
        from easydarwin_amd.dist import owner
        from easydarwin_amd.replay import _wire_images
        from easydarwin_amd.replica import DistReplicaLink
        from easydarwin_amd.trace import JOIN, PKT, TICK, rr_ssrc
        from test_gpu_parity import _trace
        tr = _trace(name)
        # global ids whose FNV-1a owner is rank 0, one per trace session
        gid = [g for g in range(10_000) if owner(g, world) == 0][:len(tr.sdps)]
        with edgpu.Context(device=rank if cross else 0) as ctx:
            link = DistReplicaLink(ctx, world, rank, pull=pull)
            local = {}
            if rank == 0:
                for s, sdp in enumerate(tr.sdps):
                    local[s] = ctx.session_add(sdp)
                    link.own(gid[s], local[s])
                    for t in range(ctx.session_tracks(local[s])):
                        ctx.source_identity(local[s], t, rr_ssrc(s * 16 + t), 0)
            pending, joins, images, meta, places = [], [], {}, {}, {}
            for ev in tr.events:
                if ev[0] == PKT and rank == 0:
                    pending.append((local[ev[2]], ev[3], ev[1], ev[4]))
                elif ev[0] == JOIN:
                    joins.append(ev)                         # (both ranks see the trace's joins)
                elif ev[0] == TICK:
                    t = ev[1]
                    if rank == 0:
                        if pending:
                            desc, so, ss, blob = edgpu.build_batch(pending)
                            ctx.ingest_host(desc, so, ss, blob)
                            ctx.keyframe_index()
                            pending = []
                        ctx.fanout(t)                        # the owner ticks (no subscribers)
                    elif joins:
                        for j in joins:                      # a replica before the sync that fills it
                            if gid[j[2]] not in link.replica_of:
                                local[j[2]] = link.want(gid[j[2]], tr.sdps[j[2]])
                    if joins:
                        link.connect()                       # join round (collective): mailbox handles
                    link.sync(t)                             # no collective: images owner -> replica
                    if joins:
                        # join round (collective): the joiners' bucket places, taken in the owner's arrays
                        given = link.places([("join", j[1], gid[j[2]], int(j[3])) for j in joins] if rank == 1 else [])
                    if rank == 0:
                        joins = []
                    else:
                        for j in joins:
                            h = ctx.subscriber_add(local[j[2]], edgpu.TRANSPORT_TCP if j[4] else edgpu.TRANSPORT_UDP)
                            ctx.subscriber_set_slot(h, given[int(j[3])])
                            places[int(j[3])] = given[int(j[3])]
                            meta[h] = (j[3], j[2], j[4])
                            for tk in range(ctx.session_tracks(local[j[2]])):
                                for k in (0, 1):
                                    images[(0, h, tk, k)] = []
                        joins = []
                        st, subs, desc, arena = ctx.read_tick(ctx.fanout(t))
                        _wire_images(subs, desc, arena, images)
            result = None
            if rank == 1:
                import struct
                recs = sorted((meta[h][0], meta[h][1], tk, k, meta[h][2], len(p), b"".join(p))
                              for (_, h, tk, k), p in images.items())
                out = [b"EDCP", struct.pack("<I", len(recs))]
                for sub_id, s, tk, k, tcp, n, data in recs:
                    out.append(struct.pack("<IIHBBQQ", sub_id, s, tk, k, tcp, n, len(data)))
                    out.append(data)
                result = (hashlib.sha256(b"".join(out)).hexdigest(), link.bytes_received, places)
            else:
                result = link.bytes_sent
            got = [None] * world
            dist.all_gather_object(got, (result, cross))
            link.close()                             # (after the gather: the replica is done reading)
            if rank == 0:
                out_q.put(got)
        dist.destroy_process_group()
    except Exception as e:          # noqa: BLE001
        out_q.put(("error", rank, repr(e)))
        raise


@pytest.mark.gpu
@pytest.mark.parametrize("pull", ["copy", "direct"])
@pytest.mark.parametrize("name", ["c1", "mixed"])
def test_session_images_move_between_engine_processes(name, pull):
    """pull="copy": the replica brings each publication over with one peer DMA copy, then imports;
    "direct": its import kernel reads the owner's mapped HBM."""
    with open(os.path.join(GOLD, name + ".json")) as f:
        fix = json.load(f)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_exchange_worker, args=(r, 2, port, name, pull, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
    assert got[0] != "error", got
    assert all(p.exitcode == 0 for p in procs)
    (sent, cross), ((digest, received, places), _) = got[0], got[1]
    assert cross == (_gpus() >= 2)
    assert sent == received > 0
    assert digest == fix["capture_sha256"]
    # every join's bucket place came from the owner process: AddOutput's first empty place, in
    # join order per session (no LEAVE in these traces)
    from easydarwin_amd.trace import JOIN
    from test_gpu_parity import _trace
    n, want = {}, {}
    for ev in _trace(name).events:
        if ev[0] == JOIN:
            want[ev[3]] = n.get(ev[2], 0)
            n[ev[2]] = want[ev[3]] + 1
    assert places == want
