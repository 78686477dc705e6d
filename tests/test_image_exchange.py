"""CPU, gloo: the cross-GPU replica feed (easydarwin_amd.replica.DistReplicaLink over peer
mailboxes, easydarwin_amd/mailbox.py) with a stand-in engine and POSIX
shared memory in place of device memory + IPC handles (the GPU export/import and the IPC
mapping are tested in tests/test_gpu_replica.py and tests/test_gpu_multiprocess.py).

* the join round (connect: the only collective) brings every requested session's owner a
  mailbox for the requesting rank; every later round (sync) moves each image from its owner to
  each rank that replicates it, intact, full the first time and deltas after, with no
  collective -- the worker makes no torch.distributed call between connect and the end;
* replica feedback (relocations) reaches the owners through the same mailboxes, in lockstep;
* the rehearsal at 2, 4 and 8 ranks reports the per-round cost of the steady-state exchange."""
import hashlib
import os
import socket
import time

import numpy as np
import pytest
import torch.multiprocessing as mp

from easydarwin_amd.dist import owner, subscriber_rank

N_SESS = 24


def _image(g, version):
    """Deterministic stand-in for a session image: length and bytes depend on both."""
    seed = hashlib.sha256(f"{g}:{version}".encode()).digest()
    n = 48 + 16 * (g % 7) + 16 * version
    return np.frombuffer((seed * (n // 32 + 1))[:n], dtype=np.uint8)


class FakeEngine:
    """The engine calls DistReplicaLink makes, host-side: the v-th image of session g sent to a
    rank is _image(g, v) -- v comes back through the link's per-(session, destination) heads
    (IMAGE_FULL the first time, then the heads this export returned) -- and imports are recorded."""

    def __init__(self, rank):
        self.rank = rank
        self.sessions = {}                          # local id -> global id
        self.imported = []                          # (global id, bytes)
        self.relocated = set()                      # local replica ids to report

    def session_add(self, sdp, udp_push=False):
        s = len(self.sessions)
        self.sessions[s] = int(sdp)                 # (the "SDP" is the global id)
        return s

    def senders_of(self, sessions):
        return 2 * len(sessions)

    def session_export(self, local, now_ms, dst=None, cap=0, since=None):
        offs, parts, heads = [0], [], []
        for i, s in enumerate(local):
            h = int(since[2 * i])
            v = 0 if h == 0xFFFFFFFFFFFFFFFF else h       # (heads carry the next version)
            parts.append(_image(self.sessions[s], v))
            offs.append(offs[-1] + len(parts[-1]))
            heads += [v + 1, v + 1]
        blob = np.concatenate(parts) if parts else np.zeros(0, np.uint8)
        assert len(blob) <= cap
        dst[:len(blob)] = blob
        return np.array(offs, np.uint64), np.array(heads, np.uint64)

    def session_import(self, src, offsets, local):
        for i, s in enumerate(local):
            self.imported.append((self.sessions[s], bytes(src[int(offsets[i]):int(offsets[i + 1])])))

    def session_relocations(self, sessions):
        return sorted(s for s in sessions if s in self.relocated)

    def session_key_update(self, sessions):
        pass


def _link_worker(rank, world, port, rounds, out_q):
    try:
        import torch.distributed as dist

        from easydarwin_amd.mailbox import HostRegion
        from easydarwin_amd.replica import DistReplicaLink
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        eng = FakeEngine(rank)
        link = DistReplicaLink(eng, world, rank, lockstep=True, session_bytes=4096, region_cls=HostRegion,
                               timeout_s=60)
        for g in range(N_SESS):
            if owner(g, world) == rank:
                link.own(g, eng.session_add(str(g)))
        # subscribers 0..59 spread over sessions; a rank replicates every session one of its
        # subscribers watches and another rank owns
        subs = [(sub, sub % N_SESS) for sub in range(60)]
        need = sorted({g for sub, g in subs if subscriber_rank(sub, world) == rank and owner(g, world) != rank})
        for g in need:
            link.want(g, str(g))
        link.connect()                                   # the join round: the only collective
        dist.barrier()
        got, times = [], []
        for r in range(rounds):
            eng.imported.clear()
            t0 = time.perf_counter()
            link.sync(1000 * r)
            # replicas relocate the sessions g with g % (rank + 2) == 0 in round 1
            eng.relocated = {link.replica_of[g] for g in need if g % (rank + 2) == 0} if r == 1 else set()
            upd = link.feedback()
            times.append(time.perf_counter() - t0)
            got.append((sorted(eng.imported), upd))
        sent = sum(mb.bytes_moved for mb, _ in link.out.values())
        recv = sum(mb.bytes_moved for mb, _ in link.inbox.values())
        dist.barrier()                                   # (teardown: every peer done reading)
        link.close()
        out_q.put((rank, need, got, sent, recv, times))
        dist.destroy_process_group()
    except Exception as e:          # noqa: BLE001 -- reported to the parent
        out_q.put(("error", rank, repr(e)))
        raise


def _run(world, rounds):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_link_worker, args=(r, world, port, rounds, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    assert all(r[0] != "error" for r in res), res
    assert all(p.exitcode == 0 for p in procs)
    return res


@pytest.mark.parametrize("world", [2, 3])
def test_mailboxes_route_images_and_feedback(world):
    res = _run(world, 3)
    total_sent = total_recv = 0
    reported = {}
    for rank, need, got, sent, recv, _ in res:
        assert need, "every rank should replicate some remote session in this layout"
        for version, (imported, _) in enumerate(got):
            want = sorted((g, bytes(_image(g, version))) for g in need)
            assert imported == want
        reported[rank] = {g for g in need if g % (rank + 2) == 0}
        total_sent += sent
        total_recv += recv
    assert total_sent == total_recv > 0
    # lockstep feedback: round 1's relocations reached their owners in round 1, once
    every = {g for s in reported.values() for g in s}
    for rank, _need, got, _s, _r, _t in res:
        assert got[1][1] == sorted(g for g in every if owner(g, world) == rank)
        assert got[0][1] == [] and got[2][1] == []


@pytest.mark.parametrize("world", [2, 4, 8])
def test_rehearsal_per_round_cost(world):
    """The steady-state exchange at 2 / 4 / 8 ranks (every rank both owner and replica): the
    per-round host time of publish + import + feedback, printed for DESIGN.md §5; bounded so a
    protocol regression (a round waiting out a timeout) fails."""
    rounds = 20
    res = _run(world, rounds)
    per = sorted(np.median(t[3:]) for *_, t in res)
    print(f"\n[mailbox rehearsal] world {world}: per-round median {1e3 * per[len(per) // 2]:.3f} ms, "
          f"max over ranks {1e3 * per[-1]:.3f} ms")
    assert per[-1] < 0.5


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _first_empty(arr):
    p = next((i for i, v in enumerate(arr) if v is None), len(arr))
    if p == len(arr):
        arr.append(None)
    return p


def _places_worker(rank, world, port, out_q):
    import random

    import torch.distributed as dist
    from easydarwin_amd.dist import route_places
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    arrays = {}                                  # owned session -> bucket array (None = empty)

    def join(g):
        a = arrays.setdefault(g, [])
        p = _first_empty(a)
        a[p] = "remote"
        return p

    def leave(g, p):
        assert arrays[g][p] == "remote"
        arrays[g][p] = None

    rng = random.Random(100 + rank)
    held, rounds = [], []
    for rnd in range(4):
        ev = []
        for i in range(12):
            t = 1000 * rnd + rng.randint(0, 999)
            if held and rng.random() < 0.3:
                g, p = held.pop(rng.randrange(len(held)))
                ev.append(("leave", t, g, p))
            else:
                ev.append(("join", t, rng.randrange(N_SESS), (rank, rnd, i)))
        ev.sort(key=lambda e: e[1])
        got = route_places(ev, join, leave, world, rank)
        held += [(e[2], got[e[3]]) for e in ev if e[0] == "join"]
        rounds.append((ev, got))
    out_q.put((rank, rounds))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_remote_places_follow_one_array(world):
    """dist.route_places: replica joins and leaves from every rank, over several rounds, get the places
    one bucket array per session would give them when the events are applied in (time, rank, order)
    -- a single server's AddOutput / RemoveOutput order."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_places_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    arrays, want = {}, {}
    for rnd in range(4):
        merged = sorted((e[1], r, i, e) for r in range(world) for i, e in enumerate(res[r][rnd][0]))
        for _t, r, _i, e in merged:
            a = arrays.setdefault(e[2], [])
            if e[0] == "join":
                p = _first_empty(a)
                a[p] = e[3]
                want[e[3]] = p
            else:
                a[e[3]] = None
    for r in range(world):
        for ev, got in res[r]:
            for e in ev:
                if e[0] == "join":
                    assert got[e[3]] == want[e[3]]
