"""CPU, gloo: the cross-GPU image exchange (easydarwin_amd.dist.exchange_images, SURVEY.md
§8.e / C4) routes each requested session's image from its owner to the requesting rank,
intact, over batched point-to-point send/recv -- with a stand-in image source (the GPU
export/import is tested in tests/test_gpu_replica.py)."""
import hashlib
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from easydarwin_amd.dist import owner, subscriber_rank

N_SESS = 24


def _image(g, dst, version):
    """Deterministic stand-in for a session image: length and bytes depend on all three."""
    seed = hashlib.sha256(f"{g}:{dst}:{version}".encode()).digest()
    n = 48 + 16 * (g % 7) + 16 * version
    return np.frombuffer((seed * (n // 32 + 1))[:n], dtype=np.uint8)


def _worker(rank, world, port, out_q):
    import torch.distributed as dist
    from easydarwin_amd.dist import exchange_images
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    versions = {}                                   # (session, dst) -> images shipped so far
    got = []

    def export_fn(sessions, dst):
        parts, offs = [], [0]
        for g in sessions:
            assert owner(g, world) == rank
            v = versions.get((g, dst), 0)
            versions[(g, dst)] = v + 1
            parts.append(_image(g, dst, v))
            offs.append(offs[-1] + len(parts[-1]))
        return torch.from_numpy(np.concatenate(parts)), offs

    def import_fn(buf, offs, sessions, src):
        for i, g in enumerate(sessions):
            got.append((g, src, bytes(buf[offs[i]:offs[i + 1]].numpy())))

    # subscribers 0..59 spread over sessions; a rank needs every session one of its
    # subscribers watches and another rank owns
    subs = [(sub, sub % N_SESS) for sub in range(60)]
    need = sorted({g for sub, g in subs if subscriber_rank(sub, world) == rank and owner(g, world) != rank})
    rounds = []
    for r in range(2):                              # join burst, then one delta round
        got.clear()
        sent, recv = exchange_images(need, export_fn, import_fn,
                                     lambda n: torch.empty(n, dtype=torch.uint8), world, rank)
        rounds.append((sorted(got), sent, recv))
    out_q.put((rank, need, rounds))
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2, 3])
def test_exchange_routes_images(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    total_sent = total_recv = 0
    for rank, need, rounds in res:
        assert need, "every rank should need some remote session in this layout"
        for version, (got, sent, recv) in enumerate(rounds):
            want = sorted((g, owner(g, world), bytes(_image(g, rank, version))) for g in need)
            assert got == want
            total_sent += sent
            total_recv += recv
    assert total_sent == total_recv > 0


def _reloc_worker(rank, world, port, out_q):
    import torch.distributed as dist
    from easydarwin_amd.dist import route_relocations
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    got = []
    # rank r's replicas relocated outputs of the sessions g with g % (r + 2) == 0 it does not own
    mine = [g for g in range(N_SESS) if g % (rank + 2) == 0 and owner(g, world) != rank]
    upd = route_relocations(mine, got.extend, world, rank)
    out_q.put((rank, mine, upd, sorted(got)))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_relocations_reach_the_owners(world):
    """Replica feedback (dist.route_relocations): every relocation a rank's replica reports
    reaches the session's owner once, and nothing else is updated."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_reloc_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {r: (m, u, g) for r, m, u, g in (q.get(timeout=120) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
    reported = {g for m, _, _ in res.values() for g in m}
    for r, (_, upd, got) in res.items():
        want = sorted(g for g in reported if owner(g, world) == r)
        assert upd == want and got == want


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
