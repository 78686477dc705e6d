"""CPU, world_size 2 over gloo: the stream-hash sharding of the multi-GPU path is output
invariant (the union of per-rank sub-stream outputs equals the single-rank output, computed
with the oracle), partitions the sessions, and the bench's reduction is max-time / sum-count."""
import os
import socket
import subprocess
import tempfile

import numpy as np
import pytest
import torch.multiprocessing as mp

from easydarwin_amd.dist import owner, reduce_run
from easydarwin_amd.synth import TrackSpec, make_sdp, session_packets
from easydarwin_amd.trace import UDP, TCP, Trace, capture_summary, read_capture
from easydarwin_amd.workload import shard_sessions

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N_SESS = 6


def _trace(sessions):
    """Sessions (global ids) -> trace; session g keeps its own seed and subscribers."""
    from scenarios import _assemble
    tracks = [TrackSpec("video", "H264/90000", 96, bitrate=300_000, gop=15, idr_bytes=3000),
              TrackSpec("audio", "PCMA/8000", 8)]
    tr = Trace()
    per, joins = [], []
    for local, g in enumerate(sessions):
        tr.add_session(make_sdp(tracks))
        per.append(session_packets(tracks, 1500, 0xEA5D + 500 + g))
        joins += [(0, local, 100 * g + k, TCP if k % 2 else UDP) for k in range(3)]
        joins.append((700, local, 100 * g + 50, UDP))
    return _assemble(tr, per, 100, 1500, joins)


def _capture(sessions, port):
    with tempfile.TemporaryDirectory() as td:
        t, c = os.path.join(td, "t.edtr"), os.path.join(td, "c.edcp")
        _trace(sessions).write(t)
        subprocess.run([port, t, c], check=True)
        cap = read_capture(open(c, "rb").read())
    return {k: v for k, v in capture_summary(cap).items()}


def _worker(rank, world, port, addr_port, out_q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(addr_port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mine = [g for g in range(N_SESS) if owner(g, world) == rank]
    summ = _capture(mine, port)
    got = [None] * world
    dist.all_gather_object(got, summ)
    elapsed, counts = reduce_run(1.0 + rank, [sum(v[0] for v in summ.values()), 1])
    if rank == 0:
        out_q.put((got, elapsed, counts))
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_sharding_partitions_sessions():
    for world in (1, 2, 4, 8):
        parts = [set(shard_sessions(8192, r, world).tolist()) for r in range(world)]
        assert set().union(*parts) == set(range(8192))
        assert sum(len(p) for p in parts) == 8192
        if world > 1:   # FNV-1a spreads stream IDs evenly (max within 10 % of the mean)
            assert max(len(p) for p in parts) < 1.1 * 8192 / world


def test_two_rank_output_invariance(oracle_bins):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, oracle_bins["port"], port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got, elapsed, counts = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    single = _capture(list(range(N_SESS)), oracle_bins["port"])
    # sub ids are global (100*g + k), so the per-rank captures merge without renumbering;
    # only the session field differs (local index), which the summary key does not carry
    merged = {}
    for part in got:
        assert not (merged.keys() & part.keys())
        merged.update(part)
    assert merged == single
    assert elapsed == 2.0                       # max over ranks
    assert counts[1] == 2                        # sum over ranks
    assert counts[0] == sum(v[0] for v in single.values())


def test_owned_sessions_balance_a_hash_sharded_population():
    """bench.py's weak-scaling population: every rank owns exactly `per_rank` stream IDs, each
    owned by its FNV-1a hash, none twice; one GPU gets range(per_rank)."""
    from easydarwin_amd.workload import fnv1a64, owned_sessions, stream_id
    for world in (1, 2, 8):
        parts = [owned_sessions(256, r, world) for r in range(world)]
        assert all(len(p) == 256 for p in parts)
        assert len(set().union(*[set(p.tolist()) for p in parts])) == 256 * world
        for r, p in enumerate(parts):
            assert all(fnv1a64(stream_id(int(g))) % world == r for g in p)
    assert owned_sessions(64, 0, 1).tolist() == list(range(64))


def test_bench_bounded_check_reports_hangs_and_errors():
    """bench.py's cross-device check runs bounded (run_bounded): a result passes through, an
    exception becomes a failed result, and a hang is reported after the deadline instead of
    holding up the line."""
    import threading
    import bench
    assert bench.run_bounded(lambda: {"ok": True}, 5.0) == ({"ok": True}, False)
    res, hung = bench.run_bounded(lambda: 1 / 0, 5.0)
    assert not hung and res["ok"] is False and "ZeroDivisionError" in res["error"]
    stop = threading.Event()
    res, hung = bench.run_bounded(lambda: stop.wait(30), 0.2)
    stop.set()
    assert hung and res == {"ok": False, "error": "timed out after 0 s"}
