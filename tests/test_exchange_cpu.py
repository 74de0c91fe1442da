"""Multi-GPU protocol on CPU: routing of requests to stores, the all-to-all of per-store parts and
the per-owner merge, run with world_size 2 (and 3) over gloo, checked against the oracle of the
sharded reference path (per-store calculatePartialDeps + PartialDeps.with, pyoracle.resolve_sharded).
The GPU engine of the same protocol is covered by tests/test_gpu_multi.py."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import parts_ref  # noqa: E402
import pyoracle  # noqa: E402
from accord_deps import exchange, synth  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _workload(kind, seed, world):
    if kind == "small":
        w = synth.random_small(seed)
        w.slices = None
        return w, synth.cut_bounds([-100, 150][:world - 1] if world <= 3 else list(range(-300, 300, 600 // world))[1:world])
    w = synth.config3(n_txns=6000, n_keys=800, seed=seed)
    return w, synth.shard_bounds(world)


def _rank_main(rank, world, port, kind, seed, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        w, (lo, hi) = _workload(kind, seed, world)
        assert len(lo) == world
        local, idx = synth.shard_local(w, lo[rank], hi[rank])
        ex = exchange.ShardExchange(parts_ref.OracleEngine(local, idx), idx, len(w.queries), rank, world)
        merged = ex.step()
        out_q.put((rank, ex.txn_base, ex.n_owned, merged))
    finally:
        dist.destroy_process_group()


def _run(world, kind, seed):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, kind, seed, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(got, key=lambda x: x[0])


@pytest.mark.parametrize("kind,seed,world", [("small", 1, 2), ("small", 4, 3), ("config3", 7, 2), ("config3", 8, 4)])
def test_exchange_matches_sharded_oracle(kind, seed, world):
    w, bounds = _workload(kind, seed, world)
    expect = pyoracle.resolve_sharded(w, world, bounds=bounds)
    got = _run(world, kind, seed)
    covered = 0
    for rank, base, n_owned, merged in got:
        assert merged.n_txns == n_owned
        ok, why = merged.equals(expect.window(base, n_owned), detail=True)
        assert ok, "rank %d: %s" % (rank, why)
        covered += n_owned
    assert covered == len(w.queries)


def test_route_partitions_probes():
    w = synth.config3(n_txns=4000, n_keys=500, seed=3)
    lo, hi = synth.shard_bounds(4)
    total = 0
    for g in range(4):
        q, idx = exchange.route(w.queries, lo[g], hi[g])
        assert np.all(np.diff(idx) > 0)
        assert np.all((q.keys > lo[g]) & (q.keys <= hi[g]))
        assert np.all(np.diff(q.key_off.astype(np.int64)) > 0)      # only requests touching the slice
        total += q.n_probes
    assert total == w.queries.n_probes


def test_owner_bases_cover_batch():
    for n, world in [(10, 3), (7, 8), (1_000_000, 8)]:
        b = exchange.owner_bases(n, world)
        assert b[0] == 0 and b[-1] == n and all(b[i] <= b[i + 1] for i in range(world))


def test_transport_roundtrip():
    w = synth.random_small(5)
    w.slices = None
    res = pyoracle.resolve(w)
    idx = np.arange(len(w.queries), dtype=np.int64) + 100
    h, k, i, o, counts = parts_ref.encode(res, idx, np.array([0, len(w.queries)], np.uint64))
    back = parts_ref.decode(h, k, i, o, [counts[0, 0]], 100, len(w.queries))[0]
    assert back.equals(res)
