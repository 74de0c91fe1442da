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


def test_build_global_dict_order_and_dups():
    # Timestamp order: msb unsigned, then (lsb >>> 16, identity flags) unsigned, then node signed;
    # ids equal under Timestamp.equals (non-identity lsb bits may differ) appear once, raw fields
    # from the first store holding them
    from accord_deps.model import Tids
    rng = np.random.default_rng(3)
    stores = []
    for s in range(3):
        n = 200
        msb = rng.integers(0, 4, n).astype(np.uint64) | np.uint64(1 << 63) * rng.integers(0, 2, n).astype(np.uint64)
        lsb = (rng.integers(0, 50, n).astype(np.uint64) << np.uint64(16)) | rng.integers(0, 16, n).astype(np.uint64) * 2
        node = rng.integers(-3, 4, n).astype(np.int32)
        stores.append(Tids(msb, lsb, node))
    # a cross-store duplicate differing only in a non-identity flag bit (0x8000 REJECTED)
    stores[2].msb[0], stores[2].lsb[0], stores[2].node[0] = stores[0].msb[5], stores[0].lsb[5] | np.uint64(0x8000), stores[0].node[5]
    g = exchange.build_global_dict(stores)

    def key(m, l, n):
        return (int(m), (int(l) >> 16, (int(l) >> 1) & 0xF), int(n))
    allk = {}
    for s in stores:
        for m, l, n in zip(s.msb, s.lsb, s.node):
            allk.setdefault(key(m, l, n), (m, l, n))
    want = sorted(allk)
    got = [key(m, l, n) for m, l, n in zip(g.msb, g.lsb, g.node)]
    assert got == want
    i = want.index(key(stores[0].msb[5], stores[0].lsb[5], stores[0].node[5]))
    assert int(g.lsb[i]) == int(stores[0].lsb[5])          # first store's raw fields


class _DictEngine:
    def __init__(self, rank):
        from accord_deps.model import Tids
        r = np.arange(10, dtype=np.uint64) * np.uint64(3) + np.uint64(rank)   # overlapping across ranks
        self.d = Tids(np.ones(10, np.uint64), r << np.uint64(16), np.zeros(10, np.int32))
        self.g = None

    def dictionary(self):
        return self.d

    def set_global_dict(self, g):
        self.g = g


def _dict_main(rank, world, port, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        e = _DictEngine(rank)
        ex = exchange.ShardExchange(e, np.arange(4), 8, rank, world)
        n = ex.install_global_dict()
        out_q.put((rank, n, e.g.lsb.tolist()))
    finally:
        dist.destroy_process_group()


def test_install_global_dict_collective():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dict_main, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = sorted(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = sorted(set((np.arange(10) * 3).tolist() + (np.arange(10) * 3 + 1).tolist()))
    for rank, n, lsb in got:
        assert n == len(want)
        assert [x >> 16 for x in lsb] == want
