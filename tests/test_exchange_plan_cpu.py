"""The library's exchange plan (ad_exchange_plan, the routine ad_exchange and ad_exchange_local share)
driven at world sizes 2..8 over gloo on CPU: each rank resolves its store's share with the oracle,
publishes its row of the exchange table (per-destination part counts + header), all-gathers the table,
asks the library for its transfers and moves the bytes exactly where the plan says (gloo isend/irecv at
the plan's offsets, own parts copied), then merges what it received with the oracle's PartialDeps.with.
The merged result must equal the sharded reference path (per-store calculatePartialDeps reduced with
PartialDeps.with: CommandStores.java:576-593, PreAccept.java:140-156; pyoracle.resolve_sharded).
With RCCL the only code left unexercised by this is the ncclSend/ncclRecv calls themselves.

Failure is collective: a rank publishing a failure status, a rank in another id format, or a rank whose
buffers are short makes every rank reach the same verdict from the same table."""
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
from accord_deps import _abi as A  # noqa: E402
from accord_deps import exchange, native, synth  # noqa: E402

UNIT_BYTES = (32, 8, 24, 4)         # triplet-format parts: hdr, key words, ids, k2t


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _workload(kind, seed, world):
    if kind == "config4":
        w = synth.config4(n_txns=500, n_keys=600, n_ranges=150, n_hist_txns=500)
        step = (1 << 32) // world
        return w, synth.cut_bounds([-(1 << 31) + step * g for g in range(1, world)])
    w = synth.config3(n_txns=2500, n_keys=300, seed=seed)
    return w, synth.shard_bounds(world)


def _as_bytes(a):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).copy())


def _rank_main(rank, world, port, kind, seed, mode, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        w, (lo, hi) = _workload(kind, seed, world)
        local, idx = synth.shard_local(w, lo[rank], hi[rank])
        n_total = len(w.queries)
        bases = exchange.owner_bases(n_total, world)
        dest_first = np.searchsorted(idx, np.asarray(bases[:world], np.int64)).astype(np.uint64).tolist() + [len(idx)]
        eng = parts_ref.OracleEngine(local, idx)
        eng.resolve()
        send, counts = eng.export(np.asarray(dest_first, np.uint64))
        fmt, status, recv_cap = A.AD_IDS_TRIPLET, 0, None
        if mode == "fail" and rank == world - 1:
            status = A.AD_E_NOMEM
        if mode == "format" and rank == 1:
            fmt = A.AD_IDS_RANK
        if mode == "grow" and rank == 0:
            recv_cap = [0, 0, 0, 0]
        row = native.exchange_row(counts, fmt, status, recv_cap=recv_cap)
        table = [torch.zeros(len(row), dtype=torch.int64) for _ in range(world)]
        dist.all_gather(table, torch.from_numpy(row.view(np.int64)))
        tab = torch.stack(table).numpy().view(np.uint64)
        rc, xf, ru, sp, flags = native.exchange_plan(tab, world, rank)
        if mode != "ok":
            out_q.put((rank, rc, flags, None))
            return
        assert rc == A.AD_OK and flags == 0
        # the move, at the plan's byte offsets: own parts copied, the rest over gloo point-to-point
        sbuf = [_as_bytes(send[k].numpy()) for k in ("hdr", "keys", "ids", "k2t")]
        rbuf = [torch.zeros(int(ru[a]) * UNIT_BYTES[a], dtype=torch.uint8) for a in range(4)]
        reqs = []
        for a in range(4):
            for p in range(world):
                so, sb, ro, rb = (int(x) for x in xf[a, p])
                if p == rank:
                    assert sb == rb
                    rbuf[a][ro:ro + rb] = sbuf[a][so:so + sb]
                    continue
                if rb:
                    reqs.append(dist.irecv(rbuf[a][ro:ro + rb], src=p, tag=a))
                if sb:
                    reqs.append(dist.isend(sbuf[a][so:so + sb].clone(), dst=p, tag=a))
        for r in reqs:
            r.wait()
        hdr, keys, ids, k2t = (rbuf[0].numpy().view(np.int64), rbuf[1].numpy().view(np.int64),
                               rbuf[2].numpy().view(np.int64), rbuf[3].numpy().view(np.int32))
        base, n_owned = bases[rank], bases[rank + 1] - bases[rank]
        per_src = parts_ref.decode(hdr, keys, ids, k2t, sp, base, n_owned)
        out_q.put((rank, rc, flags, (base, n_owned, pyoracle.merge_batches(per_src), int(sum(sp)), len(hdr) // 4)))
    finally:
        dist.destroy_process_group()


def _run(world, kind, seed, mode="ok"):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, kind, seed, mode, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(got, key=lambda x: x[0])


@pytest.mark.parametrize("kind,seed,world", [("config3", 31, 2), ("config3", 32, 3), ("config4", 0, 4),
                                             ("config3", 33, 5), ("config3", 34, 8)])
def test_plan_moves_parts_to_owners(kind, seed, world):
    w, bounds = _workload(kind, seed, world)
    expect = pyoracle.resolve_sharded(w, world, bounds=bounds)
    covered = 0
    for rank, rc, flags, (base, n_owned, merged, n_parts, n_hdr) in _run(world, kind, seed):
        assert n_parts == n_hdr                     # src_parts sums to the parts received
        ok, why = merged.equals(expect.window(base, n_owned), detail=True)
        assert ok, "rank %d: %s" % (rank, why)
        covered += n_owned
    assert covered == len(w.queries)


@pytest.mark.parametrize("mode,want_rc", [("fail", A.AD_E_PEER), ("format", A.AD_E_STATE), ("grow", A.AD_OK)])
def test_plan_verdict_is_collective(mode, want_rc):
    got = _run(3, "config3", 35, mode)
    for rank, rc, flags, _ in got:
        assert rc == want_rc, (mode, rank, rc)
        if mode == "grow":
            assert flags & A.AD_XPLAN_GROW          # every rank takes the growth round, not only rank 0


def test_plan_single_rank_and_layout():
    # world 1 (bench.py --exchange on one GPU): everything is a self copy; offsets are grouped by owner
    counts = np.array([[3, 5, 7, 9]], np.uint64)
    rc, xf, ru, sp, fl = native.exchange_plan(native.exchange_row(counts, A.AD_IDS_RANK), 1, 0)
    assert rc == A.AD_OK and fl == 0
    assert list(ru) == [3, 5, 7, 9] and list(sp) == [3]
    assert [tuple(int(v) for v in xf[a, 0]) for a in range(4)] == [(0, 96, 0, 96), (0, 40, 0, 40), (0, 28, 0, 28),
                                                                   (0, 36, 0, 36)]
    # world 3, rank 1: sends grouped by destination, receives in source order
    c = [np.array([[1, 1, 1, 1], [2, 2, 2, 2], [3, 3, 3, 3]], np.uint64) * (s + 1) for s in range(3)]
    tab = np.stack([native.exchange_row(c[s], A.AD_IDS_TRIPLET) for s in range(3)])
    rc, xf, ru, sp, fl = native.exchange_plan(tab, 3, 1)
    assert rc == A.AD_OK
    assert [int(x) for x in sp] == [2, 4, 6]                        # c[s][1][0]
    assert [int(xf[0, p, 0]) // 32 for p in range(3)] == [0, 2, 6]  # rank 1's own row: 2, 4, 6 parts
    assert [int(xf[0, p, 2]) // 32 for p in range(3)] == [0, 2, 6]
    assert int(xf[2, 2, 1]) == 6 * 24 and int(ru[2]) == 12
    # a malformed row is rejected, not planned
    bad = tab.copy()
    bad[2, 4 * 3] = 0
    assert native.exchange_plan(bad, 3, 0)[0] == A.AD_E_INVAL
