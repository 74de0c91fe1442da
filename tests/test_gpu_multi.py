"""GPU parity of the multi-GPU data path on one MI355X: several CommandStores (token slices) on
cuda:0, each resolving the requests routed to it, exporting parts (ad_parts_export, HIP), an
emulated all-to-all (the same source-order concatenation RCCL produces), and the K3 merge
(ad_parts_merge, HIP) on each owner — bit-exact against the oracle of the sharded reference path
(per-store calculatePartialDeps + PartialDeps.with, pyoracle.resolve_sharded)."""
import numpy as np
import pytest
import torch

import pyoracle
from accord_deps import _abi as A
from accord_deps import exchange, native, synth

pytestmark = pytest.mark.gpu

UNITS = (("hdr", 4), ("keys", 1), ("ids", 3), ("k2t", 1))
UNITS_RANK = (("hdr", 4), ("keys", 1), ("ids", 1), ("k2t", 1))


def _parts(tensors, totals, rank_ids=False):
    p = A.AdParts()
    p.hdr, p.keys, p.ids, p.k2t = (tensors[k].data_ptr() for k in ("hdr", "keys", "ids", "k2t"))
    p.n_parts, p.n_key_words, p.n_ids, p.n_k2t = (int(x) for x in totals)
    p.id_format = A.AD_IDS_RANK if rank_ids else A.AD_IDS_TRIPLET
    return p


def _run_sharded(w, bounds, n_owners, rank_ids=False, parts_only=True):
    dev = torch.device("cuda", 0)
    lo, hi = bounds
    n_total = len(w.queries)
    bases = exchange.owner_bases(n_total, n_owners)
    engines, keep = [], []
    for g in range(len(lo)):
        local, idx = synth.shard_local(w, lo[g], hi[g])
        st = native.DeviceCommandStore(0, w.range_start_inclusive, 1, local.slices)
        st.load(local)
        qdev, k = native.device_queries(local.queries, dev)
        keep.append(k)
        e = exchange.GpuEngine(st, qdev, idx, dev, parts_only=parts_only)
        engines.append((e, idx))
    if rank_ids:
        # the ingest-time global dictionary (what ShardExchange.install_global_dict gathers)
        g = exchange.build_global_dict([e.dictionary() for e, _ in engines])
        for e, _ in engines:
            e.set_global_dict(g)
    done = []
    for e, idx in engines:
        e.resolve()
        dest_first = np.searchsorted(idx, np.asarray(bases[:n_owners], np.int64)).astype(np.uint64).tolist() + [len(idx)]
        send, counts = e.export(np.asarray(dest_first, np.uint64))
        done.append((e, send, counts))
    engines = done
    units = UNITS_RANK if rank_ids else UNITS
    torch.cuda.synchronize()
    out = []
    for d in range(n_owners):
        recv, totals, src_parts = {}, np.zeros(4, np.int64), []
        for a, (name, mult) in enumerate(units):
            pieces = []
            for e, send, counts in engines:
                start = int(counts[:d, a].sum()) * mult
                pieces.append(send[name][start:start + int(counts[d, a]) * mult])
            recv[name] = torch.cat(pieces) if pieces else torch.zeros(0, device=dev)
        for e, send, counts in engines:
            totals += counts[d]
            src_parts.append(int(counts[d, 0]))
        owner = engines[d % len(engines)][0].store
        torch.cuda.synchronize()                 # recv tensors were built on torch's stream
        mg = owner.merge_parts(_parts(recv, totals, rank_ids), src_parts, bases[d], bases[d + 1] - bases[d])
        out.append((bases[d], bases[d + 1] - bases[d], owner.merged_to_host(mg), mg.ms_device))
    for e, _, _ in engines:
        e.store.close()
    return out


def _check(w, bounds, n_owners, rank_ids=False, parts_only=True):
    expect = pyoracle.resolve_sharded(w, len(bounds[0]), bounds=bounds)
    for base, n, got, _ in _run_sharded(w, bounds, n_owners, rank_ids, parts_only):
        ok, why = got.equals(expect.window(base, n), detail=True)
        if not ok:
            bad = got.first_mismatch(expect.window(base, n))
            pytest.fail("owner base %d: %s; first mismatch %s" % (base, why, bad[:2] if bad else None))


@pytest.mark.parametrize("rank_ids", [False, True])
@pytest.mark.parametrize("seed", range(12))
def test_random_small_three_stores(seed, rank_ids):
    w = synth.random_small(seed)
    w.slices = None
    _check(w, synth.cut_bounds([-100, 150]), 2, rank_ids)


@pytest.mark.parametrize("rank_ids", [False, True])
@pytest.mark.parametrize("seed", range(6))
def test_range_requests_three_stores(seed, rank_ids):
    # Range-domain requests routed to every store one of their ranges meets, sliced by each store,
    # merged by K3 (PartialDeps.with) -- against the sharded oracle
    w = synth.random_small(500 + seed, range_frac=0.5, n_keys=60)
    w.slices = None
    _check(w, synth.cut_bounds([-100, 150]), 2, rank_ids)


@pytest.mark.parametrize("rank_ids", [False, True])
@pytest.mark.parametrize("n_stores,n_owners", [(2, 2), (4, 4), (8, 8), (8, 3)])
def test_config3_scaled(n_stores, n_owners, rank_ids):
    w = synth.config3(n_txns=40000, n_keys=6000, seed=11 + n_stores)
    _check(w, synth.shard_bounds(n_stores), n_owners, rank_ids)


@pytest.mark.parametrize("rank_ids", [False, True])
def test_export_from_packed_arrays(rank_ids):
    # export of a full result (packed arrays) instead of the parts-only batch's regions
    w = synth.config3(n_txns=20000, n_keys=3000, seed=41)
    _check(w, synth.shard_bounds(4), 4, rank_ids, parts_only=False)


@pytest.mark.parametrize("rank_ids", [False, True])
def test_config4_ranges_sharded(rank_ids):
    w = synth.config4(n_txns=3000, n_keys=4000, n_ranges=800, n_hist_txns=3000)
    lo, hi = synth.cut_bounds([-(1 << 30), 0, 1 << 30])
    _check(w, (lo, hi), 4, rank_ids)


@pytest.mark.parametrize("rank_ids", [False, True])
def test_config2_scaled_sharded(rank_ids):
    w = synth.config2(n_txns=20000, n_keys=20000, n_hist_entries=200000)
    _check(w, synth.shard_bounds(4), 4, rank_ids)


@pytest.mark.parametrize("width", ["2", "4", "8", "16", "32"])
def test_export_and_copy_lane_widths(width, monkeypatch):
    # the export at every lane width per request, whatever the batch's average ids per request would pick; big
    # groups included
    monkeypatch.setenv("AD_EXPORT_G", width)
    w = synth.config3(n_txns=20000, n_keys=3000, seed=43)
    _check(w, synth.shard_bounds(4), 3, rank_ids=True)
    _check(w, synth.shard_bounds(3), 2, rank_ids=False)
    w = synth.config2(n_txns=300, n_keys=40, n_hist_entries=60000, keys_per_txn=8, tail_unapplied=400)
    _check(w, synth.shard_bounds(4), 2, rank_ids=True)


def test_big_groups_rank_merge():
    # hot keys with thousands of live entries on every store: merged groups beyond 64 ids take the
    # binary-search path of the rank merge
    w = synth.config2(n_txns=300, n_keys=40, n_hist_entries=60000, keys_per_txn=8, tail_unapplied=400)
    _check(w, synth.shard_bounds(4), 2, rank_ids=True)


def test_rank_merge_many_sources():
    # more sources than the 16-lane per-request merge takes: the per-group rank merge
    w = synth.config3(n_txns=12000, n_keys=3000, seed=9)
    _check(w, synth.shard_bounds(18), 3, rank_ids=True)


def test_global_dict_before_prepare():
    # the snapshot built once over an installed node dictionary (bench config 3's ingest order)
    w = synth.config3(n_txns=20000, n_keys=3000, seed=13)
    lo, hi = synth.shard_bounds(2)
    locs = [synth.shard_local(w, lo[g], hi[g]) for g in range(2)]
    probe = []
    for local, _ in locs:
        st = native.DeviceCommandStore(0, w.range_start_inclusive, 1, local.slices)
        st.load(local)
        probe.append(st.dictionary())
        st.close()
    g = exchange.build_global_dict(probe)
    local, idx = locs[0]
    st = native.DeviceCommandStore(0, w.range_start_inclusive, 1, local.slices)
    st.load(local, prepare=False)
    st.set_global_dict(g)
    d = st.dictionary()
    assert len(d.msb) == len(g.msb) and np.array_equal(d.msb, g.msb)
    got = st.calculate_partial_deps(local.queries)
    exp = pyoracle.resolve(local)
    ok, why = got.equals(exp, detail=True)
    assert ok, why
    # a dictionary missing one of the store's ids is refused and leaves the store usable
    st2 = native.DeviceCommandStore(0, w.range_start_inclusive, 1, local.slices)
    st2.load(local, prepare=False)
    with pytest.raises(native.AccordDepsError) as ei:
        st2.set_global_dict(g.take(np.arange(1, len(g.msb))))
    assert ei.value.code == A.AD_E_INVAL
    ok, why = st2.calculate_partial_deps(local.queries).equals(exp, detail=True)
    assert ok, why
    st.close()
    st2.close()


def test_merge_rejects_overlapping_sources():
    dev = torch.device("cuda", 0)
    w = synth.config3(n_txns=4000, n_keys=500, seed=5)
    st = native.DeviceCommandStore(0)
    st.load(w)
    qdev, keep = native.device_queries(w.queries, dev)
    e = exchange.GpuEngine(st, qdev, np.arange(len(w.queries)), dev, parts_only=False)
    e.resolve()
    send, counts = e.export(np.array([0, len(w.queries)], np.uint64))
    recv = {k: torch.cat([send[k][:int(counts[0, a]) * m]] * 2) for a, (k, m) in enumerate(UNITS)}
    torch.cuda.synchronize()
    with pytest.raises(native.AccordDepsError) as ei:
        st.merge_parts(_parts(recv, 2 * counts[0]), [int(counts[0, 0])] * 2, 0, len(w.queries))
    assert ei.value.code == A.AD_E_INVAL
    st.close()


def _run_exchange_local(w, bounds, rank_ids):
    """The library's own node exchange (ad_exchange_local): N stores in this process on cuda:0,
    parts moved device-to-device and merged on each owner -- no Python transport."""
    dev = torch.device("cuda", 0)
    lo, hi = bounds
    n = len(lo)
    n_total = len(w.queries)
    bases = exchange.owner_bases(n_total, n)
    stores, keep, idxs, tis = [], [], [], []
    for g in range(n):
        local, idx = synth.shard_local(w, lo[g], hi[g])
        st = native.DeviceCommandStore(0, w.range_start_inclusive, 1, local.slices)
        st.load(local)
        qdev, k = native.device_queries(local.queries, dev)
        keep.append((qdev, k))
        ti = torch.from_numpy(np.ascontiguousarray(idx, np.int64)).to(dev)
        keep.append(ti)
        stores.append(st)
        idxs.append(idx)
        tis.append(ti.data_ptr())
    if rank_ids:
        g = exchange.build_global_dict([st.dictionary() for st in stores])
        for st in stores:
            st.set_global_dict(g)
    results = []
    for st, (qdev, _) in zip(stores, keep[0::2]):
        res, _ = st.deps_batch_device(qdev, None, parts_only=True)
        results.append(res)
    dfs = [np.searchsorted(idx, np.asarray(bases[:n], np.int64)).astype(np.uint64).tolist() + [len(idx)] for idx in idxs]
    torch.cuda.synchronize()
    merged, stats = native.exchange_local(stores, results, tis, dfs, bases[:n], [bases[d + 1] - bases[d] for d in range(n)])
    out = [(bases[d], bases[d + 1] - bases[d], stores[d].merged_to_host(merged[d])) for d in range(n)]
    for st in stores:
        st.close()
    return out, stats


@pytest.mark.parametrize("rank_ids", [False, True])
@pytest.mark.parametrize("case", ["random3", "config3_2", "config3_4", "config3_8", "config4_4", "config2_4"])
def test_exchange_local(case, rank_ids):
    if case == "random3":
        w = synth.random_small(7)
        w.slices = None
        bounds = synth.cut_bounds([-100, 150])
    elif case.startswith("config3"):
        n = int(case.split("_")[1])
        w = synth.config3(n_txns=40000, n_keys=6000, seed=21 + n)
        bounds = synth.shard_bounds(n)
    elif case == "config4_4":
        w = synth.config4(n_txns=3000, n_keys=4000, n_ranges=800, n_hist_txns=3000)
        bounds = synth.cut_bounds([-(1 << 30), 0, 1 << 30])
    else:
        w = synth.config2(n_txns=20000, n_keys=20000, n_hist_entries=200000)
        bounds = synth.shard_bounds(4)
    expect = pyoracle.resolve_sharded(w, len(bounds[0]), bounds=bounds)
    out, stats = _run_exchange_local(w, bounds, rank_ids)
    for base, n, got in out:
        ok, why = got.equals(expect.window(base, n), detail=True)
        if not ok:
            bad = got.first_mismatch(expect.window(base, n))
            pytest.fail("owner base %d: %s; first mismatch %s" % (base, why, bad[:2] if bad else None))
    assert len(bounds[0]) == 1 or stats["bytes_moved"] > 0


def _whole_from_shards(parts):
    """The node-wide workload the config3_shard stores slice: their CommandsForKeys concatenated
    (disjoint, slice order) and every request with all its keys -- the input of the sharded oracle."""
    from accord_deps.model import CfkSnapshot, Queries, RangeCommands, Redundant, Tids, Workload
    cfks = [p[0].cfk for p in parts]
    keys = np.concatenate([c.keys for c in cfks])
    segs = [c.seg.astype(np.int64) for c in cfks]
    off = np.cumsum([0] + [int(s[-1]) for s in segs])
    seg = np.concatenate([segs[0]] + [s[1:] + o for s, o in zip(segs[1:], off[1:])]).astype(np.uint64)
    cfk = CfkSnapshot(keys, seg, Tids.concat([c.txn for c in cfks]), Tids.concat([c.exec for c in cfks]),
                      np.concatenate([c.status for c in cfks]))
    Q = parts[0][2]
    rows, toks = [], []
    for w, idx, _, _ in parts:
        q = w.queries
        cnt = np.diff(q.key_off.astype(np.int64))
        rows.append(np.repeat(idx, cnt))
        toks.append(q.keys)
    rows = np.concatenate(rows)
    toks = np.concatenate(toks)
    o = np.lexsort((toks, rows))
    rows, toks = rows[o], toks[o]
    cnt = np.bincount(rows, minlength=Q)
    key_off = np.zeros(Q + 1, np.uint64)
    key_off[1:] = np.cumsum(cnt)
    # request ids: every store holds the same txnId for a request it sees
    msb = np.zeros(Q, np.uint64)
    lsb = np.zeros(Q, np.uint64)
    node = np.zeros(Q, np.int32)
    for w, idx, _, _ in parts:
        msb[idx], lsb[idx], node[idx] = w.queries.txn.msb, w.queries.txn.lsb, w.queries.txn.node
    t = Tids(msb, lsb, node)
    q = Queries(t, Tids(msb.copy(), lsb.copy(), node.copy()), key_off, toks)
    return Workload("config3_whole", cfk, RangeCommands.empty(), Redundant.empty(), q)


@pytest.mark.parametrize("world", [2, 4])
def test_config3_shards_exchange_local(world):
    # bench.py's N > 1 workload (config3_shard per store, the analytic global dictionary, rank-format
    # parts) through the library's node exchange, against the sharded oracle of the whole job
    dev = torch.device("cuda", 0)
    parts = [synth.config3_shard(r, world, txns_per_gpu=12000, keys_per_gpu=2000) for r in range(world)]
    whole = _whole_from_shards(parts)
    expect = pyoracle.resolve_sharded(whole, world)
    g = synth.config3_global_dict(parts[0][0].params, [p[3] for p in parts])
    Q = parts[0][2]
    bases = exchange.owner_bases(Q, world)
    stores, keep, tis, dfs, results = [], [], [], [], []
    for w, idx, _, _ in parts:
        st = native.DeviceCommandStore(0, 0, 1, w.slices)
        st.load(w)
        st.set_global_dict(g)
        qdev, k = native.device_queries(w.queries, dev)
        ti = torch.from_numpy(np.ascontiguousarray(idx, np.int64)).to(dev)
        keep += [qdev, k, ti]
        stores.append(st)
        tis.append(ti.data_ptr())
        dfs.append(np.searchsorted(idx, np.asarray(bases[:world], np.int64)).astype(np.uint64).tolist() + [len(idx)])
        res, _ = st.deps_batch_device(qdev, None, parts_only=True)
        results.append(res)
    torch.cuda.synchronize()
    merged, stats = native.exchange_local(stores, results, tis, dfs, bases[:world],
                                          [bases[d + 1] - bases[d] for d in range(world)])
    for d in range(world):
        got = stores[d].merged_to_host(merged[d])
        ok, why = got.equals(expect.window(bases[d], bases[d + 1] - bases[d]), detail=True)
        assert ok, (d, why)
    assert stats["bytes_moved"] > 0
    for st in stores:
        st.close()


def _sample(n, head=2000, spread=2000, seed=7):
    rng = np.random.default_rng(seed)
    return np.unique(np.concatenate([np.arange(min(n, head)), rng.choice(n, min(n, spread), replace=False)]))


def test_node_exchange_config3_share_full(oracle):
    # bench.py's multi-GPU step at full size on one GPU: rank 0's whole config-3 share (1/8 of BASELINE
    # config 3: 2M requests, 8M probes over a 24M-entry store) through NodeExchange -- the library's RCCL
    # communicator (ad_comm_init, world 1), ad_exchange (sizes -> table all-gather -> plan -> parts ->
    # grouped send/recv -> K3) -- sampled bit-exact against the reference path over the same store
    dev = torch.device("cuda", 0)
    w, idx, n_total, exec_ids = synth.config3_shard(0, 1)
    st = native.DeviceCommandStore(0, 0, 1, w.slices)
    try:
        st.load(w, prepare=False)
        st.set_global_dict(synth.config3_global_dict(w.params, [exec_ids]))
        qdev, keep = native.device_queries(w.queries, dev)
        nx = exchange.NodeExchange(st, qdev, idx, n_total, 0, 1, dev)
        mg = nx.step()                            # grows the exchange buffers (growth round)
        mg = nx.step()                            # steady step on the grown buffers
        assert mg.n_txns == n_total and nx.last_exchange["bytes_moved"] == 0     # world 1: all self copies
        sample = _sample(n_total)
        got = st.merged_to_host(mg, sample)
        exp = oracle.OracleStore(w.range_start_inclusive, 1, w.slices).load(w).deps_batch(w.queries.take(sample), w.flags)
        ok, why = got.equals(exp, detail=True)
        if not ok:
            mm = got.first_mismatch(exp)
            raise AssertionError("%s; first mismatch %r" % (why, mm[:2] if mm else None))
        # a rank whose export fails publishes its status in the table: the step fails on every rank
        # before the move, the communicator survives and the next step is whole again
        bad = list(nx.dest_first)
        bad[-1] += 1
        with pytest.raises(native.AccordDepsError) as ei:
            st.exchange(nx.last_res, nx.ti.data_ptr(), bad, nx.txn_base, nx.n_owned)
        assert ei.value.code == A.AD_E_INVAL
        mg = nx.step()
        ok, why = st.merged_to_host(mg, sample).equals(exp, detail=True)
        assert ok, why
    finally:
        st.close()


def test_node_exchange_small_triplets_and_ranks(oracle):
    # the same step over a small store in both id formats (the global dictionary installed or not)
    dev = torch.device("cuda", 0)
    w = synth.config3(n_txns=20000, n_keys=3000, seed=17)
    exp = pyoracle.resolve(w)
    for rank_ids in (False, True):
        st = native.DeviceCommandStore(0, w.range_start_inclusive, 1, w.slices)
        try:
            st.load(w)
            if rank_ids:
                st.set_global_dict(st.dictionary())
            qdev, keep = native.device_queries(w.queries, dev)
            nx = exchange.NodeExchange(st, qdev, np.arange(len(w.queries)), len(w.queries), 0, 1, dev)
            for _ in range(2):
                mg = nx.step()
                assert mg.id_format == (A.AD_IDS_RANK if rank_ids else A.AD_IDS_TRIPLET)
                ok, why = st.merged_to_host(mg).equals(exp, detail=True)
                assert ok, (rank_ids, why)
        finally:
            st.close()
