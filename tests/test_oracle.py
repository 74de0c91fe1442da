"""CPU tests of the oracle (oracle/refcpu.c): known answers from the reference's own tests, a
cross-check against an independent Python restatement, and Timestamp order/identity."""
import random

import numpy as np
import pytest

from accord_deps import _abi as A
from accord_deps import synth
from accord_deps.model import CfkSnapshot, Queries, RangeCommands, Redundant, Workload, make_txn_ids

import refmodel


def _request(batch, i):
    out = []
    for m in range(3):
        ks, ke, t, k2t = batch.maps[m].request(i)
        keys = [int(k) for k in ks] if ke is None else [(int(a), int(b)) for a, b in zip(ks, ke)]
        out.append((keys, t.tuples(), [int(x) for x in k2t]))
    return out


def _single_key_queries(txns, keys_per_txn):
    """Queries for a list of TxnIds (Tids) with per-request keys (lists)."""
    key_off = np.zeros(len(keys_per_txn) + 1, np.uint64)
    key_off[1:] = np.cumsum([len(k) for k in keys_per_txn])
    keys = np.concatenate([np.asarray(k, np.int64) for k in keys_per_txn])
    return Queries(txns, txns, key_off, keys)


# --------------------------------------------------------------------------------------------
# Known answers of PreAcceptTest (accord-core/src/test/java/accord/messages/PreAcceptTest.java).
# Every PreAcceptOk there carries PartialDeps with KeyDeps.NONE, RangeDeps.NONE, KeyDeps.NONE.
# --------------------------------------------------------------------------------------------
def _preaccept_store(oracle):
    st = oracle.OracleStore()
    w = Workload("kat", CfkSnapshot.empty(), RangeCommands.empty(), Redundant.empty(), None)
    st.load(w)
    return st


def _empty(batch):
    return all(batch.pair_count(m) == 0 for m in range(3)) and all(len(batch.maps[m].keys) == 0 for m in range(3))


def test_kat_initial_command(oracle):
    # initialCommandTest (:87-121): first write on key 10 -> no deps (:114)
    st = _preaccept_store(oracle)
    t = make_txn_ids([1], [101], [A.KIND_WRITE], [2])
    r = st.deps_batch(_single_key_queries(t, [[10]]), A.AD_SEQUENTIAL)
    assert _empty(r)


def test_kat_multi_key_timestamp_update(oracle):
    # multiKeyTimestampUpdate (:183-215): txn1 writes key 10 at hlc ~110; txn2 = TxnId(1, 50, Write,
    # Key, ID3) on keys {10, 11} started before txn1, so it has no deps (:209)
    st = _preaccept_store(oracle)
    t1 = make_txn_ids([1], [110], [A.KIND_WRITE], [2])
    assert _empty(st.deps_batch(_single_key_queries(t1, [[10]]), A.AD_SEQUENTIAL))
    t2 = make_txn_ids([1], [50], [A.KIND_WRITE], [3])
    assert _empty(st.deps_batch(_single_key_queries(t2, [[10, 11]]), A.AD_SEQUENTIAL))


def test_kat_single_key_newer_timestamp(oracle):
    # singleKeyNewerTimestamp (:221-245): TxnId(1, 110, Write, Key, ID2) on an empty store (:241)
    st = _preaccept_store(oracle)
    t = make_txn_ids([1], [110], [A.KIND_WRITE], [2])
    assert _empty(st.deps_batch(_single_key_queries(t, [[10]]), A.AD_SEQUENTIAL))


def test_kat_superseding_epoch(oracle):
    # supersedingEpochPrecludesFastPath (:247-290): epoch-2 topology, first txn on key 10 (:283)
    st = _preaccept_store(oracle)
    t = make_txn_ids([1], [101], [A.KIND_WRITE], [2])
    assert _empty(st.deps_batch(_single_key_queries(t, [[10]]), A.AD_SEQUENTIAL))


# witnessedAt of the same tests: rc_preaccept (the store's minNonConflicting + decision) composed
# with the host node clock (accord_deps.clock, Node.uniqueNow). IntKey k routes as the range
# (k - 1, k] (IntKey.asRange, end-inclusive), so a key's maxConflicts entry starts at k - 1.
def _witnessed(oracle, clk, txns, keys, maxc, node_epoch):
    q = _single_key_queries(txns, keys)
    mn, fl = oracle.preaccept(maxc, None, q, 1, node_epoch)
    return clk.witnessed_at_batch(txns, mn, fl), fl


def _maxc_after(keys, ts):
    from accord_deps.model import RangeMap, Tids
    starts = []
    for k in keys:
        starts += [k - 1, k]
    vals = Tids(np.array([ts[0]] * len(keys), np.uint64), np.array([ts[1]] * len(keys), np.uint64),
                np.array([ts[2]] * len(keys), np.int32))
    # one value per (k-1, k]; a gap (absent value) between non-adjacent keys
    st, v, pres = [], [], []
    for i, k in enumerate(keys):
        if st and st[-1] == k - 1:
            st.append(k)
        else:
            if st:
                v.append(i - 1)
                pres.append(0)
            st += [k - 1, k]
        v.append(i)
        pres.append(1)
    take = np.asarray(v, np.int64)
    return RangeMap(np.asarray(st, np.int64), vals.take(take), np.asarray(pres, np.uint8), 1)


def test_kat_witnessed_at_multi_key(oracle):
    # multiKeyTimestampUpdate (:187-218): node ID1, clock 100; txn1 = idForNode(1, ID2) on key 10 takes
    # the fast path; at clock 110, TxnId(1, 50, Write, Key, ID3) on {10, 11} is answered
    # Timestamp.fromValues(1, 110, ID1).withExtraFlags(txnId2.flags()) (:210)
    from accord_deps import clock
    clk = clock.NodeClock(1, 100, epoch=0)
    clk.set_epoch(1)
    t1 = make_txn_ids([1], [100], [A.KIND_WRITE], [2])
    w1, f1 = _witnessed(oracle, clk, t1, [[10]], None, 1)
    assert f1[0] & clock.AD_PA_FAST and w1[0] == t1.tuples()[0]
    clk.advance(10)
    t2 = make_txn_ids([1], [50], [A.KIND_WRITE], [3])
    w2, f2 = _witnessed(oracle, clk, t2, [[10, 11]], _maxc_after([10], t1.tuples()[0]), 1)
    assert not f2[0] & clock.AD_PA_FAST
    assert w2[0] == clock.make(1, 110, clock.flags_of(t2.tuples()[0]), 1)


def test_kat_witnessed_at_superseding_epoch(oracle):
    # supersedingEpochPrecludesFastPath (:251-291): topology at epoch 2; idForNode(1, ID2) at clock 100,
    # processed at 110 -> Timestamp.fromValues(2, 110, ID1) (:284)
    from accord_deps import clock
    clk = clock.NodeClock(1, 100, epoch=0)
    clk.set_epoch(1)
    clk.set_epoch(2)
    t = make_txn_ids([1], [100], [A.KIND_WRITE], [2])
    clk.advance(10)
    w, f = _witnessed(oracle, clk, t, [[10]], None, 2)
    assert not f[0] & clock.AD_PA_FAST
    assert w[0] == clock.make(2, 110, 0, 1)


def test_kat_witnessed_at_fast_paths(oracle):
    # initialCommandTest (:115) and singleKeyNewerTimestamp (:242): PreAcceptOk(txnId, txnId, ...)
    from accord_deps import clock
    for hlc in (100, 110):
        clk = clock.NodeClock(1, 100, epoch=0)
        clk.set_epoch(1)
        t = make_txn_ids([1], [hlc], [A.KIND_WRITE], [2])
        w, f = _witnessed(oracle, clk, t, [[10]], None, 1)
        assert f[0] & clock.AD_PA_FAST and w[0] == t.tuples()[0]


def test_node_clock_unique_and_rejected():
    # uniqueNow is strictly increasing; a rejected answer carries REJECTED_FLAG (Timestamp.asRejected)
    from accord_deps import clock
    clk = clock.NodeClock(7, 1000, epoch=3)
    a = clk.unique_now()
    b = clk.unique_now()
    assert clock.compare(a, b) < 0 and clock.hlc_of(a) == 1001 and clock.hlc_of(b) == 1002
    t = clock.make(3, 5000, 2, 9)
    r = clk.witnessed_at(t, (0, 0, 0), clock.AD_PA_REJECTED)
    assert r[1] & clock.REJECTED_FLAG and clock.hlc_of(r) == 5001 and r[2] == 7


def test_derived_write_after_write(oracle):
    # derived from the code (not a reference KAT): a later write on the same key depends on the
    # earlier PREACCEPTED write (never elided), a later read too (Ws), a later read on another key not
    st = _preaccept_store(oracle)
    t = make_txn_ids([1, 1, 1, 1], [100, 110, 120, 130], [A.KIND_WRITE, A.KIND_WRITE, A.KIND_READ, A.KIND_READ],
                     [2, 3, 2, 3])
    r = st.deps_batch(_single_key_queries(t, [[10], [10], [10, 11], [11]]), A.AD_SEQUENTIAL)
    reqs = [_request(r, i) for i in range(4)]
    tup = t.tuples()
    assert reqs[0][0] == ([], [], [])
    assert reqs[1][0] == ([10], [tup[0]], [2, 0])      # heads are absolute: nKeys + count
    assert reqs[2][0] == ([10], [tup[0], tup[1]], [3, 0, 1])
    assert reqs[3][0] == ([], [], [])                  # reads do not witness reads


def test_elision_of_transitive_dependencies(oracle):
    # CommandsForKey.java:913-950: M = executeAt of the last committed write before S (the STABLE
    # write at 120); committed reads/writes executing before M are elided (ELIDE_TRANSITIVE_DEPENDENCIES)
    t = make_txn_ids([1, 1, 1], [100, 110, 120], [A.KIND_WRITE] * 3, [1, 1, 1])
    cfk = CfkSnapshot(np.array([7]), np.array([0, 3]), t, t, np.array([A.ST_APPLIED, A.ST_APPLIED, A.ST_STABLE]))
    q = _single_key_queries(make_txn_ids([1], [200], [A.KIND_WRITE], [4]), [[7]])
    w = Workload("elide", cfk, RangeCommands.empty(), Redundant.empty(), q)
    r = oracle.resolve(w)
    assert _request(r, 0)[0] == ([7], [t.tuples()[2]], [2, 0])
    r = oracle.resolve(w, elide=0)
    assert _request(r, 0)[0] == ([7], t.tuples(), [4, 0, 1, 2])   # elision off: all three


@pytest.mark.parametrize("seed", range(30))
def test_crosscheck_python_restatement(oracle, seed):
    w = synth.random_small(seed, with_slices=(seed % 3 == 2), start_inclusive=(seed % 4 == 1))
    batch = oracle.resolve(w)
    for i in range(len(w.queries)):
        kd, rd, dd = refmodel.request_pairs(w, i)
        got = _request(batch, i)
        for m, pairs in ((0, kd), (1, rd), (2, dd)):
            keys, vals, k2t = refmodel.csr(pairs)
            assert got[m] == (keys, vals, k2t), (seed, i, A.MAP_NAMES[m])


@pytest.mark.parametrize("seed", range(24))
def test_crosscheck_range_domain_requests(oracle, seed):
    # Range-domain txns (SafeCommandStore.mapReduceActive over Ranges): every CommandsForKey key inside the
    # sliced ranges (InMemoryCommandStore.java:289-304), range commands intersecting the sliced ranges
    # (:884-1017), RedundantBefore entries intersecting the unsliced ranges (RedundantBefore.java:420-423)
    w = synth.random_small(900 + seed, n_keys=40 + seed, n_txns=80, range_frac=0.5, with_slices=(seed % 3 == 1),
                           start_inclusive=(seed % 4 == 2), n_redundant=(0 if seed % 5 == 4 else 4),
                           n_range_cmds=(0 if seed % 6 == 5 else 16))
    assert w.queries.n_ranges > 0
    batch = oracle.resolve(w)
    n_range_hits = 0
    for i in range(len(w.queries)):
        kd, rd, dd = refmodel.request_pairs(w, i)
        n_range_hits += bool(w.queries.ranges_of(i)) and bool(kd or rd or dd)
        got = _request(batch, i)
        for m, pairs in ((0, kd), (1, rd), (2, dd)):
            assert got[m] == refmodel.csr(pairs), (seed, i, A.MAP_NAMES[m])
    assert n_range_hits > 0


def test_with_range_requests_transform(oracle):
    # synth.with_range_requests (bench.py --range-frac): a share of config 2's requests become Range-domain txns
    # (domain bit set on txnId and executeAt, no keys) over one range holding 1-8 of the store's keys; the oracle
    # agrees with the model on them and on the key-domain requests around them
    w, _, _ = synth.config2_sharded(0, 1, n_txns_per_gpu=1500, n_keys_per_gpu=1500, n_hist_entries_per_gpu=12000)
    n_before = len(w.queries)
    w = synth.with_range_requests(w, 0.05, seed=11)
    q = w.queries
    assert len(q) == n_before
    isr = np.diff(q.range_off.astype(np.int64)) > 0
    assert 0 < int(isr.sum()) < n_before
    assert np.all(np.diff(q.key_off.astype(np.int64))[isr] == 0)
    assert np.all((q.txn.lsb[isr] & np.uint64(1)) == 1) and np.all((q.txn.lsb[~isr] & np.uint64(1)) == 0)
    keys = np.sort(w.cfk.keys)
    inside = [int(np.count_nonzero((keys > a) & (keys <= b))) for a, b in zip(q.range_start, q.range_end)]
    assert min(inside) >= 1 and max(inside) <= 8
    batch = oracle.resolve(w)
    for i in list(np.nonzero(isr)[0][:40]) + list(np.nonzero(~isr)[0][:20]):
        kd, rd, dd = refmodel.request_pairs(w, int(i))
        got = _request(batch, int(i))
        for m, pairs in ((0, kd), (1, rd), (2, dd)):
            assert got[m] == refmodel.csr(pairs), (int(i), A.MAP_NAMES[m])


def test_range_domain_request_rejections(oracle):
    w = synth.random_small(5, range_frac=0.5)
    q = w.queries
    i = next(i for i in range(len(q)) if q.ranges_of(i))
    # keys and ranges together
    bad = q.take(np.arange(len(q)))
    bad.key_off = bad.key_off.copy()
    j = int(bad.range_off[i])
    bad.keys = np.insert(bad.keys, int(bad.key_off[i]), 3)
    bad.key_off[i + 1:] += 1
    w2 = synth.Workload(w.name, w.cfk, w.cmds, w.redundant, bad, w.flags, w.params, w.range_start_inclusive, w.slices)
    with pytest.raises(RuntimeError):
        oracle.resolve(w2)
    # ranges not normalised (end <= start)
    bad = q.take(np.arange(len(q)))
    bad.range_end = bad.range_end.copy()
    bad.range_end[j] = bad.range_start[j]
    w2 = synth.Workload(w.name, w.cfk, w.cmds, w.redundant, bad, w.flags, w.params, w.range_start_inclusive, w.slices)
    with pytest.raises(RuntimeError):
        oracle.resolve(w2)


@pytest.mark.parametrize("seed", range(8))
def test_crosscheck_ephemeral_reads_at_timestamp_max(oracle, seed):
    # GetEphemeralReadDeps.apply computes deps at executeAt = Timestamp.MAX (GetEphemeralReadDeps.java:76,
    # Timestamp.java:29): every witnessed Write of the key started before MAX, elision below the key's
    # last committed Write; the id's flag bits read as kind 7
    w = synth.with_ephemeral_reads(synth.random_small(300 + seed, with_slices=(seed % 3 == 2)), frac=0.5, seed=seed)
    batch = oracle.resolve(w)
    n_eph = 0
    for i in range(len(w.queries)):
        n_eph += int(w.queries.exec.msb[i]) == synth.TIMESTAMP_MAX[0]
        kd, rd, dd = refmodel.request_pairs(w, i)
        got = _request(batch, i)
        for m, pairs in ((0, kd), (1, rd), (2, dd)):
            assert got[m] == refmodel.csr(pairs), (seed, i, A.MAP_NAMES[m])
    assert n_eph > 0


def test_crosscheck_no_elision(oracle):
    w = synth.random_small(77)
    batch = oracle.resolve(w, elide=0)
    for i in range(len(w.queries)):
        kd, rd, dd = refmodel.request_pairs(w, i, elide=False)
        got = _request(batch, i)
        assert got[0] == tuple(refmodel.csr(kd))
        assert got[2] == tuple(refmodel.csr(dd))


def test_sequential_equals_augmented_snapshot(oracle):
    # SEQUENTIAL (in ascending TxnId order) == SNAPSHOT over history + batch as PREACCEPTED
    # (SURVEY Appendix B), the identity the device implementation relies on
    w = synth.config1(n_txns=600, n_keys=60)
    seq = oracle.resolve(w)
    q = w.queries
    ent = []
    for i in range(len(q)):
        for k in q.keys[int(q.key_off[i]):int(q.key_off[i + 1])]:
            ent.append((int(k), i))
    ent.sort()
    keys = sorted({k for k, _ in ent})
    seg = np.zeros(len(keys) + 1, np.uint64)
    seg[1:] = np.cumsum([sum(1 for kk, _ in ent if kk == k) for k in keys])
    idx = np.array([i for _, i in ent])
    t = q.txn.take(idx)
    cfk = CfkSnapshot(np.array(keys), seg, t, t, np.full(len(idx), A.ST_PREACCEPTED, np.uint8))
    snap = oracle.resolve(Workload("aug", cfk, RangeCommands.empty(), Redundant.empty(), q))
    assert seq.equals(snap)


def test_timestamp_compare_and_equals(oracle):
    rng = random.Random(3)
    vals = []
    for _ in range(400):
        msb = rng.choice([0, 1, 5, (1 << 63) + 7, (1 << 64) - 1, rng.getrandbits(64)])
        lsb = rng.choice([0, 1, 0x1E, 0x8000, 0xFFFF, rng.getrandbits(64)])
        node = rng.choice([0, 1, -1, 2 ** 31 - 1, -2 ** 31, rng.randint(-5, 5)])
        vals.append((msb, lsb, node))
    for _ in range(4000):
        a, b = rng.choice(vals), rng.choice(vals)
        c = oracle.tid_cmp(a, b)
        kk = (refmodel.key(a) > refmodel.key(b)) - (refmodel.key(a) < refmodel.key(b))
        assert np.sign(c) == kk
        assert (c == 0) == refmodel.eq(a, b)
    # domain bit and REJECTED flag are not identity (Timestamp.java:41-45)
    assert oracle.tid_cmp((1, 0x10000, 3), (1, 0x10001, 3)) == 0
    assert oracle.tid_cmp((1, 0x10000, 3), (1, 0x18000, 3)) == 0
    assert oracle.tid_cmp((1, 0x10000, 3), (1, 0x10002, 3)) < 0
    assert oracle.tid_cmp((1 << 63, 0, 0), (1, 0, 0)) > 0          # unsigned msb


def test_levels_match_round_simulation(oracle):
    # level(T) = apply round when every txn applies as soon as all it waits on have applied
    g, _ = synth.config5(n_txns=3000, n_keys=300)
    assert np.array_equal(refmodel.levels_by_rounds(g), oracle.levels(g).astype(np.int64))


@pytest.mark.parametrize("seed", range(6))
def test_levels_all_kinds_match_round_simulation(oracle, seed):
    # every Txn.Kind (incl. EphemeralRead / LocalOnly, witnessed by nobody), direct deps both ways
    g = synth.random_graph(seed, n_txns=300, n_keys=12 + 4 * seed, long_runs=(seed == 5))
    assert np.array_equal(refmodel.levels_by_rounds(g), oracle.levels(g).astype(np.int64))


def test_oracle_rejects_invalid_inputs(oracle):
    t = make_txn_ids([1, 1], [110, 100], [A.KIND_WRITE] * 2, [1, 1])
    cfk = CfkSnapshot(np.array([1]), np.array([0, 2]), t, t, np.array([A.ST_APPLIED] * 2))
    st = oracle.OracleStore()
    with pytest.raises(oracle.OracleError) as e:
        st.load(Workload("bad", cfk, RangeCommands.empty(), Redundant.empty(), None))
    assert e.value.code == A.AD_E_ORDER


@pytest.mark.parametrize("seed", range(20))
def test_preaccept_oracle_vs_model(oracle, seed):
    # rc_preaccept (ReducingRangeMap.foldl restated with its search structure) against the key-by-key
    # model in refmodel.py: both interval conventions, null values, keys on interval starts, ties
    # of equal Timestamps with different non-identity flags, ExclusiveSyncPoints, rejectBefore
    import refmodel
    for ie in (0, 1):
        q, mc, rb = synth.preaccept_workload(seed, inclusive_ends=ie, with_reject=(seed % 3 != 0))
        for permit, ep in ((1, 0), (0, 0), (1, 2)):
            got, fl = oracle.preaccept(mc, rb, q, permit, ep)
            exp = refmodel.preaccept_model(mc, rb, q, permit, ep)
            for t, (v, f) in enumerate(exp):
                assert (int(got.msb[t]), int(got.lsb[t]), int(got.node[t])) == v and int(fl[t]) == f, (ie, permit, ep, t)


def test_preaccept_oracle_empty_maps(oracle):
    from accord_deps.model import RangeMap
    q, _, _ = synth.preaccept_workload(1)
    got, fl = oracle.preaccept(RangeMap.empty(), None, q, 1, 0)
    assert not got.msb.any() and not got.lsb.any()
    kinds = (q.txn.lsb >> np.uint64(1)) & np.uint64(7)
    assert np.array_equal(fl, np.where(kinds == 4, 4, 1).astype(np.uint8))    # NONE <= every txnId


@pytest.mark.parametrize("seed", range(16))
def test_sequential_range_txns_match_model(oracle, seed):
    # SEQUENTIAL batches with Range-domain txns: each registers as a range command before its deps are
    # computed (PreAccept.java:116-132, InMemoryCommandStore.java:740-763), sliced to the store and less
    # its shard-redundant ranges (RedundantBefore.java:216-225); later requests see it. The oracle's
    # request-by-request restatement against the model's augmented snapshot (refmodel.sequential_augmented)
    w = synth.sequential_ranges(2000 + seed, n_keys=30 + 2 * seed, n_txns=70, with_slices=(seed % 3 == 1),
                                start_inclusive=(seed % 4 == 2), n_redundant=(0 if seed % 5 == 4 else 4))
    q = w.queries
    assert q.n_ranges > 0
    seq = oracle.resolve(w)
    aug = refmodel.sequential_augmented(w)
    for i in range(len(q)):
        kd, rd, dd = refmodel.request_pairs(aug, i)
        got = _request(seq, i)
        for m, pairs in ((0, kd), (1, rd), (2, dd)):
            assert got[m] == tuple(refmodel.csr(pairs)), (seed, i, A.MAP_NAMES[m], q.ranges_of(i))
    # and the oracle's own SNAPSHOT over the augmented store (the identity the library relies on)
    assert seq.equals(oracle.resolve(aug))


def test_sequential_range_txns_seen_by_later_requests(oracle):
    # a registered range txn is a dependency of later requests on its ranges: some request's rangeDeps
    # name a txnId of the batch itself
    w = synth.sequential_ranges(2100, n_keys=40, n_txns=120, range_frac=0.5, n_range_cmds=0)
    seq = oracle.resolve(w)
    batch = set(w.queries.txn.tuples())
    named = sum(1 for i in range(len(w.queries)) for t in _request(seq, i)[1][1] if t in batch)
    assert named > 0
