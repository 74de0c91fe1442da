"""GPU parity of Range-domain requests: a txn whose Seekables are Ranges
(SafeCommandStore.mapReduceActive, SafeCommandStore.java:292) visits every CommandsForKey inside its
ranges sliced to the store (InMemoryCommandStore.mapReduceForKey, case Range, :289-304), the range
commands whose ranges intersect those sliced ranges (mapReduceRangesInternal, :884-1017;
CheckpointIntervalArray.forEachRange's job, :96-129) and the RedundantBefore entries intersecting its
unsliced ranges (RedundantBefore.collectDeps, RedundantBefore.java:420-423). HIP path (ad_deps_batch,
ad_deps_batch_device, ad_deps_batch_into) bit-exact against the oracle (oracle/refcpu.c, itself
checked against tests/refmodel.py in tests/test_oracle.py)."""
import numpy as np
import pytest

from accord_deps import _abi as A
from accord_deps import native, synth
from accord_deps.model import Workload

pytestmark = pytest.mark.gpu


def _w(seed, **kw):
    return synth.random_small(1000 + seed, range_frac=kw.pop("range_frac", 0.5), **kw)


def _eq(got, exp, what):
    ok, why = got.equals(exp, detail=True)
    assert ok, "%s: %s; first mismatch %r" % (what, why, got.first_mismatch(exp))


@pytest.mark.parametrize("seed", range(24))
def test_range_requests_match_oracle(oracle, seed):
    # mixed batches of key- and Range-domain requests of every kind (incl. ExclusiveSyncPoint ranges),
    # both inclusivities, sliced stores, with and without range commands and redundant-before entries
    w = _w(seed, n_keys=30 + 3 * seed, with_slices=(seed % 3 == 1), start_inclusive=(seed % 4 == 2),
           n_redundant=(0 if seed % 5 == 4 else 4), n_range_cmds=(0 if seed % 6 == 5 else 16))
    assert w.queries.n_ranges > 0
    exp = oracle.resolve(w)
    for via in ("host", "device", "regions"):
        _eq(native.resolve(w, via=via), exp, "seed %d via %s" % (seed, via))


@pytest.mark.parametrize("seed", range(8))
def test_range_requests_beside_lean(oracle, seed):
    # stores the lean kernels serve (no redundant-before entries, elision on; with and without range commands):
    # the key-domain requests of a mixed batch run the lean passes while its Range-domain requests are handed,
    # by k_prepare's record and the general kernel, to the split kernels after the first pack pass
    w = _w(300 + seed, n_keys=40 + 7 * seed, n_txns=240, n_hist_txns=400, range_frac=0.08 + 0.04 * (seed % 3),
           n_redundant=0, n_range_cmds=(0 if seed % 2 else 20), with_slices=(seed % 4 == 1),
           start_inclusive=(seed % 4 == 2))
    assert w.queries.n_ranges > 0
    exp = oracle.resolve(w)
    for via in ("host", "device", "regions"):
        _eq(native.resolve(w, via=via), exp, "seed %d via %s" % (seed, via))


def test_range_requests_beside_lean_config2_shape(oracle):
    # config 2's shape, scaled: Zipf keys over a 16x history, a few percent of the requests Range-domain
    # (synth.with_range_requests, bench.py --range-frac), checked on every request
    w, _, _ = synth.config2_sharded(0, 1, n_txns_per_gpu=6000, n_keys_per_gpu=6000, n_hist_entries_per_gpu=96000)
    w = synth.with_range_requests(w, 0.03)
    assert w.queries.n_ranges > 0
    _eq(native.resolve(w, via="regions"), oracle.resolve(w), "config2 shape + ranges")


@pytest.mark.parametrize("seed", range(3))
def test_range_requests_only_on_lean_store(oracle, seed):
    # a batch of Range-domain requests only, on a store the lean passes serve: lean pass 1 takes no request
    # and every one goes to the split kernels
    w = _w(400 + seed, n_keys=50, n_txns=150, n_hist_txns=300, range_frac=1.0, n_redundant=0,
           n_range_cmds=(0 if seed % 2 else 12), with_slices=(seed == 2))
    q = w.queries
    idx = np.array([i for i in range(len(q)) if q.ranges_of(i)])
    assert len(idx) > 50
    w = Workload(w.name, w.cfk, w.cmds, w.redundant, q.take(idx), w.flags, w.params, w.range_start_inclusive, w.slices)
    exp = oracle.resolve(w)
    for via in ("device", "regions"):
        _eq(native.resolve(w, via=via), exp, "seed %d via %s" % (seed, via))


@pytest.mark.parametrize("with_slices", [False, True])
def test_range_requests_holding_no_key(oracle, with_slices):
    # Range-domain requests whose one range lies beyond every key of the store (no CommandsForKey inside,
    # possibly outside its slices) beside key-domain requests the lean passes serve: empty expansions
    w = _w(420, n_keys=60, n_txns=220, n_hist_txns=400, range_frac=0.3, n_redundant=0, n_range_cmds=10,
           with_slices=with_slices)
    q = w.queries
    rs, re_ = q.range_start.copy(), q.range_end.copy()
    moved = 0
    for i in range(len(q)):
        a = int(q.range_off[i])
        if int(q.range_off[i + 1]) == a + 1:
            far = 10 ** 9 + 1000 * i
            rs[a], re_[a] = (far, far + 100) if i % 2 else (-far - 100, -far)
            moved += 1
    assert moved > 5
    q.range_start, q.range_end = rs, re_
    exp = oracle.resolve(w)
    for via in ("host", "device", "regions"):
        _eq(native.resolve(w, via=via), exp, "far ranges via %s" % via)


def test_range_requests_only_esp(oracle):
    # every request an ExclusiveSyncPoint over ranges (witnesses AnyGloballyVisible)
    w = _w(7, range_frac=1.0, n_keys=60, n_txns=120)
    q = w.queries
    lsb = (q.txn.lsb & ~np.uint64(0xE)) | np.uint64(A.KIND_EXCLUSIVE_SYNC_POINT << 1)
    q.txn.lsb = lsb
    q.exec.lsb = (q.exec.lsb & ~np.uint64(0xE)) | np.uint64(A.KIND_EXCLUSIVE_SYNC_POINT << 1)
    _eq(native.resolve(w), oracle.resolve(w), "esp")


@pytest.mark.parametrize("k2_big", [None, "8"])
def test_wide_ranges_many_keys(oracle, k2_big, monkeypatch):
    # ranges over most of the key line: hundreds of CommandsForKey per request (the K2 scratch and
    # workgroup paths), and the heavy-request path forced with AD_K2_BIG
    if k2_big:
        monkeypatch.setenv("AD_K2_BIG", k2_big)
    w = synth.random_small(77, n_keys=700, n_hist_txns=1500, n_txns=90, max_keys=6, range_frac=1.0,
                           n_range_cmds=60, n_redundant=6)
    q = w.queries
    # one range over almost everything for every third request
    rs, re_ = q.range_start.copy(), q.range_end.copy()
    for i in range(0, len(q), 3):
        a = int(q.range_off[i])
        if int(q.range_off[i + 1]) == a + 1:
            rs[a], re_[a] = -530, 530
    q.range_start, q.range_end = rs, re_
    _eq(native.resolve(w), oracle.resolve(w), "wide")


@pytest.mark.parametrize("slices", [1, 3])
def test_range_requests_into(oracle, slices):
    # the Panama path: caller-owned pinned outputs, the batch in slices (range offsets rebased per slice)
    w = _w(3, n_keys=80, n_txns=300, with_slices=True)
    st = native.DeviceCommandStore(0, w.range_start_inclusive, 1, w.slices)
    try:
        st.load(w)
        got, _, out = st.deps_batch_into(w.queries, slices=slices)
        out.release()
        _eq(got, oracle.resolve(w), "into")
    finally:
        st.close()


def test_range_requests_sampled_windows(oracle):
    # a sample of the batch (Queries.take) resolves to the same PartialDeps as in the full batch
    w = _w(11, n_txns=200)
    exp = oracle.resolve(w)
    idx = np.arange(0, 200, 7)
    w2 = Workload(w.name, w.cfk, w.cmds, w.redundant, w.queries.take(idx), w.flags, w.params,
                  w.range_start_inclusive, w.slices)
    got = native.resolve(w2)
    _eq(got, exp.take(idx), "sample")


def _bad(w, mutate):
    q = w.queries.take(np.arange(len(w.queries)))
    mutate(q)
    return Workload(w.name, w.cfk, w.cmds, w.redundant, q, w.flags, w.params, w.range_start_inclusive, w.slices)


def test_rejections():
    w = _w(5)
    q = w.queries
    i = next(i for i in range(len(q)) if q.ranges_of(i))
    j = int(q.range_off[i])

    def keys_and_ranges(b):
        b.keys = np.insert(b.keys, int(b.key_off[i]), 3)
        b.key_off = b.key_off.copy()
        b.key_off[i + 1:] += 1

    def empty_range(b):
        b.range_end = b.range_end.copy()
        b.range_end[j] = b.range_start[j]

    def overlapping(b):
        if int(b.range_off[i + 1]) - j < 2:
            b.range_start = np.insert(b.range_start, j + 1, b.range_start[j])
            b.range_end = np.insert(b.range_end, j + 1, b.range_end[j] + 5)
            b.range_off = b.range_off.copy()
            b.range_off[i + 1:] += 1
        else:
            b.range_start = b.range_start.copy()
            b.range_start[j + 1] = b.range_start[j]

    for mutate in (keys_and_ranges, empty_range, overlapping):
        bw = _bad(w, mutate)
        for via in ("host", "device"):
            with pytest.raises(native.AccordDepsError) as e:
                native.resolve(bw, via=via)
            assert e.value.code == A.AD_E_INVAL, (mutate.__name__, via)
    # SEQUENTIAL batches take key-domain requests only; a recovery scan of Range-domain requests on a
    # store whose range commands carry no recovery facts is refused as for key-domain ones
    st = native.DeviceCommandStore(0, w.range_start_inclusive, 1, w.slices)
    try:
        st.load(w)
        with pytest.raises(native.AccordDepsError) as e:
            st.calculate_partial_deps(q, A.AD_SEQUENTIAL)
        assert e.value.code == A.AD_E_INVAL
        with pytest.raises(native.AccordDepsError) as e:
            st.recovery_scan(q, 0)
        assert e.value.code == A.AD_E_STATE
        # the store still answers afterwards
        native_ok = st.calculate_partial_deps(q)
        assert native_ok.n_txns == len(q)
    finally:
        st.close()


def test_unnormalised_slices_rejected():
    with pytest.raises(native.AccordDepsError) as e:
        native.DeviceCommandStore(0, 0, 1, np.array([[0, 300], [-400, -100]], np.int64))
    assert e.value.code == A.AD_E_INVAL


@pytest.mark.parametrize("seed", range(10))
def test_sequential_range_txns(oracle, seed):
    # SEQUENTIAL batches mixing key- and Range-domain PreAccepts: each range txn registers as a range
    # command before its deps are computed (PreAccept.java:116-132, InMemoryCommandStore.java:740-763),
    # sliced and less its shard-redundant ranges (RedundantBefore.java:216-225); ad_deps_batch and
    # ad_deps_batch_into against the oracle's request-by-request restatement
    w = synth.sequential_ranges(3000 + seed, n_keys=30 + 3 * seed, n_txns=80, with_slices=(seed % 3 == 1),
                                start_inclusive=(seed % 4 == 2), n_redundant=(0 if seed % 5 == 4 else 4))
    assert w.queries.n_ranges > 0
    exp = oracle.resolve(w)
    _eq(native.resolve(w), exp, "seed %d" % seed)


def test_sequential_range_txns_persist(oracle):
    # the registered range commands stay in the store: two SEQUENTIAL batches, then a SNAPSHOT batch of
    # later requests, on one store and on one oracle store
    import pyoracle
    w = synth.sequential_ranges(3100, n_keys=50, n_txns=150, range_frac=0.5)
    q = w.queries
    h = len(q) // 2
    st = native.DeviceCommandStore(0, w.range_start_inclusive, 1, w.slices)
    ost = pyoracle.OracleStore(w.range_start_inclusive, 1, w.slices)
    try:
        st.load(w)
        ost.load(w)
        for lo, hi in ((0, h), (h, len(q))):
            part = q.window(lo, hi)
            _eq(st.calculate_partial_deps(part, A.AD_SEQUENTIAL), ost.deps_batch(part, A.AD_SEQUENTIAL), "batch %d" % lo)
        # every request again as SNAPSHOT reads: each sees the whole batch below its txnId, itself excluded
        _eq(st.calculate_partial_deps(q), ost.deps_batch(q), "snapshot after")
    finally:
        st.close()
        ost.close()


@pytest.mark.parametrize("seed", [1, 7])
def test_sequential_range_txn_below_registered(oracle, seed):
    # the library appends a registered range txn to the store's range commands where the oracle inserts it
    # in TxnId order (a TreeMap): nothing may depend on the registry's order. These seeds register a
    # Range-domain txn that sorts below an existing range command; the SEQUENTIAL batch, then SNAPSHOT
    # reads of every request on the grown registry, against the oracle
    import pyoracle
    w = synth.sequential_ranges(3000 + seed, n_keys=30 + 3 * seed, n_txns=80, with_slices=(seed % 3 == 1),
                                start_inclusive=(seed % 4 == 2), n_redundant=4)
    q, cm = w.queries, w.cmds
    top = max(zip(cm.txn.msb.tolist(), cm.txn.lsb.tolist()))
    assert any(q.ranges_of(i) and (int(q.txn.msb[i]), int(q.txn.lsb[i])) < top for i in range(len(q)))
    st = native.DeviceCommandStore(0, w.range_start_inclusive, 1, w.slices)
    ost = pyoracle.OracleStore(w.range_start_inclusive, 1, w.slices)
    try:
        st.load(w)
        ost.load(w)
        _eq(st.calculate_partial_deps(q, A.AD_SEQUENTIAL), ost.deps_batch(q, A.AD_SEQUENTIAL), "sequential")
        _eq(st.calculate_partial_deps(q), ost.deps_batch(q), "snapshot after")
    finally:
        st.close()
        ost.close()


def test_sequential_range_txn_already_registered():
    # a range txn the store already holds as a range command is refused, the store unchanged
    w = synth.sequential_ranges(3200, n_txns=40)
    q = w.queries
    i = next(i for i in range(len(q)) if q.ranges_of(i))
    st = native.DeviceCommandStore(0, w.range_start_inclusive, 1, w.slices)
    try:
        st.load(w)
        st.calculate_partial_deps(q.window(i, i + 1), A.AD_SEQUENTIAL)
        with pytest.raises(native.AccordDepsError) as e:
            st.calculate_partial_deps(q.window(i, i + 1), A.AD_SEQUENTIAL)
        assert e.value.code == A.AD_E_INVAL
        assert st.calculate_partial_deps(q).n_txns == len(q)
    finally:
        st.close()
