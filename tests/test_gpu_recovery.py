"""GPU parity of the recovery scans: ad_recovery_batch (k_encode_recover,
k_probe_keys, k_scan_full, k_build, offsets, k_pack) vs the oracle's mapReduceFull restatement
(rc_recovery_batch), bit-exact keyDeps / rangeDeps / directKeyDeps for each of the four
BeginRecovery scans."""
import numpy as np
import pytest

from accord_deps import _abi as A, native, synth
from accord_deps.model import Queries

pytestmark = pytest.mark.gpu


def _same(w, oracle, scans=A.RECOVER_SCANS):
    st = native.DeviceCommandStore(0, w.range_start_inclusive, 1, w.slices)
    try:
        st.load(w)
        for s in scans:
            got = st.recovery_scan(w.queries, s)
            exp = oracle.recover(w, s)
            ok, why = got.equals(exp, detail=True)
            assert ok, "scan %d: %s" % (s, why)
    finally:
        st.close()


@pytest.mark.parametrize("seed", range(10))
def test_random_recovery(oracle, seed):
    w = synth.recovery_workload(seed, n_hist_txns=150 + 40 * seed, with_slices=(seed % 3 == 2),
                                start_inclusive=(seed % 4 == 1))
    _same(w, oracle)


def test_no_missing_lists(oracle):
    w = synth.recovery_workload(21)
    w.cfk.miss_off, w.cfk.miss = None, None           # every entry NO_TXNIDS
    _same(w, oracle)


def test_scaled_config2_recovery(oracle):
    # config 2's snapshot shape (Zipf hot keys, long segments) scaled down, recovering txnIds of its
    # history (known) and of its batch (unknown), entries with missing() lists
    w = synth.config2(n_txns=3000, n_keys=3000, n_hist_entries=60000, seed=5)
    rng = np.random.default_rng(5)
    e = rng.choice(w.cfk.n_entries, 1500, replace=False)
    key_of = np.repeat(np.arange(len(w.cfk.keys)), np.diff(w.cfk.seg.astype(np.int64)))
    hist = w.cfk.txn.take(e)
    from accord_deps.model import Tids
    txn = Tids.concat([hist, w.queries.txn.take(np.arange(1500))])
    keys = [np.array([w.cfk.keys[key_of[i]]], np.int64) for i in e] + \
           [w.queries.keys[int(w.queries.key_off[i]):int(w.queries.key_off[i + 1])] for i in range(1500)]
    off = np.zeros(len(keys) + 1, np.uint64)
    off[1:] = np.cumsum([len(k) for k in keys])
    w.queries = Queries(txn, txn, off, np.concatenate(keys))
    w.cfk = synth.with_missing(w.cfk, 5, frac=0.3)
    _same(w, oracle)


def test_big_segments(oracle):
    # a few keys with thousands of entries (many 64-entry scan rounds per probe)
    w = synth.recovery_workload(8, n_keys=4, n_hist_txns=3000, n_txns=40, max_keys=3)
    _same(w, oracle)


def test_empty_batch_and_keys(oracle):
    w = synth.recovery_workload(2)
    q = w.queries
    w.queries = Queries(q.txn.take(np.zeros(0, np.int64)), q.txn.take(np.zeros(0, np.int64)),
                        np.zeros(1, np.uint64), np.zeros(0, np.int64))
    _same(w, oracle)
    w.queries = Queries(q.txn, q.txn, np.zeros(len(q) + 1, np.uint64), np.zeros(0, np.int64))
    _same(w, oracle)


def test_errors():
    w = synth.random_small(3)                          # live range commands: not supported
    st = native.DeviceCommandStore(0)
    try:
        st.load(w)
        with pytest.raises(native.AccordDepsError) as e:
            st.recovery_scan(w.queries, 0)
        assert e.value.code == A.AD_E_STATE
        w2 = synth.recovery_workload(4)
        st.load(w2)
        with pytest.raises(native.AccordDepsError) as e:
            st.recovery_scan(w2.queries, 4)
        assert e.value.code == A.AD_E_INVAL
        q = w2.queries
        bad = q.txn.take(np.arange(len(q)))
        bad.lsb[0] = (bad.lsb[0] & ~np.uint64(0xE)) | np.uint64(5 << 1)     # LocalOnly: witnessedBy() throws
        with pytest.raises(native.AccordDepsError) as e:
            st.recovery_scan(Queries(bad, bad, q.key_off, q.keys), 0)
        assert e.value.code == A.AD_E_INVAL
        # the store stays usable after errors
        got = st.recovery_scan(w2.queries, 3)
        assert got.n_txns == len(q)
    finally:
        st.close()


@pytest.mark.parametrize("seed", range(8))
def test_random_recovery_with_ranges(oracle, seed):
    # live range commands with their recovery facts: the range half of mapReduceFull
    # (InMemoryCommandStore.java:884-958) -> rangeDeps, plus erased / historical commands it skips
    w = synth.recovery_workload(seed, n_range_cmds=16 + 8 * seed, with_slices=(seed % 3 == 2),
                                start_inclusive=(seed % 4 == 1))
    _same(w, oracle)


def test_many_range_commands_recovery(oracle):
    # hundreds of range entries: several frames of the range descent per probe
    w = synth.recovery_workload(31, n_range_cmds=400, n_hist_txns=300)
    assert sum(oracle.recover(w, s).pair_count(1) for s in A.RECOVER_SCANS) > 0
    _same(w, oracle)


def test_range_facts_cleared_by_reload():
    # loading range commands again drops the facts of the previous ones: recovery refuses until reloaded
    w = synth.recovery_workload(5, n_range_cmds=12)
    st = native.DeviceCommandStore(0)
    try:
        st.load(w)
        st.recovery_scan(w.queries, 3)
        from accord_deps import native as N
        import ctypes as C
        N.lib().ad_range_cmds_load(st.h, C.byref(w.cmds.soa()))
        with pytest.raises(native.AccordDepsError) as e:
            st.recovery_scan(w.queries, 3)
        assert e.value.code == A.AD_E_STATE
    finally:
        st.close()


@pytest.mark.parametrize("seed", range(10))
def test_range_domain_recovery(oracle, seed):
    # recovering sync points and range txns over Ranges (BeginRecovery.java:334,348,365,378 hand their
    # Seekables to mapReduceFull): the CommandsForKeys inside the sliced ranges
    # (InMemoryCommandStore.java:289-304, CommandsForKey.mapReduceFull :809-908) and the range commands
    # intersecting them under the four predicate sets (:896-961); sliced stores, both inclusivities,
    # with and without range commands
    w = synth.recovery_workload(seed, with_slices=(seed % 3 == 2), start_inclusive=(seed % 4 == 1),
                                n_range_cmds=(0 if seed % 5 == 4 else 16 + 4 * seed), range_frac=0.6, n_txns=70)
    assert w.queries.n_ranges > 0
    _same(w, oracle)


@pytest.mark.parametrize("seed", range(3))
def test_range_domain_recovery_device(oracle, seed):
    # the device entry (ad_recovery_batch_device) with Range-domain requests, via the region output
    w = synth.recovery_workload(40 + seed, n_range_cmds=24, range_frac=0.5, n_txns=90, with_slices=(seed == 1))
    import torch
    dev = torch.device("cuda", 0)
    st = native.DeviceCommandStore(0, w.range_start_inclusive, 1, w.slices)
    try:
        st.load(w)
        qdev, keep = native.device_queries(w.queries, dev)
        for s in A.RECOVER_SCANS:
            res, _ = st.recovery_scan_device(qdev, s)
            got = st.device_result_to_host(res)
            exp = oracle.recover(w, s)
            ok, why = got.equals(exp, detail=True)
            assert ok, "scan %d: %s" % (s, why)
    finally:
        st.close()


def test_range_domain_recovery_wide(oracle):
    # ranges over most of the key line: hundreds of CommandsForKey per request (the K2 scratch and
    # workgroup build), long segments, many range commands
    w = synth.recovery_workload(57, n_keys=600, n_hist_txns=1500, n_txns=60, max_keys=5, n_range_cmds=120,
                                range_frac=1.0)
    q = w.queries
    rs, re_ = q.range_start.copy(), q.range_end.copy()
    for i in range(0, len(q), 3):
        a, b = int(q.range_off[i]), int(q.range_off[i + 1])
        if b > a:
            rs[a:b] = [-600 + 10 * j for j in range(b - a)]
            re_[a:b] = [-600 + 10 * j + 5 for j in range(b - a)]
            re_[b - 1] = 600
    q.range_start, q.range_end = rs, re_
    assert max(int(q.range_off[i + 1] - q.range_off[i]) for i in range(len(q))) >= 1
    _same(w, oracle)
