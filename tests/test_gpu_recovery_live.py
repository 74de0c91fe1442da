"""Recovery scans on a live store (SURVEY §8 f4 over f1): a config-2-shaped store serving a stream --
per step a batch of fresh PreAccepts inserted (CommandsForKey.update), the previous batch applied and
history entries moved on (ad_cfk_update_device) -- then the four BeginRecovery scans
(BeginRecovery.java:329-380; CommandsForKey.mapReduceFull :809-908) for txns of the stream and of the
history, after EVERY update batch. The RecoveryView is rebuilt from the device state (no host copy of
the store), and must answer bit-exactly as the oracle's mapReduceFull over the oracle's CommandsForKeys
after the same updates (oracle/cfk_update.py, rc_recovery_batch). With missing() lists kept on the
device (updates carrying deps), the same after each batch."""
import os
import sys

import numpy as np
import pytest

from accord_deps import _abi as A, native, synth
from accord_deps.model import CfkUpdates, Queries, Tids

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import cfk_update as U  # noqa: E402

pytestmark = pytest.mark.gpu


def _recovery_queries(cfk, stream_q, rng, n_hist=300, n_new=300):
    """Recovering txnIds: history entries (over their key + a random one) and requests of the stream."""
    key_of = np.repeat(np.arange(len(cfk.keys)), np.diff(cfk.seg.astype(np.int64)))
    e = rng.choice(cfk.n_entries, n_hist, replace=False)
    nq = min(n_new, len(stream_q))
    txn = Tids.concat([cfk.txn.take(e), stream_q.txn.take(np.arange(nq))])
    keys = [np.unique(np.array([cfk.keys[key_of[i]], cfk.keys[rng.integers(len(cfk.keys))]], np.int64)) for i in e] + \
           [stream_q.keys[int(stream_q.key_off[i]):int(stream_q.key_off[i + 1])] for i in range(nq)]
    off = np.zeros(len(keys) + 1, np.uint64)
    off[1:] = np.cumsum([len(k) for k in keys])
    return Queries(txn, txn, off, np.concatenate(keys))


def _check(st, w, cfk, q, oracle):
    old_cfk, old_q = w.cfk, w.queries
    w.cfk, w.queries = cfk, q
    try:
        for s in A.RECOVER_SCANS:
            got = st.recovery_scan(q, s)
            exp = oracle.recover(w, s)
            ok, why = got.equals(exp, detail=True)
            assert ok, "scan %d: %s" % (s, why)
    finally:
        w.cfk, w.queries = old_cfk, old_q


def test_recovery_after_every_update_batch(oracle):
    import torch
    dev = torch.device("cuda", 0)
    w = synth.config2(n_txns=2000, n_keys=3000, n_hist_entries=80000, seed=9)
    rng = np.random.default_rng(9)
    stream = synth.config2_stream(w, 3, 400, seed=19, held_keys_only=True)
    st = native.DeviceCommandStore(0)
    try:
        st.load(w)
        cfk = w.cfk
        prev = None
        for b, q in enumerate(stream):
            rows = np.repeat(np.arange(len(q)), np.diff(q.key_off.astype(np.int64)))
            ti = q.txn.take(rows)
            key_of = np.repeat(cfk.keys, np.diff(cfk.seg.astype(np.int64)))
            live = np.nonzero(cfk.status < A.ST_APPLIED)[0]
            e = np.sort(rng.choice(live, min(300, len(live)), replace=False))
            tst = np.maximum(cfk.status[e] + 1, A.ST_ACCEPTED).astype(np.uint8)
            parts = [(q.keys, ti, ti, np.full(len(rows), A.ST_PREACCEPTED, np.uint8)),
                     (key_of[e], cfk.txn.take(e), cfk.exec.take(e), tst)]
            if prev is not None:
                parts.append((prev[0], prev[1], prev[1], np.full(len(prev[0]), A.ST_APPLIED, np.uint8)))
            prev = (q.keys, ti)
            u = CfkUpdates(np.concatenate([p[0] for p in parts]), Tids.concat([p[1] for p in parts]),
                           Tids.concat([p[2] for p in parts]), np.concatenate([p[3] for p in parts]))
            exp, _ = U.cfk_update(cfk, u)
            if U.dup_committed_exec(exp):
                pytest.skip("generator produced a duplicate committed executeAt")
            ud, keep = native.device_updates(u, dev)
            st.cfk_update_device(ud)
            torch.cuda.synchronize()
            cfk = exp
            _check(st, w, cfk, _recovery_queries(cfk, q, rng), oracle)
    finally:
        st.close()


def test_recovery_live_with_device_missing_lists(oracle):
    # updates carrying deps keep every entry's missing() on the device; the view reads those lists
    import cfk_update_gen as G
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from test_gpu_cfk_missing import consistent_missing, with_deps
    w = synth.recovery_workload(33, n_hist_txns=300)
    consistent_missing(w.cfk, np.random.default_rng(33))
    rng = np.random.default_rng(34)
    st = native.DeviceCommandStore(0, w.range_start_inclusive, 1, w.slices)
    try:
        st.load(w)
        cfk = w.cfk
        for rnd in range(3):
            u = with_deps(cfk, G.concat(G.transitions(cfk, rng, 40, statuses=(3, 4, 5, 6))[0],
                                        G.fresh_preaccepts(cfk, rng, 10, statuses=(2, 3), epoch=9 + rnd,
                                                           hlc0=1 + 1000 * rnd)), rng)
            exp, _, _ = U.cfk_update_missing(cfk, u, u.dep_off, u.deps)
            if U.dup_committed_exec(exp):
                continue
            st.cfk_update(u)
            cfk = exp
            _check(st, w, cfk, w.queries, oracle)
    finally:
        st.close()


def test_device_view_equals_host_view(oracle, monkeypatch):
    # the same scans through the host-built view (AD_RV_HOST: a host copy of the store, on a second
    # store given the same updates) and the device-built one
    w = synth.recovery_workload(44, n_hist_txns=250)
    w.cfk.miss_off, w.cfk.miss = None, None
    rng = np.random.default_rng(44)
    import cfk_update_gen as G
    u = G.concat(G.transitions(w.cfk, rng, 60)[0], G.older_inserts(w.cfk, rng, 20, w=w))
    exp, _ = U.cfk_update(w.cfk, u)
    if U.dup_committed_exec(exp):
        pytest.skip("duplicate committed executeAt")
    res = []
    for host in (False, True):
        if host:
            monkeypatch.setenv("AD_RV_HOST", "1")
        st = native.DeviceCommandStore(0, w.range_start_inclusive, 1, w.slices)
        try:
            st.load(w)
            st.cfk_update(u)
            res.append([st.recovery_scan(w.queries, s) for s in A.RECOVER_SCANS])
            if not host:
                _check(st, w, exp, w.queries, oracle)
        finally:
            st.close()
    for s, a, b in zip(A.RECOVER_SCANS, res[0], res[1]):
        ok, why = a.equals(b, detail=True)
        assert ok, "scan %d: %s" % (s, why)
