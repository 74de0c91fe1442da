"""GPU parity of device-resident CommandsForKey maintenance: ad_cfk_update applies
a batch of CommandsForKey.update status transitions to the snapshot in HBM (k_upd_locate,
k_upd_apply, re-derivation of ent / committedByExecuteAt / cand / cwr / krec / KeyEntry / trees).
Checked against the oracle's restatement (oracle/cfk_update.py): the entries' status and
executeAt, and the deps every later batch computes (bit-exact vs the oracle's calculatePartialDeps
over the updated CommandsForKey) on the lean, general and split paths; error batches leave the
store unchanged."""
import os
import sys

import numpy as np
import pytest

from accord_deps import _abi as A, native, synth
from accord_deps.model import CfkUpdates, Tids

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import cfk_update as U  # noqa: E402
import cfk_update_gen as G  # noqa: E402

pytestmark = pytest.mark.gpu


def _java_would_throw(w, new_cfk, oracle):
    """Random transitions can leave a state the reference rejects when read (the prunedBefore walk running past
    committedByExecuteAt, CommandsForKey.java:952-965): such a batch is not applied."""
    old = w.cfk
    w.cfk = new_cfk
    try:
        oracle.resolve(w)
        return False
    except oracle.OracleError as e:
        return e.code == A.AD_E_STATE
    finally:
        w.cfk = old


def _check(w, st, oracle, new_cfk):
    s, x = st.cfk_entries()
    assert s.tolist() == new_cfk.status.tolist()
    assert x.msb.tolist() == new_cfk.exec.msb.tolist() and x.lsb.tolist() == new_cfk.exec.lsb.tolist()
    assert x.node.tolist() == new_cfk.exec.node.tolist()
    w2 = w
    old = w2.cfk
    w2.cfk = new_cfk
    try:
        exp = oracle.resolve(w2)
        got = st.calculate_partial_deps(w2.queries, w2.flags)
        ok, why = got.equals(exp, detail=True)
        assert ok, why
    finally:
        w2.cfk = old


@pytest.mark.parametrize("path", [0, 1])
@pytest.mark.parametrize("seed", range(8))
def test_random_transitions(oracle, seed, path):
    w = synth.random_small(seed, with_slices=(seed % 4 == 3), start_inclusive=(seed % 3 == 1))
    w.flags = A.AD_SNAPSHOT
    rng = np.random.default_rng(100 + seed)
    st = native.DeviceCommandStore(0, w.range_start_inclusive, 1, w.slices, path=path)
    try:
        st.load(w)
        cfk = w.cfk
        for rnd in range(3):                     # successive batches on the same device state
            u, e = G.transitions(cfk, rng, 60 + 30 * rnd)
            new, _ = U.cfk_update(cfk, u)
            n_applied, _ = st.cfk_update(u)
            assert n_applied == int((new.status != cfk.status).sum())
            _check(w, st, oracle, new)
            cfk = new
    finally:
        st.close()


def test_update_then_reload_equals_fresh_load(oracle):
    # the derived device state after updates answers exactly as a store loaded from the updated SoA
    w = synth.random_small(31, n_hist_txns=300, n_txns=120)
    w.flags = A.AD_SNAPSHOT
    rng = np.random.default_rng(31)
    u, _ = G.transitions(w.cfk, rng, 400)
    new, _ = U.cfk_update(w.cfk, u)
    a = native.DeviceCommandStore(0, w.range_start_inclusive, 1, w.slices)
    b = native.DeviceCommandStore(0, w.range_start_inclusive, 1, w.slices)
    try:
        a.load(w)
        a.cfk_update(u)
        old = w.cfk
        w.cfk = new
        b.load(w)
        ra, rb = a.calculate_partial_deps(w.queries), b.calculate_partial_deps(w.queries)
        w.cfk = old
        ok, why = ra.equals(rb, detail=True)
        assert ok, why
    finally:
        a.close()
        b.close()


def test_config2_scaled_commit_wave(oracle):
    # config 2's shape: the unapplied tail of every key commits (executeAt = txnId or its own), then applies
    w = synth.config2(n_txns=2000, n_keys=2000, n_hist_entries=40000, seed=9)
    live = np.nonzero(w.cfk.status < A.ST_APPLIED)[0]
    st = native.DeviceCommandStore(0)
    try:
        st.load(w)
        cfk = w.cfk
        keys = G.entry_keys(cfk)
        for target in (A.ST_COMMITTED, A.ST_APPLIED):
            u = CfkUpdates(keys[live], cfk.txn.take(live), cfk.exec.take(live), np.full(len(live), target, np.uint8))
            new, _ = U.cfk_update(cfk, u)
            st.cfk_update(u)
            _check(w, st, oracle, new)
            cfk = new
    finally:
        st.close()


def test_device_buffers_and_recovery_follow(oracle):
    import torch
    w = synth.recovery_workload(4)
    rng = np.random.default_rng(4)
    # statuses that keep TxnInfo.missing() (ACCEPTED..APPLIED, CommandsForKey.java:278)
    u, _ = G.transitions(w.cfk, rng, 100, statuses=range(A.ST_ACCEPTED, A.ST_APPLIED + 1))
    new, _ = U.cfk_update(w.cfk, u)
    st = native.DeviceCommandStore(0, w.range_start_inclusive, 1, w.slices)
    try:
        st.load(w)
        dev = torch.device("cuda", 0)
        ud, keep = native.device_updates(u, dev)
        st.cfk_update_device(ud, torch.cuda.current_stream(dev).cuda_stream)
        old = w.cfk
        w.cfk = new
        new.miss_off, new.miss = old.miss_off, old.miss        # entries did not move: missing() lists hold
        try:
            for s in A.RECOVER_SCANS:
                ok, why = st.recovery_scan(w.queries, s).equals(oracle.recover(w, s), detail=True)
                assert ok, "scan %d: %s" % (s, why)
        finally:
            w.cfk = old
        # an entry with missing() ids invalidated: the lists must be loaded again
        e = int(np.nonzero(np.diff(w.cfk.miss_off.astype(np.int64)) > 0)[0][0])
        inv = CfkUpdates(G.entry_keys(w.cfk)[[e]], w.cfk.txn.take([e]), w.cfk.txn.take([e]),
                         np.array([A.ST_INVALID], np.uint8))
        st.cfk_update(inv)
        with pytest.raises(native.AccordDepsError) as ei:
            st.recovery_scan(w.queries, 0)
        assert ei.value.code == A.AD_E_STATE
    finally:
        st.close()


def _unchanged_after_error(w, st, oracle, u, code):
    before = st.calculate_partial_deps(w.queries, w.flags)
    with pytest.raises(native.AccordDepsError) as ei:
        st.cfk_update(u)
    assert ei.value.code == code
    s, x = st.cfk_entries()
    assert s.tolist() == w.cfk.status.tolist() and x.lsb.tolist() == w.cfk.exec.lsb.tolist()
    ok, why = st.calculate_partial_deps(w.queries, w.flags).equals(before, detail=True)
    assert ok, why


def test_errors_leave_store_unchanged(oracle):
    w = synth.random_small(7)
    w.flags = A.AD_SNAPSHOT
    rng = np.random.default_rng(7)
    st = native.DeviceCommandStore(0, w.range_start_inclusive, 1, w.slices)
    try:
        st.load(w)
        u, _ = G.transitions(w.cfk, rng, 30, statuses=[A.ST_STABLE])
        bad_st = CfkUpdates(u.keys, u.txn, u.exec, u.status.copy())
        bad_st.status[0] = 9
        _unchanged_after_error(w, st, oracle, bad_st, A.AD_E_INVAL)
        # two entries of one key committed at one executeAt (CommandsForKey.java:1439): rolled back
        seg = w.cfk.seg.astype(np.int64)
        k = int(np.argmax(np.diff(seg)))
        kd = [e for e in range(int(seg[k]), int(seg[k + 1])) if (int(w.cfk.txn.lsb[e]) & 1) == 0]
        e0, e1 = kd[0], kd[1]
        dup = CfkUpdates(np.array([w.cfk.keys[k]] * 2), w.cfk.txn.take([e0, e1]),
                         w.cfk.txn.take([e0, e0]), np.array([A.ST_APPLIED, A.ST_APPLIED]))
        new, _ = U.cfk_update(w.cfk, dup)
        assert U.dup_committed_exec(new)
        _unchanged_after_error(w, st, oracle, dup, A.AD_E_DUP_EXEC)
        # and the store still takes a good batch afterwards
        new, _ = U.cfk_update(w.cfk, u)
        st.cfk_update(u)
        _check(w, st, oracle, new)
    finally:
        st.close()


def test_empty_batch_and_sequential_follows(oracle):
    w = synth.config1(n_txns=300, n_keys=50)
    st = native.DeviceCommandStore(0)
    try:
        st.load(w)
        assert st.cfk_update(CfkUpdates(np.zeros(0, np.int64), Tids(np.zeros(0), np.zeros(0), np.zeros(0)),
                                        Tids(np.zeros(0), np.zeros(0), np.zeros(0)), np.zeros(0, np.uint8)))[0] == 0
    finally:
        st.close()


# ---- insertion of ids newer than the store (fresh PreAccepts) --------------------------------
@pytest.mark.parametrize("path", [0, 1])
@pytest.mark.parametrize("seed", range(6))
def test_insert_fresh_preaccepts(oracle, seed, path):
    w = synth.random_small(40 + seed, with_slices=(seed % 3 == 2))
    w.flags = A.AD_SNAPSHOT
    rng = np.random.default_rng(40 + seed)
    st = native.DeviceCommandStore(0, w.range_start_inclusive, 1, w.slices, path=path)
    try:
        st.load(w)
        cfk = w.cfk
        for rnd in range(3):                     # each round inserts newer txns, raises older ones
            ins = G.fresh_preaccepts(cfk, rng, 15 + 10 * rnd, epoch=9 + rnd, statuses=(0, 2, 3, 4, 6),
                                     new_exec_frac=0.3)
            tr, _ = G.transitions(cfk, rng, 40)
            u = G.concat(tr, ins, ins) if rnd == 1 else G.concat(ins, tr)
            new, _ = U.cfk_update(cfk, u)
            st.cfk_update(u)
            assert new.n_entries > cfk.n_entries
            _check(w, st, oracle, new)
            cfk = new
        # a known txnId appended to a key that does not hold it (newer than the key's last id) is
        # an insertion too; one older than the key's last id is not on the device
        seg = cfk.seg.astype(np.int64)
        last = int(np.lexsort((cfk.txn.node, cfk.txn.lsb >> np.uint64(16), cfk.txn.msb))[-1])   # the newest id
        k_of = np.repeat(np.arange(len(cfk.keys)), np.diff(seg))
        holds = set(k_of[(cfk.txn.msb == cfk.txn.msb[last]) & (cfk.txn.lsb == cfk.txn.lsb[last]) &
                         (cfk.txn.node == cfk.txn.node[last])].tolist())
        other = [k for k in range(len(cfk.keys)) if k not in holds][0]
        u = CfkUpdates(np.array([cfk.keys[other]]), cfk.txn.take([last]), cfk.txn.take([last]),
                       np.array([A.ST_ACCEPTED], np.uint8))
        new, _ = U.cfk_update(cfk, u)
        st.cfk_update(u)
        _check(w, st, oracle, new)
    finally:
        st.close()


# ---- insertion below the newest id: mid-segment inserts, dictionary merge + rank remap ---------
@pytest.mark.parametrize("path", [0, 1])
@pytest.mark.parametrize("seed", range(6))
def test_insert_older_ids(oracle, seed, path):
    # ids the dictionary does not hold, older than its newest id (txnIds and executeAts), and known
    # ids inserted into keys that do not hold them: every rank of the store is remapped (range
    # entries, stabbing cells, RedundantBefore watermarks, prunedBefore included)
    w = synth.random_small(60 + seed, with_slices=(seed % 3 == 2), start_inclusive=(seed % 2 == 1))
    w.flags = A.AD_SNAPSHOT
    rng = np.random.default_rng(60 + seed)
    st = native.DeviceCommandStore(0, w.range_start_inclusive, 1, w.slices, path=path)
    try:
        st.load(w)
        cfk = w.cfk
        for rnd in range(3):
            old = G.older_inserts(cfk, rng, 20 + 10 * rnd, w=w)
            tr, _ = G.transitions(cfk, rng, 30)
            fresh = G.fresh_preaccepts(cfk, rng, 5, epoch=9 + rnd)
            u = G.concat(old, tr, fresh, old) if rnd == 1 else G.concat(tr, old, fresh)
            new, _ = U.cfk_update(cfk, u)
            if U.dup_committed_exec(new):
                continue
            _, stats = st.cfk_update(u)
            assert new.n_entries > cfk.n_entries
            _check(w, st, oracle, new)
            cfk = new
    finally:
        st.close()


def _sequential_check(w, st, oracle, cfk, rng, epoch=12):
    """A SEQUENTIAL batch of newer PreAccepts over the store as updated (the host copy follows the
    device, prunedBefore included, before inserting the batch): bit-exact vs the oracle."""
    from accord_deps.model import Queries
    q = G.fresh_preaccepts(cfk, rng, 30, epoch=epoch)
    rows = np.r_[0, np.nonzero(np.diff(q.txn.lsb.astype(np.int64)))[0] + 1]
    off = np.r_[rows, len(q)].astype(np.uint64)
    keys = np.concatenate([np.sort(q.keys[int(off[i]):int(off[i + 1])]) for i in range(len(rows))])
    old_q, old_cfk, old_flags = w.queries, w.cfk, w.flags
    w.queries = Queries(q.txn.take(rows), q.txn.take(rows), off, keys)
    w.cfk = cfk
    try:
        w.flags = A.AD_SEQUENTIAL
        exp = oracle.resolve(w)
        got = st.calculate_partial_deps(w.queries, A.AD_SEQUENTIAL)
        ok, why = got.equals(exp, detail=True)
        assert ok, why
    finally:
        w.queries, w.cfk, w.flags = old_q, old_cfk, old_flags


def test_insert_older_then_sequential(oracle):
    # mid-segment inserts move prunedBefore's byId index: a host rebuild must find it again
    for seed in range(4):
        w = synth.random_small(90 + seed, n_range_cmds=0)
        w.flags = A.AD_SNAPSHOT
        rng = np.random.default_rng(90 + seed)
        st = native.DeviceCommandStore(0, w.range_start_inclusive, 1, w.slices)
        try:
            st.load(w)
            u = G.older_inserts(w.cfk, rng, 40, statuses=(0, 2, 3), w=w)
            new, _ = U.cfk_update(w.cfk, u)
            st.cfk_update(u)
            _check(w, st, oracle, new)
            _sequential_check(w, st, oracle, new, rng)
        finally:
            st.close()


def test_insert_older_than_key_and_unknown_exec(oracle):
    w = synth.random_small(50)
    w.flags = A.AD_SNAPSHOT
    st = native.DeviceCommandStore(0, w.range_start_inclusive, 1, w.slices)
    try:
        st.load(w)
        seg = w.cfk.seg.astype(np.int64)
        k = int(np.argmax(np.diff(seg)))
        e = int(seg[k])                          # right after the key's first id: a mid-segment insert
        t = Tids(w.cfk.txn.msb[[e]], w.cfk.txn.lsb[[e]], np.array([w.cfk.txn.node[e] + 100], np.int32))
        x = Tids(w.cfk.txn.msb[[e]], w.cfk.txn.lsb[[e]], np.array([w.cfk.txn.node[e] + 200], np.int32))
        u = CfkUpdates(np.array([w.cfk.keys[k]]), t, x, np.array([A.ST_ACCEPTED], np.uint8))
        new, _ = U.cfk_update(w.cfk, u)
        _, stats = st.cfk_update(u)
        assert new.txn.node[e + 1] == t.node[0] and int(new.seg[k + 1]) - 1 > e + 1
        _check(w, st, oracle, new)
        # a failed batch after a merge: content unchanged, the merged ids stay (no answer changes)
        bad = CfkUpdates(u.keys, Tids(t.msb, t.lsb, t.node + 7), t, np.array([9], np.uint8))   # status 9: invalid
        w.cfk = new
        _unchanged_after_error(w, st, oracle, CfkUpdates(np.r_[u.keys, bad.keys], Tids.concat([bad.txn, bad.txn]),
                                                         Tids.concat([t, t]), np.r_[u.status, bad.status]), A.AD_E_INVAL)
        _check(w, st, oracle, new)
    finally:
        st.close()


def test_insert_duplicate_exec_rolls_back(oracle):
    w = synth.random_small(51)
    w.flags = A.AD_SNAPSHOT
    rng = np.random.default_rng(51)
    st = native.DeviceCommandStore(0, w.range_start_inclusive, 1, w.slices)
    try:
        st.load(w)
        ins = G.fresh_preaccepts(w.cfk, rng, 2, max_keys=1, statuses=(A.ST_APPLIED,))
        k = np.array([w.cfk.keys[0]] * len(ins))
        x = Tids(np.repeat(ins.txn.msb[:1], len(ins)), np.repeat(ins.txn.lsb[:1], len(ins)),
                 np.repeat(ins.txn.node[:1], len(ins)))
        dup = CfkUpdates(k, ins.txn, x, ins.status)
        _unchanged_after_error(w, st, oracle, dup, A.AD_E_DUP_EXEC)
        new, _ = U.cfk_update(w.cfk, ins)
        st.cfk_update(ins)
        _check(w, st, oracle, new)
    finally:
        st.close()


def test_sequential_and_recovery_after_inserts(oracle):
    w = synth.random_small(52, n_range_cmds=0)
    rng = np.random.default_rng(52)
    st = native.DeviceCommandStore(0, w.range_start_inclusive, 1, w.slices)
    try:
        st.load(w)
        ins = G.fresh_preaccepts(w.cfk, rng, 20, statuses=(2, 3, 4))
        new, _ = U.cfk_update(w.cfk, ins)
        st.cfk_update(ins)
        old = w.cfk
        w.cfk = new
        # SEQUENTIAL PreAccepts newer still (ascending, executeAt == txnId)
        from accord_deps.model import Queries
        q = G.fresh_preaccepts(new, rng, 30, epoch=12)
        rows = np.r_[0, np.nonzero(np.diff(q.txn.lsb.astype(np.int64)))[0] + 1]
        off = np.r_[rows, len(q)].astype(np.uint64)
        keys = np.concatenate([np.sort(q.keys[int(off[i]):int(off[i + 1])]) for i in range(len(rows))])
        w.queries = Queries(q.txn.take(rows), q.txn.take(rows), off, keys)
        try:
            w.flags = A.AD_SEQUENTIAL             # the host copy follows the device before inserting the batch
            exp = oracle.resolve(w)
            got = st.calculate_partial_deps(w.queries, A.AD_SEQUENTIAL)
            ok, why = got.equals(exp, detail=True)
            assert ok, why
        finally:
            w.cfk = old
    finally:
        st.close()


def _carry_missing(old, new):
    """TxnInfo.missing() of every entry of `new` from its entry in `old` (inserted entries: none)."""
    import ctypes as C  # noqa: F401
    ok = np.repeat(old.keys, np.diff(old.seg.astype(np.int64)))
    nk = np.repeat(new.keys, np.diff(new.seg.astype(np.int64)))
    at = {(int(ok[e]), int(old.txn.msb[e]), int(old.txn.lsb[e]), int(old.txn.node[e])): e for e in range(old.n_entries)}
    off, parts = [0], []
    for e in range(new.n_entries):
        o = at.get((int(nk[e]), int(new.txn.msb[e]), int(new.txn.lsb[e]), int(new.txn.node[e])))
        if o is not None:
            a, b = int(old.miss_off[o]), int(old.miss_off[o + 1])
            parts.append(np.arange(a, b))
            off.append(off[-1] + b - a)
        else:
            off.append(off[-1])
    idx = np.concatenate(parts) if parts else np.zeros(0, np.int64)
    new.miss_off = np.array(off, np.uint64)
    new.miss = old.miss.take(idx.astype(np.int64))
    return new


@pytest.mark.parametrize("seed", range(3))
def test_recovery_after_older_inserts(oracle, seed):
    # recovery views are built from host rank copies: after a dictionary merge they follow the remap
    # (entries, range commands with their recovery facts, prunedBefore)
    import ctypes as C
    w = synth.recovery_workload(5 + seed)
    rng = np.random.default_rng(5 + seed)
    u = G.older_inserts(w.cfk, rng, 40, statuses=(0, 2, 3, 4, 5, 6), w=w)
    new, _ = U.cfk_update(w.cfk, u)
    if U.dup_committed_exec(new):
        pytest.skip("generated batch breaks CommandsForKey.java:1439")
    st = native.DeviceCommandStore(0, w.range_start_inclusive, 1, w.slices)
    try:
        st.load(w)
        _, stats = st.cfk_update(u)
        assert stats["n_keys"][1] > 0                    # ids merged into the dictionary
        with pytest.raises(native.AccordDepsError) as ei:
            st.recovery_scan(w.queries, 0)               # entries moved: missing() lists are stale
        assert ei.value.code == A.AD_E_STATE
        _carry_missing(w.cfk, new)
        st._check(native.lib().ad_cfk_missing_load(st.h, C.byref(new.missing_soa())))
        old = w.cfk
        w.cfk = new
        try:
            for s in A.RECOVER_SCANS:
                ok, why = st.recovery_scan(w.queries, s).equals(oracle.recover(w, s), detail=True)
                assert ok, "scan %d: %s" % (s, why)
        finally:
            w.cfk = old
    finally:
        st.close()


# ---- ballots (CommandsForKey.java:1018-1034; TxnInfo.create :254-262) ---------------------------
def _check_ballots(st, new):
    b = st.cfk_ballots()
    exp = new.ballot
    assert b.msb.tolist() == exp.msb.tolist() and b.lsb.tolist() == exp.lsb.tolist() and b.node.tolist() == exp.node.tolist()


@pytest.mark.parametrize("path", [0, 1])
@pytest.mark.parametrize("seed", range(6))
def test_ballot_replacement(oracle, seed, path):
    # equal-status updates with higher ballots, invalidations outbidding Accepts, ballots carried
    # through insertions (fresh and older ids) and cleared by ballot-free batches
    w = synth.random_small(70 + seed, with_slices=(seed % 3 == 1))
    w.flags = A.AD_SNAPSHOT
    rng = np.random.default_rng(70 + seed)
    if seed % 2:          # a store loaded with ballots
        w.cfk.ballot = G.ballots(rng, w.cfk.n_entries)
        w.cfk.ballot = Tids(np.where(np.isin(w.cfk.status, (2, 3, 4)), w.cfk.ballot.msb, 0).astype(np.uint64),
                            np.where(np.isin(w.cfk.status, (2, 3, 4)), w.cfk.ballot.lsb, 0).astype(np.uint64),
                            np.where(np.isin(w.cfk.status, (2, 3, 4)), w.cfk.ballot.node, 0).astype(np.int32))
    st = native.DeviceCommandStore(0, w.range_start_inclusive, 1, w.slices, path=path)
    try:
        st.load(w)
        cfk = w.cfk
        for rnd in range(4):
            bt, _ = G.ballot_transitions(cfk, rng, 60)
            if rnd == 0:
                u = bt
            elif rnd == 1:
                ins = G.fresh_preaccepts(cfk, rng, 10, epoch=9, statuses=(2, 3, 4))
                ins.ballot = G.ballots(rng, len(ins))
                u = G.concat(bt, ins, ins)
            elif rnd == 2:
                old = G.older_inserts(cfk, rng, 20, w=w)
                old.ballot = G.ballots(rng, len(old))
                u = G.concat(old, bt, old)
            else:
                u, _ = G.transitions(cfk, rng, 40)            # Ballot.ZERO: replacements drop ballots
            new, _ = U.cfk_update(cfk, u)
            if U.dup_committed_exec(new) or _java_would_throw(w, new, oracle):
                continue
            if new.ballot is None:
                new.ballot = Tids(np.zeros(new.n_entries, np.uint64), np.zeros(new.n_entries, np.uint64),
                                  np.zeros(new.n_entries, np.int32))
            st.cfk_update(u)
            _check(w, st, oracle, new)
            _check_ballots(st, new)
            cfk = new
    finally:
        st.close()


def test_ballot_rules_known_answers(oracle):
    # one entry per rule: (status, ballot) over (cur status, cur ballot) -> replaced?
    from accord_deps.model import make_timestamps
    w = synth.random_small(80, n_range_cmds=0)
    w.flags = A.AD_SNAPSHOT
    seg = w.cfk.seg.astype(np.int64)
    k = int(np.argmax(np.diff(seg)))
    es = [e for e in range(int(seg[k]), int(seg[k + 1])) if (int(w.cfk.txn.lsb[e]) & 1) == 0][:6]
    assert len(es) == 6
    hi, lo = make_timestamps(1, 50, 0, 1), make_timestamps(1, 10, 0, 1)
    cur = [(3, hi), (3, lo), (3, lo), (4, lo), (5, lo), (2, lo)]
    w.cfk.status = w.cfk.status.copy()
    bm, bl, bn = (np.zeros(w.cfk.n_entries, np.uint64), np.zeros(w.cfk.n_entries, np.uint64),
                  np.zeros(w.cfk.n_entries, np.int32))
    for e, (s, b) in zip(es, cur):
        w.cfk.status[e] = s
        w.cfk.exec.msb[e], w.cfk.exec.lsb[e], w.cfk.exec.node[e] = w.cfk.txn.msb[e], w.cfk.txn.lsb[e], w.cfk.txn.node[e]
        if s in (2, 3, 4):
            bm[e], bl[e], bn[e] = b.msb[0], b.lsb[0], b.node[0]
    w.cfk.ballot = Tids(bm, bl, bn)
    # updates: ACCEPTED lower ballot (no), ACCEPTED higher (yes), PREACC-invalidate higher over
    # ACCEPTED (yes, executeAt -> txnId), PREACC higher over COMMITTED (no), STABLE equal status
    # (hasInfo, higher: yes), PREACC equal higher (hasInfo via ballot: yes)
    ups = [(3, lo), (3, hi), (2, hi), (2, hi), (5, hi), (2, hi)]
    expect = [False, True, True, False, True, True]
    t = w.cfk.txn.take(es)
    # STABLE keeps no ballot: its equal-status replacement shows in executeAt (a new Timestamp)
    xs = make_timestamps(1, 10 ** 6, 0, 77)
    x = Tids(t.msb.copy(), t.lsb.copy(), t.node.copy())
    x.msb[4], x.lsb[4], x.node[4] = xs.msb[0], xs.lsb[0], xs.node[0]
    u = CfkUpdates(np.full(6, w.cfk.keys[k]), t, x, np.array([s for s, _ in ups], np.uint8),
                   Tids(np.array([b.msb[0] for _, b in ups], np.uint64), np.array([b.lsb[0] for _, b in ups], np.uint64),
                        np.array([b.node[0] for _, b in ups], np.int32)))
    new, n = U.cfk_update(w.cfk, u)
    assert [bool(new.status[e] != w.cfk.status[e] or new.ballot.lsb[e] != w.cfk.ballot.lsb[e] or
                 new.exec.lsb[e] != w.cfk.exec.lsb[e]) for e in es] == expect
    st = native.DeviceCommandStore(0, w.range_start_inclusive, 1, w.slices)
    try:
        st.load(w)
        st.cfk_update(u)
        _check(w, st, oracle, new)
        _check_ballots(st, new)
    finally:
        st.close()


# ---- keys without a CommandsForKey (the update creates one) -------------------------------------
@pytest.mark.parametrize("path", [0, 1])
@pytest.mark.parametrize("seed", range(6))
def test_new_keys(oracle, seed, path):
    # fresh PreAccepts and older ids on keys the store has never seen, mixed with updates of known
    # keys, over rounds: key indices remapped, key hash rebuilt, KeyLines placed incrementally
    # (range commands and their stabbing cells in the store), then deps on every path
    w = synth.random_small(110 + seed, start_inclusive=(seed % 2 == 1))
    w.flags = A.AD_SNAPSHOT
    rng = np.random.default_rng(110 + seed)
    st = native.DeviceCommandStore(0, w.range_start_inclusive, 1, w.slices, path=path)
    try:
        st.load(w)
        cfk = w.cfk
        for rnd in range(3):
            nk = G.unused_keys(cfk, rng, 3 + 4 * rnd)
            ins = G.fresh_preaccepts(cfk, rng, 15, epoch=9 + rnd, statuses=(2, 3, 4, 6), new_keys=nk)
            tr, _ = G.transitions(cfk, rng, 20)
            u = G.concat(tr, ins) if rnd % 2 else G.concat(ins, tr, ins)
            new, _ = U.cfk_update(cfk, u)
            if U.dup_committed_exec(new):
                continue
            _, stats = st.cfk_update(u)
            assert len(new.keys) >= len(cfk.keys)
            # requests over the new keys too
            from accord_deps.model import Queries
            q = w.queries
            keys = np.concatenate([q.keys, nk])
            _check(w, st, oracle, new)
            cfk = new
        # every key the store now holds answers on the lean path
        from accord_deps.model import Queries
        rq = G.fresh_preaccepts(cfk, rng, 40, epoch=20, max_keys=6)
        rows = np.r_[0, np.nonzero(np.diff(rq.txn.lsb.astype(np.int64)))[0] + 1]
        off = np.r_[rows, len(rq)].astype(np.uint64)
        keys = np.concatenate([np.sort(rq.keys[int(off[i]):int(off[i + 1])]) for i in range(len(rows))])
        old_q, old_cfk = w.queries, w.cfk
        w.queries, w.cfk = Queries(rq.txn.take(rows), rq.txn.take(rows), off, keys), cfk
        try:
            exp = oracle.resolve(w)
            got = st.calculate_partial_deps(w.queries, A.AD_SNAPSHOT)
            ok, why = got.equals(exp, detail=True)
            assert ok, why
        finally:
            w.queries, w.cfk = old_q, old_cfk
        _sequential_check(w, st, oracle, cfk, rng, epoch=30)
    finally:
        st.close()


def test_new_keys_recovery_and_empty_store(oracle):
    # recovery views after keys were created; a store loaded empty takes its first keys
    import ctypes as C
    w = synth.recovery_workload(9)
    rng = np.random.default_rng(9)
    nk = G.unused_keys(w.cfk, rng, 5, lo=-(1 << 20), hi=1 << 20)
    u = G.fresh_preaccepts(w.cfk, rng, 10, epoch=9, statuses=(3, 4, 5), new_keys=nk)
    new, _ = U.cfk_update(w.cfk, u)
    st = native.DeviceCommandStore(0, w.range_start_inclusive, 1, w.slices)
    try:
        st.load(w)
        st.cfk_update(u)
        _carry_missing(w.cfk, new)
        st._check(native.lib().ad_cfk_missing_load(st.h, C.byref(new.missing_soa())))
        old = w.cfk
        w.cfk = new
        try:
            for s_ in A.RECOVER_SCANS:
                ok, why = st.recovery_scan(w.queries, s_).equals(oracle.recover(w, s_), detail=True)
                assert ok, "scan %d: %s" % (s_, why)
        finally:
            w.cfk = old
    finally:
        st.close()
