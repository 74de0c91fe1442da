"""GPU parity of TxnInfo.missing() maintenance and the deps-derived additions on the device
(include/accord_deps.h ad_cfk_update_soa dep_*): batches of CommandsForKey.update
carrying each command's deps on the key, applied by ad_cfk_update, against the oracle's per-update
restatement of Updating.insertOrUpdate (oracle/cfk_update.py cfk_update_missing): the CommandsForKeys
left (keys, segments, TxnIds, statuses, executeAts -- additions included), every entry's missing()
list (ad_cfk_missing), and the four BeginRecovery scans (which read missing()) bit-exact vs the
oracle's mapReduceFull over the oracle's CommandsForKeys, over successive batches."""
import os
import sys

import numpy as np
import pytest

from accord_deps import _abi as A, native, synth
from accord_deps.model import CfkUpdates, Tids, make_txn_ids

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import cfk_update as U  # noqa: E402
import cfk_update_gen as G  # noqa: E402

pytestmark = pytest.mark.gpu


def _norm(m, l, n):
    return U.norm(m, l, n)


_PAST = [1_000_000]


def with_deps(cfk, u, rng, keep=0.7, n_new=2, dep_kinds=(0, 1), esp=0, past_unwitnessed=0, below_pruned=0):
    """Deps per update with a deps status: a `keep` share of the key's ids below the txn's
    depsKnownBefore plus `n_new` ids the store does not hold (some below, some past its ids), all of
    kinds the txn witnesses; then
      * `esp` ExclusiveSyncPoint ids (witnessed by ExclusiveSyncPoints only: the kind the Java lets a
        command depend on without witnessing it, Updating.java:256-259) -- half in the txn's window,
        half past every id of the batch;
      * `past_unwitnessed` ids of a kind the txn does not witness, past every id the key will hold when
        the update runs (epoch 100, rising in batch order): added only because they are past byId's
        end (:253-262);
      * `below_pruned` witnessed ids below the key's prunedBefore that byId lacks: dropped by
        removePrunedAdditions and handed back as LoadPruned (:111-117)."""
    seg = cfk.seg.astype(np.int64)
    by_key = {int(cfk.keys[k]): (int(seg[k]), int(seg[k + 1])) for k in range(len(cfk.keys))}
    pb = {}
    if cfk.pruned_before is not None:
        for k in range(len(cfk.keys)):
            p = int(cfk.pruned_before[k])
            if p >= 0:
                e = int(seg[k]) + p
                pb[int(cfk.keys[k])] = (int(cfk.txn.msb[e]), int(cfk.txn.lsb[e]), int(cfk.txn.node[e]))
    offs, dm, dl, dn = [0], [], [], []
    for i in range(len(u)):
        ids = []
        if int(u.status[i]) in (3, 4, 5, 6):
            lo, hi = by_key.get(int(u.keys[i]), (0, 0))
            for e in range(lo, hi):
                if (int(cfk.txn.lsb[e]) & 1) == 0 and rng.random() < keep:
                    ids.append((int(cfk.txn.msb[e]), int(cfk.txn.lsb[e]), int(cfk.txn.node[e])))
            hlc = int(u.txn.lsb[i]) >> 16
            nw = make_txn_ids(int(u.txn.msb[i]) >> 15, rng.integers(max(1, hlc - 50), hlc + 50, n_new),
                              rng.choice(np.array(dep_kinds, np.uint64), n_new), rng.integers(20, 30, n_new))
            for j in range(n_new):
                ids.append((int(nw.msb[j]), int(nw.lsb[j]), int(nw.node[j])))
            t = (int(u.txn.msb[i]), int(u.txn.lsb[i]), int(u.txn.node[i]))
            # a command's deps hold only kinds it witnesses (Updating.java:243-247 asserts it of the rest)
            ids = [x for x in ids if _norm(*x) != _norm(*t) and U._witnesses(t, x)]
            tk = (t[1] >> 1) & 7
            for j in range(esp):
                if j % 2 == 0:
                    e = make_txn_ids(int(u.txn.msb[i]) >> 15, [int(rng.integers(max(1, hlc - 50), hlc + 50))], [4],
                                     [int(rng.integers(50, 60))])
                else:
                    _PAST[0] += 3
                    e = make_txn_ids(100, [_PAST[0]], [4], [int(rng.integers(50, 60))])
                ids.append((int(e.msb[0]), int(e.lsb[0]), int(e.node[0])))
            unw = [k for k in (0, 1, 2, 3) if not U._witnesses(t, (0, k << 1, 0))]
            for j in range(past_unwitnessed if unw else 0):
                _PAST[0] += 3
                e = make_txn_ids(100, [_PAST[0]], [int(rng.choice(unw))], [int(rng.integers(60, 70))])
                ids.append((int(e.msb[0]), int(e.lsb[0]), int(e.node[0])))
            p = pb.get(int(u.keys[i]))
            if p is not None and below_pruned and tk != 4:
                phlc = p[1] >> 16
                for j in range(below_pruned):
                    e = make_txn_ids(int(p[0]) >> 15, [int(rng.integers(max(1, phlc - 40), phlc))], [1],
                                     [int(rng.integers(70, 80))])
                    ids.append((int(e.msb[0]), int(e.lsb[0]), int(e.node[0])))
            ids = sorted(set(ids), key=lambda x: _norm(*x))
            # one id per Timestamp.equals class
            uniq, seen = [], set()
            for x in ids:
                if _norm(*x) not in seen:
                    seen.add(_norm(*x))
                    uniq.append(x)
            ids = uniq
        for x in ids:
            dm.append(x[0]), dl.append(x[1]), dn.append(x[2])
        offs.append(len(dm))
    return CfkUpdates(u.keys, u.txn, u.exec, u.status, u.ballot, np.array(offs, np.uint64),
                      Tids(np.array(dm, np.uint64), np.array(dl, np.uint64), np.array(dn, np.int32)))


def consistent_missing(cfk, rng, frac=0.5):
    """missing() lists that satisfy CommandsForKey's invariant (Utils.validateMissing,
    Utils.java:42-62): for an entry with deps, a subset of the key's entries below its
    depsKnownBefore, below COMMITTED, that its kind witnesses (the ones its deps would lack)."""
    seg = cfk.seg.astype(np.int64)
    offs, mm, ml, mn = [0], [], [], []
    for k in range(len(cfk.keys)):
        lo, hi = int(seg[k]), int(seg[k + 1])
        for e in range(lo, hi):
            st = int(cfk.status[e])
            if st in (3, 4, 5, 6) and rng.random() < frac:
                t = (int(cfk.txn.msb[e]), int(cfk.txn.lsb[e]), int(cfk.txn.node[e]))
                x = (int(cfk.exec.msb[e]), int(cfk.exec.lsb[e]), int(cfk.exec.node[e]))
                dkb = _norm(*t) if st == 3 else _norm(*x)
                for p in range(lo, hi):
                    q = (int(cfk.txn.msb[p]), int(cfk.txn.lsb[p]), int(cfk.txn.node[p]))
                    if p != e and int(cfk.status[p]) < 4 and _norm(*q) < dkb and U._witnesses(t, q) and rng.random() < 0.5:
                        mm.append(q[0]), ml.append(q[1]), mn.append(q[2])
            offs.append(len(mm))
    cfk.miss_off = np.array(offs, np.uint64)
    cfk.miss = Tids(np.array(mm, np.uint64), np.array(ml, np.uint64), np.array(mn, np.int32))
    return cfk


def _workload(seed, **kw):
    w = synth.recovery_workload(seed, **kw)
    consistent_missing(w.cfk, np.random.default_rng(seed ^ 0xBEEF))
    return w


def _check(w, st, oracle, exp):
    keys, seg, txn, pruned = st.cfk_byid()
    assert keys.tolist() == exp.keys.tolist() and seg.tolist() == exp.seg.tolist()
    assert [_norm(*x) for x in zip(txn.msb, txn.lsb, txn.node)] == [_norm(*x) for x in zip(exp.txn.msb, exp.txn.lsb, exp.txn.node)]
    s, x = st.cfk_entries()
    assert s.tolist() == exp.status.tolist()
    assert x.lsb.tolist() == exp.exec.lsb.tolist() and x.msb.tolist() == exp.exec.msb.tolist()
    off, ms = st.cfk_missing()
    assert off.tolist() == exp.miss_off.tolist(), "missing() list sizes differ"
    assert [_norm(*m) for m in zip(ms.msb, ms.lsb, ms.node)] == [_norm(*m) for m in zip(exp.miss.msb, exp.miss.lsb, exp.miss.node)]
    old = w.cfk
    w.cfk = exp
    try:
        for scan in A.RECOVER_SCANS:
            got = st.recovery_scan(w.queries, scan)
            want = oracle.recover(w, scan)
            ok, why = got.equals(want, detail=True)
            assert ok, "scan %d: %s" % (scan, why)
    finally:
        w.cfk = old


@pytest.mark.parametrize("seed", range(6))
def test_missing_and_additions(oracle, seed):
    w = _workload(60 + seed, n_hist_txns=200)
    rng = np.random.default_rng(seed)
    st = native.DeviceCommandStore(0, w.range_start_inclusive, 1, w.slices)
    try:
        st.load(w)
        cfk = w.cfk
        for rnd in range(3):
            parts = [G.transitions(cfk, rng, 40)[0], G.fresh_preaccepts(cfk, rng, 10, statuses=(2, 3), epoch=9 + rnd,
                                                                         hlc0=1 + 1000 * rnd)]
            if rnd == 1:
                parts.append(G.older_inserts(cfk, rng, 10, w=w))
            u = with_deps(cfk, G.concat(*parts), rng)
            exp, applied, nadd = U.cfk_update_missing(cfk, u, u.dep_off, u.deps)
            if U.dup_committed_exec(exp):
                continue                      # AD_E_DUP_EXEC on both sides: not this test's subject
            n_applied, stats = st.cfk_update(u)
            assert n_applied == applied + nadd and stats["n_keys"][2] == nadd
            _check(w, st, oracle, exp)
            cfk = exp
    finally:
        st.close()


def test_accept_commit_apply_chain(oracle):
    # one wave of PreAccepts, then Accept -> Commit -> Apply with deps (the common life cycle)
    w = _workload(77, n_hist_txns=150)
    rng = np.random.default_rng(77)
    st = native.DeviceCommandStore(0, w.range_start_inclusive, 1, w.slices)
    try:
        st.load(w)
        cfk = w.cfk
        base = G.fresh_preaccepts(cfk, rng, 12, statuses=(2,), kinds=(0, 1))
        for target in (2, 3, 4, 6):
            u = CfkUpdates(base.keys, base.txn, base.txn, np.full(len(base), target, np.uint8))
            u = with_deps(cfk, u, rng, keep=0.8, n_new=1)
            exp, applied, nadd = U.cfk_update_missing(cfk, u, u.dep_off, u.deps)
            st.cfk_update(u)
            _check(w, st, oracle, exp)
            cfk = exp
    finally:
        st.close()


def test_batch_without_deps_hands_lists_back(oracle):
    w = _workload(80, n_hist_txns=150)
    rng = np.random.default_rng(80)
    st = native.DeviceCommandStore(0, w.range_start_inclusive, 1, w.slices)
    try:
        st.load(w)
        u = with_deps(w.cfk, G.transitions(w.cfk, rng, 30, statuses=(3, 4, 5, 6))[0], rng)
        exp, _, _ = U.cfk_update_missing(w.cfk, u, u.dep_off, u.deps)
        st.cfk_update(u)
        _check(w, st, oracle, exp)
        # a status-only batch (no deps) on entries that keep their deps status leaves the lists valid
        keep = np.nonzero(np.isin(exp.status, (5, 6)))[0][:5]
        u2 = CfkUpdates(G.entry_keys(exp)[keep], exp.txn.take(keep), exp.exec.take(keep), np.full(len(keep), 6, np.uint8))
        st.cfk_update(u2)
        off, _ = st.cfk_missing()
        assert len(off) == exp.n_entries + 1
    finally:
        st.close()


@pytest.mark.parametrize("seed", range(6))
def test_unwitnessed_past_end_and_load_pruned(oracle, seed):
    # deps the command's kind does not witness: ExclusiveSyncPoints (in the window and past the end) and
    # other kinds past the key's last id -- inserted exactly when past byId's end as the update sees it
    # (earlier updates of the batch raise it); witnessed deps below prunedBefore come back as LoadPruned
    w = _workload(90 + seed, n_hist_txns=220)
    rng = np.random.default_rng(900 + seed)
    st = native.DeviceCommandStore(0, w.range_start_inclusive, 1, w.slices)
    try:
        st.load(w)
        cfk = w.cfk
        n_lp = n_add = 0
        for rnd in range(3):
            parts = [G.transitions(cfk, rng, 40, statuses=(3, 4, 5, 6))[0],
                     G.fresh_preaccepts(cfk, rng, 12, statuses=(2, 3), epoch=9 + rnd, hlc0=1 + 1000 * rnd,
                                        kinds=(0, 1, 3, 4))]
            u = with_deps(cfk, G.concat(*parts), rng, esp=2, past_unwitnessed=1 + seed % 2, below_pruned=2)
            lp = []
            exp, applied, nadd = U.cfk_update_missing(cfk, u, u.dep_off, u.deps, load_pruned=lp)
            if U.dup_committed_exec(exp):
                continue
            n_applied, stats = st.cfk_update(u)
            assert n_applied == applied + nadd and stats["n_keys"][2] == nadd
            _check(w, st, oracle, exp)
            got = [(i, k, _norm(*t)) for i, k, t in st.cfk_load_pruned()]
            assert got == [(i, k, _norm(*t)) for i, k, t in lp]
            n_lp += len(lp)
            n_add += nadd
            cfk = exp
        assert n_add > 0
    finally:
        st.close()


def test_load_pruned_collected():
    # the generator reaches the LoadPruned path somewhere in the seeds above (guards the test's reach)
    total = 0
    for seed in range(6):
        w = _workload(90 + seed, n_hist_txns=220)
        rng = np.random.default_rng(900 + seed)
        u = with_deps(w.cfk, G.transitions(w.cfk, rng, 40, statuses=(3, 4, 5, 6))[0], rng, below_pruned=2)
        lp = []
        U.cfk_update_missing(w.cfk, u, u.dep_off, u.deps, load_pruned=lp)
        total += len(lp)
    assert total > 0


@pytest.mark.parametrize("seed", range(3))
def test_unwitnessed_non_esp_dep_rejected(oracle, seed):
    # Updating.java:243-247: a dep the command's kind does not witness that falls between the key's byId
    # entries must be an ExclusiveSyncPoint; anything else is the Java's IllegalStateException -> AD_E_PARTIAL
    w = _workload(95 + seed, n_hist_txns=220)
    rng = np.random.default_rng(950 + seed)
    st = native.DeviceCommandStore(0, w.range_start_inclusive, 1, w.slices)
    try:
        st.load(w)
        cfk = w.cfk
        base = G.transitions(cfk, rng, 30, statuses=(3, 4, 5, 6))[0]
        u = with_deps(cfk, base, rng)
        # a Read txn (witnesses Writes only) gets a fresh Read dep inside the key's window
        seg = cfk.seg.astype(np.int64)

        def cur_status(i):
            k = int(np.searchsorted(cfk.keys, u.keys[i]))
            nt = _norm(int(u.txn.msb[i]), int(u.txn.lsb[i]), int(u.txn.node[i]))
            for e in range(int(seg[k]), int(seg[k + 1])):
                if _norm(int(cfk.txn.msb[e]), int(cfk.txn.lsb[e]), int(cfk.txn.node[e])) == nt:
                    return int(cfk.status[e])
            return -1
        # a Read update that applies (a higher status than the entry's) with a deps status
        reads = [i for i in range(len(u)) if (int(u.txn.lsb[i]) >> 1) & 7 == 0 and int(u.status[i]) in (3, 4, 5, 6)
                 and int(u.status[i]) > cur_status(i)]
        assert reads, "generator gave no Read update with a deps status"
        i = reads[0]
        hlc = int(u.txn.lsb[i]) >> 16
        bad = make_txn_ids(int(u.txn.msb[i]) >> 15, [max(1, hlc - 3)], [0], [97])
        ids = [(int(a), int(b), int(c)) for a, b, c in zip(u.deps.msb, u.deps.lsb, u.deps.node)]
        lo, hi = int(u.dep_off[i]), int(u.dep_off[i + 1])
        row = sorted(ids[lo:hi] + [(int(bad.msb[0]), int(bad.lsb[0]), int(bad.node[0]))], key=lambda x: _norm(*x))
        ids = ids[:lo] + row + ids[hi:]
        off = u.dep_off.astype(np.int64).copy()
        off[i + 1:] += 1
        u = type(u)(u.keys, u.txn, u.exec, u.status, u.ballot, off.astype(np.uint64),
                    Tids(np.array([x[0] for x in ids], np.uint64), np.array([x[1] for x in ids], np.uint64),
                         np.array([x[2] for x in ids], np.int32)))
        with pytest.raises(U.UnwitnessedDep):
            U.cfk_update_missing(cfk, u, u.dep_off, u.deps)
        with pytest.raises(native.AccordDepsError) as e:
            st.cfk_update(u)
        # AD_E_PARTIAL, not AD_E_INVAL: the explicit updates stand (a caller must not retry the batch), the
        # failing update is named, no addition was made and the lists ask for a reload
        assert e.value.code == A.AD_E_PARTIAL and "ExclusiveSyncPoint" in str(e.value)
        assert st.cfk_update_status() == (True, i)
        exp, _ = U.cfk_update(cfk, u)
        keys, seg, txn, _ = st.cfk_byid()
        assert np.array_equal(keys, exp.keys) and np.array_equal(seg, exp.seg)
        assert np.array_equal(txn.msb, exp.txn.msb) and np.array_equal(txn.lsb, exp.txn.lsb)
        status, ex = st.cfk_entries()
        assert np.array_equal(status, exp.status) and np.array_equal(ex.lsb, exp.exec.lsb)
        with pytest.raises(native.AccordDepsError) as e2:
            st.cfk_missing()
        assert e2.value.code == A.AD_E_STATE
        # the store still answers, as the oracle over the updated CommandsForKeys
        got = st.calculate_partial_deps(w.queries)
        w2 = type(w)(w.name, exp, w.cmds, w.redundant, w.queries, w.flags, w.params, w.range_start_inclusive, w.slices)
        assert got.equals(oracle.resolve(w2))
    finally:
        st.close()


def _kat_cases():
    """The hand-derived known answers of tests/test_cfk_update_oracle.py (test_kat_*), as (store, updates,
    expect the AD_E_PARTIAL rejection of Updating.java:247)."""
    import test_cfk_update_oracle as K
    W, R, esp = A.KIND_WRITE, A.KIND_READ, A.KIND_EXCLUSIVE_SYNC_POINT
    out = []
    c = K._miss_store()
    off, dp = K._deps([[(60, W)], [(55, esp)]])
    u = K._upd([7, 7], [20, 30], [W, R], [A.ST_ACCEPTED, A.ST_ACCEPTED], [20, 30])
    out.append((c, CfkUpdates(u.keys, u.txn, u.exec, u.status, None, off, dp), False))
    c = K._miss_store()
    c.pruned_before = np.array([1])
    off, dp = K._deps([[(15, W)], [(15, W)]])
    u = K._upd([7, 7], [40, 45], [W, W], [A.ST_ACCEPTED, A.ST_ACCEPTED])
    out.append((c, CfkUpdates(u.keys, u.txn, u.exec, u.status, None, off, dp), False))
    c = K._miss_store()
    off, dp = K._deps([[(10, W), (17, R)]])
    u = K._upd([7], [30], [R], [A.ST_ACCEPTED])
    out.append((c, CfkUpdates(u.keys, u.txn, u.exec, u.status, None, off, dp), True))
    return out


@pytest.mark.parametrize("case", range(3))
def test_hand_derived_kats_on_the_device(case):
    # the same known answers through ad_cfk_update on the GPU: CommandsForKey, LoadPruned, or the rejection
    from accord_deps.model import Queries, RangeCommands, Redundant, Workload
    cfk, u, rejects = _kat_cases()[case]
    z = np.zeros(0, np.uint64)
    q = Queries(Tids(z, z, np.zeros(0, np.int32)), Tids(z, z, np.zeros(0, np.int32)), np.zeros(1, np.uint64),
                np.zeros(0, np.int64))
    w = Workload("kat", cfk, RangeCommands.empty(), Redundant.empty(), q)
    st = native.DeviceCommandStore(0)
    try:
        st.load(w)
        if rejects:
            with pytest.raises(native.AccordDepsError) as e:
                st.cfk_update(u)
            assert e.value.code == A.AD_E_PARTIAL
            assert st.cfk_update_status() == (True, 0)
            return
        lp = []
        exp, applied, nadd = U.cfk_update_missing(cfk, u, u.dep_off, u.deps, load_pruned=lp)
        n_applied, stats = st.cfk_update(u)
        assert n_applied == applied + nadd
        keys, seg, txn, pruned = st.cfk_byid()
        assert seg.tolist() == exp.seg.tolist()
        assert [_norm(*x) for x in zip(txn.msb, txn.lsb, txn.node)] == \
            [_norm(*x) for x in zip(exp.txn.msb, exp.txn.lsb, exp.txn.node)]
        s, _ = st.cfk_entries()
        assert s.tolist() == exp.status.tolist()
        assert [(i, k, _norm(*t)) for i, k, t in st.cfk_load_pruned()] == [(i, k, _norm(*t)) for i, k, t in lp]
    finally:
        st.close()
