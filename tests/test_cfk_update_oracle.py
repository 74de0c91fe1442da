"""The CommandsForKey.update restatement (oracle/cfk_update.py) on known answers
derived from CommandsForKey.java:992-1042: raise only above the current status, batch order,
insertion at the binarySearch position (with prunedBefore following), new keys."""
import os
import sys

import numpy as np

from accord_deps import _abi as A, synth
from accord_deps.model import CfkSnapshot, CfkUpdates, Tids, make_txn_ids

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import cfk_update as U  # noqa: E402


def _store():
    # key 10: txns hlc 100 (Write, PREACCEPTED), 200 (Read, COMMITTED); key 20: hlc 150 (Write, APPLIED)
    txn = make_txn_ids(1, [100, 200, 150], [A.KIND_WRITE, A.KIND_READ, A.KIND_WRITE], 1)
    return CfkSnapshot(np.array([10, 20]), np.array([0, 2, 3]), txn, txn,
                       np.array([A.ST_PREACCEPTED, A.ST_COMMITTED, A.ST_APPLIED]), np.array([1, -1]))


def _upd(keys, hlcs, kinds, statuses, exec_hlcs=None):
    t = make_txn_ids(1, hlcs, kinds, 1)
    x = t if exec_hlcs is None else make_txn_ids(1, exec_hlcs, kinds, 1)
    return CfkUpdates(np.array(keys), t, x, np.array(statuses))


def test_raise_skip_and_order():
    c = _store()
    # raise 100 to COMMITTED (exec 300), then a lower ACCEPTED (skipped), then STABLE (raises again);
    # 200 stays COMMITTED under an equal COMMITTED
    u = _upd([10, 10, 10, 10], [100, 100, 100, 200], [1, 1, 1, 0],
             [A.ST_COMMITTED, A.ST_ACCEPTED, A.ST_STABLE, A.ST_COMMITTED], [300, 300, 310, 999])
    n, applied = U.cfk_update(c, u)
    assert applied == 2
    assert n.status.tolist() == [A.ST_STABLE, A.ST_COMMITTED, A.ST_APPLIED]
    assert int(n.exec.lsb[0]) >> 16 == 310 and int(n.exec.lsb[1]) >> 16 == 200
    assert n.seg.tolist() == c.seg.tolist()


def test_insert_position_and_pruned():
    c = _store()
    # 50 goes before byId[0] of key 10 (prunedBefore index 1 -> 2), 250 after; 30 is a new key
    u = _upd([10, 10, 30, 10], [250, 50, 400, 50], [1, 0, 1, 0],
             [A.ST_PREACCEPTED, A.ST_TRANSITIVELY_KNOWN, A.ST_ACCEPTED, A.ST_PREACCEPTED])
    n, applied = U.cfk_update(c, u)
    assert applied == 4        # 50 inserted, then raised to PREACCEPTED
    assert n.keys.tolist() == [10, 20, 30]
    assert n.seg.tolist() == [0, 4, 5, 6]
    assert [int(x) >> 16 for x in n.txn.lsb] == [50, 100, 200, 250, 150, 400]
    assert n.status.tolist() == [A.ST_PREACCEPTED, A.ST_PREACCEPTED, A.ST_COMMITTED, A.ST_PREACCEPTED,
                                 A.ST_APPLIED, A.ST_ACCEPTED]
    assert n.pruned_before.tolist() == [2, -1, -1]


def test_identity_is_timestamp_equals():
    # an id equal under Timestamp.equals (same msb, hlc, identity flags, node) finds the entry
    c = _store()
    t = make_txn_ids(1, [100], [A.KIND_WRITE], 1)
    u = CfkUpdates(np.array([10]), t, t, np.array([A.ST_ACCEPTED]))
    n, applied = U.cfk_update(c, u)
    assert applied == 1 and n.n_entries == 3 and n.status[0] == A.ST_ACCEPTED


def test_random_transitions_match_a_per_entry_model():
    # independent model: for every entry, the first update of the highest status above its own
    # (no ballots: Ballot.ZERO never outbids)
    import cfk_update_gen as G
    for seed in range(6):
        w = synth.random_small(seed)
        rng = np.random.default_rng(seed)
        u, e = G.transitions(w.cfk, rng, 80)
        n, applied = U.cfk_update(w.cfk, u)
        exp_st = w.cfk.status.copy()
        exp_x = w.cfk.exec.lsb.copy()
        best = {}
        for i, ent in enumerate(e.tolist()):
            if ent not in best or u.status[i] > u.status[best[ent]]:
                best[ent] = i
        cnt = 0
        for ent, i in best.items():
            if u.status[i] > exp_st[ent]:
                exp_st[ent] = u.status[i]
                # executeAt only for statuses with one (TxnInfo.create, CommandsForKey.java:254-262)
                exp_x[ent] = u.exec.lsb[i] if 3 <= u.status[i] <= 6 else u.txn.lsb[i]
                cnt += 1
        assert n.status.tolist() == exp_st.tolist()
        assert n.exec.lsb.tolist() == exp_x.tolist()
        assert applied >= cnt


def test_ballot_rules():
    # CommandsForKey.java:1018-1034 per case; InternalStatus.hasBallot / hasInfo (:495-538)
    b = lambda h: (1 << 15, h << 16, 1)                      # noqa: E731  Ballot(epoch 1, hlc h)
    z = (0, 0, 0)
    assert U.replaces(4, 3, z, b(9))                          # higher status: always
    assert not U.replaces(3, 3, b(5), b(9)) and U.replaces(3, 3, b(10), b(9))
    assert not U.replaces(3, 3, b(9), b(9))                   # equal ballot: no
    assert U.replaces(2, 3, b(10), b(9))                      # invalidation outbids an Accept
    assert not U.replaces(2, 4, b(10), b(9))                  # ... not a Commit
    assert not U.replaces(1, 2, b(10), z)                     # lower status otherwise: no
    assert not U.replaces(0, 0, b(10), z)                     # TRANSITIVELY_KNOWN has no info
    assert not U.replaces(7, 7, b(10), z)
    assert U.replaces(6, 6, b(10), z)                         # APPLIED hasInfo (executeAt)
    # the replacing TxnInfo: ballot kept only with hasBallot, executeAt only with hasExecuteAt
    c = _store()
    t = make_txn_ids(1, [100], [A.KIND_WRITE], 1)
    x = make_txn_ids(1, [300], [A.KIND_WRITE], 1)
    bt = Tids(np.array([b(7)[0]], np.uint64), np.array([b(7)[1]], np.uint64), np.array([1], np.int32))
    n, _ = U.cfk_update(c, CfkUpdates(np.array([10]), t, x, np.array([A.ST_ACCEPTED]), bt))
    assert int(n.exec.lsb[0]) >> 16 == 300 and int(n.ballot.lsb[0]) == b(7)[1]
    n2, _ = U.cfk_update(n, CfkUpdates(np.array([10]), t, x, np.array([A.ST_STABLE]), bt))
    assert int(n2.ballot.lsb[0]) == 0 and int(n2.exec.lsb[0]) >> 16 == 300
    bt2 = Tids(np.array([b(8)[0]], np.uint64), np.array([b(8)[1]], np.uint64), np.array([1], np.int32))
    n3, _ = U.cfk_update(n, CfkUpdates(np.array([10]), t, x, np.array([A.ST_PREACCEPTED]), bt2))
    assert n3.status[0] == A.ST_PREACCEPTED and int(n3.exec.lsb[0]) == int(t.lsb[0]) and int(n3.ballot.lsb[0]) == b(8)[1]


# ---- Pruning.maybePrune / pruneBefore (Pruning.java:164-331) known answers -----------------------
def _prune_store(rows, pruned=-1):
    """One key (7): rows of (txn hlc, kind, status, executeAt hlc) in byId order."""
    hl = [r[0] for r in rows]
    kinds = [r[1] for r in rows]
    txn = make_txn_ids(1, hl, kinds, 1)
    exe = make_txn_ids(1, [r[3] for r in rows], kinds, 1)
    return CfkSnapshot(np.array([7]), np.array([0, len(rows)]), txn, exe, np.array([r[2] for r in rows]),
                       np.array([pruned]))


W, R = A.KIND_WRITE, A.KIND_READ
AP, ST, CM, PA, INV = A.ST_APPLIED, A.ST_STABLE, A.ST_COMMITTED, A.ST_PREACCEPTED, 7


def _hlcs(c):
    return [int(x) >> 16 for x in c.txn.lsb]


def test_prune_latest_applied_write_before_max():
    # committedByExecuteAt = [W10, R20, W30, W40]; maxAppliedWrite = W40 (index 3 >= interval 1);
    # the latest APPLIED Write before it is W30 -> prunedBefore; W10 and R20 executed before it: gone
    c = _prune_store([(10, W, AP, 10), (20, R, AP, 20), (30, W, AP, 30), (40, W, AP, 40)])
    n, removed, keys = U.cfk_prune(c, None, 1, 0)
    assert (removed, keys) == (2, 1)
    assert _hlcs(n) == [30, 40] and n.pruned_before.tolist() == [0]


def test_prune_interval_and_hlc_delta():
    c = _prune_store([(10, W, AP, 10), (20, R, AP, 20), (30, W, AP, 30), (40, W, AP, 40)])
    assert U.cfk_prune(c, None, 4, 0)[1:] == (0, 0)            # maxAppliedWrite index 3 < 4 (:168)
    assert U.cfk_prune(c, None, 3, 0)[1:] == (2, 1)
    # hlc(W40) - 10 = 30: W30 qualifies; - 11 = 29: only W10 (byId[0]: pos 0, :192-193)
    assert U.cfk_prune(c, None, 1, 10)[1:] == (2, 1)
    assert U.cfk_prune(c, None, 1, 11)[1:] == (0, 0)
    assert U.cfk_prune(c, None, 1, 100)[1:] == (0, 0)          # no candidate (:182-183)


def test_prune_keeps_undecided_committed_and_later_executing():
    # below W50: INVALID goes; PREACCEPTED, STABLE and COMMITTED stay; APPLIED R20 executing after
    # W50 (executeAt 60) stays; APPLIED W15 executing before goes
    c = _prune_store([(10, W, INV, 10), (15, W, AP, 15), (20, R, AP, 60), (25, W, PA, 25), (30, W, ST, 30),
                      (35, R, CM, 35), (50, W, AP, 50), (70, W, AP, 70)])
    n, removed, keys = U.cfk_prune(c, None, 1, 0)
    assert removed == 2 and _hlcs(n) == [20, 25, 30, 35, 50, 70]
    assert n.status.tolist() == [AP, PA, ST, CM, AP, AP] and n.pruned_before.tolist() == [4]


def test_prune_not_beyond_current_pruned_before():
    rows = [(10, W, AP, 10), (20, R, AP, 20), (30, W, AP, 30), (40, W, AP, 40)]
    # prunedBefore already W30 (index 2): the candidate is not above it (:184-185)
    assert U.cfk_prune(_prune_store(rows, pruned=2), None, 1, 0)[1:] == (0, 0)
    # nothing to remove below the candidate: the CommandsForKey stays as it was (:255-256)
    c = _prune_store([(10, W, PA, 10), (30, W, AP, 30), (40, W, AP, 40)])
    n, removed, keys = U.cfk_prune(c, None, 1, 0)
    assert (removed, keys) == (0, 0) and n.pruned_before.tolist() == [-1]


def test_prune_key_list():
    c = _prune_store([(10, W, AP, 10), (20, R, AP, 20), (30, W, AP, 30), (40, W, AP, 40)])
    assert U.cfk_prune(c, [8, 9], 1, 0)[1:] == (0, 0)
    assert U.cfk_prune(c, [7], 1, 0)[1:] == (2, 1)


# ---- TxnInfo.missing() and deps-derived additions (Updating.java:99-470, Utils.java:68-352) -------
def _miss_store():
    # key 7: A(10, W, PREACCEPTED), B(20, W, COMMITTED exec 20), C(30, R, PREACCEPTED)
    c = _prune_store([(10, W, PA, 10), (20, W, CM, 20), (30, R, PA, 30)])
    c.pruned_before = None
    return c


def _ids(hlcs, kinds):
    return make_txn_ids(1, hlcs, kinds, 1)


def _deps(lists):
    """CSR of per-update deps lists of (hlc, kind)."""
    off = np.zeros(len(lists) + 1, np.uint64)
    flat = [d for l in lists for d in l]
    off[1:] = np.cumsum([len(l) for l in lists])
    return off, _ids([d[0] for d in flat], [d[1] for d in flat])


def _miss_of(c, hlc):
    e = _hlcs(c).index(hlc)
    return [int(x) >> 16 for x in c.miss.lsb[int(c.miss_off[e]):int(c.miss_off[e + 1])]]


def test_missing_of_an_accepted_txn_and_additions():
    c = _miss_store()
    # D(40, W) ACCEPTED, deps {A, X(25, W), Y(50, W)}: missing(D) = entries below depsKnownBefore (its
    # txnId) it witnesses, not committed, not in its deps = {C}; additions X (inside the merge) and Y
    # (past byId's end) inserted TRANSITIVELY_KNOWN (:194-287, :364-470)
    off, dp = _deps([[(10, W), (25, W), (50, W)]])
    u = _upd([7], [40], [W], [A.ST_ACCEPTED])
    n, applied, nadd = U.cfk_update_missing(c, u, off, dp)
    assert (applied, nadd) == (1, 2)
    assert _hlcs(n) == [10, 20, 25, 30, 40, 50]
    assert n.status.tolist() == [PA, CM, A.ST_TRANSITIVELY_KNOWN, PA, A.ST_ACCEPTED, A.ST_TRANSITIVELY_KNOWN]
    assert _miss_of(n, 40) == [30] and _miss_of(n, 20) == []


def test_commit_leaves_missing_and_gets_its_own():
    c = _miss_store()
    off, dp = _deps([[(10, W), (25, W), (50, W)], [(10, W), (20, W)]])
    # then C (R) commits at 30 with deps {A, B}: it leaves D's missing (removeSelfMissing /
    # removeFromMissingArrays); its own = below executeAt 30, Writes (a Read witnesses Ws), not
    # committed, not in deps = {X}
    u = _upd([7, 7], [40, 30], [W, R], [A.ST_ACCEPTED, A.ST_COMMITTED], [40, 30])
    n, applied, nadd = U.cfk_update_missing(c, u, off, dp)
    assert _miss_of(n, 40) == [] and _miss_of(n, 30) == [25]


def test_pending_insert_joins_committed_after_and_accepted_after():
    c = _miss_store()
    off, dp = _deps([[(10, W), (25, W), (50, W)], [(10, W), (20, W)], []])
    # T(27, W) PREACCEPTED inserted: joins C (committed, executes at 30 > 27, a Read witnesses a
    # Write) and D (ACCEPTED, 40 > 27) (addToMissingArrays, Utils.java:123-210)
    u = _upd([7, 7, 7], [40, 30, 27], [W, R, W], [A.ST_ACCEPTED, A.ST_COMMITTED, A.ST_PREACCEPTED], [40, 30, 27])
    n, _, _ = U.cfk_update_missing(c, u, off, dp)
    assert _miss_of(n, 30) == [25, 27] and _miss_of(n, 40) == [27]
    # a Read (R 35) is not witnessed by... every kind here: a Write witnesses Reads, so D gets it too;
    # C (a Read) does not
    u2 = _upd([7], [35], [R], [A.ST_PREACCEPTED])
    n2, _, _ = U.cfk_update_missing(n, u2, np.zeros(2, np.uint64), _ids([], []))
    assert _miss_of(n2, 40) == [27, 35] and _miss_of(n2, 30) == [25, 27]


def test_additions_below_pruned_before_are_dropped():
    c = _miss_store()
    c.pruned_before = np.array([1])                  # prunedBefore = B (20)
    off, dp = _deps([[(15, W), (25, W)]])
    u = _upd([7], [40], [W], [A.ST_ACCEPTED])
    n, _, nadd = U.cfk_update_missing(c, u, off, dp)
    assert nadd == 1 and _hlcs(n) == [10, 20, 25, 30, 40] and n.pruned_before.tolist() == [1]


def test_missing_only_for_statuses_with_deps_and_matches_plain_update():
    # without deps the statuses/executeAts equal the plain restatement's
    w = synth.random_small(7)
    rng = np.random.default_rng(7)
    import cfk_update_gen as G
    u, _ = G.transitions(w.cfk, rng, 200)
    a, na = U.cfk_update(w.cfk, u)
    b, nb, nadd = U.cfk_update_missing(w.cfk, u)
    assert na == nb and nadd == 0
    assert a.status.tolist() == b.status.tolist() and a.exec.lsb.tolist() == b.exec.lsb.tolist()
    for e in range(b.n_entries):
        if b.status[e] not in (3, 4, 5, 6):
            assert b.miss_off[e + 1] == b.miss_off[e]


def test_prune_missing_subset_of_merged():
    # R5 pending; W10 and W20 APPLIED each missing R5; W30 (the new prunedBefore) missing nothing.
    # W10's list is not inside {} -> kept, and (executing at its txnId) merged; W20's {R5} is then
    # inside the merged set -> removed (Pruning.java:239-251)
    c = _prune_store([(5, R, PA, 5), (10, W, AP, 10), (20, W, AP, 20), (30, W, AP, 30), (40, W, AP, 40)])
    r5 = _ids([5], [R])
    c.miss_off = np.array([0, 0, 1, 2, 2, 2], np.uint64)
    c.miss = Tids.concat([r5, r5])
    n, removed, keys = U.cfk_prune(c, None, 1, 0)
    assert (removed, keys) == (1, 1)
    assert _hlcs(n) == [5, 10, 30, 40] and n.pruned_before.tolist() == [2]
    assert n.miss_off.tolist() == [0, 0, 1, 1, 1]


def test_unwitnessed_deps_past_end_are_added():
    # Updating.java:210-263: while byId has entries the Java adds only deps the command's kind
    # witnesses (an ExclusiveSyncPoint it does not witness is skipped, :256-259); once byId is
    # exhausted every remaining dep is added (:253-262). C (Read, hlc 30) ACCEPTED with deps
    # {ESP 15, ESP 45, Read 50}: ESP 15 lies inside byId -> skipped; ESP 45 and Read 50 lie past
    # C itself, byId's end -> added although a Read witnesses neither
    c = _miss_store()
    esp, rd = A.KIND_EXCLUSIVE_SYNC_POINT, A.KIND_READ
    off, dp = _deps([[(10, W), (15, esp), (20, W), (45, esp), (50, rd)]])
    u = _upd([7], [30], [R], [A.ST_ACCEPTED])
    n, applied, nadd = U.cfk_update_missing(c, u, off, dp)
    assert (applied, nadd) == (1, 2)
    assert _hlcs(n) == [10, 20, 30, 45, 50]


def test_past_end_moves_with_the_batch():
    # byId's end is the one the update sees: T (Write, 60) inserted earlier in the batch raises it, so
    # C's ESP 55 dep is then inside byId (skipped); without T it would be past the end (added)
    c = _miss_store()
    esp = A.KIND_EXCLUSIVE_SYNC_POINT
    off, dp = _deps([[], [(55, esp)]])
    u = _upd([7, 7], [60, 30], [W, R], [A.ST_PREACCEPTED, A.ST_ACCEPTED])
    _, _, nadd = U.cfk_update_missing(c, u, off, dp)
    assert nadd == 0
    off, dp = _deps([[(55, esp)], []])
    u = _upd([7, 7], [30, 60], [R, W], [A.ST_ACCEPTED, A.ST_PREACCEPTED])
    n, _, nadd = U.cfk_update_missing(c, u, off, dp)
    assert nadd == 1 and 55 in _hlcs(n)


def test_load_pruned_reports_dropped_additions():
    # removePrunedAdditions (Updating.java:111-117): additions below prunedBefore are not inserted and
    # go to Pruning.loadPruned; the LoadPruned post-process (:171) asks the store to load them
    c = _miss_store()
    c.pruned_before = np.array([1])                  # prunedBefore = B (20)
    off, dp = _deps([[(12, W), (15, W), (25, W)]])
    u = _upd([7], [40], [W], [A.ST_ACCEPTED])
    lp = []
    n, _, nadd = U.cfk_update_missing(c, u, off, dp, load_pruned=lp)
    assert nadd == 1
    assert [(i, k, int(t[1]) >> 16) for i, k, t in lp] == [(0, 7, 12), (0, 7, 15)]


def test_kat_non_applied_update_does_not_move_byid_end():
    # Known answer from CommandsForKey.update (:992-1042) + Updating.computeInfoAndAdditions (:210-263),
    # derived by hand: update 0 lowers B (COMMITTED) to ACCEPTED -- not applied (:1013-1036), so its deps
    # never reach computeInfoAndAdditions and byId's last id stays C (30). Update 1 accepts C (a Read) with
    # deps {ESP 55}: the merge loop runs out of byId (10, 20, 30) first, so 55 is past the end and is added
    # without the witness test (:253-262). Had the skipped update counted, its dep 60 would have moved the
    # end past 55 and the ESP would have been skipped (:256-259).
    c = _miss_store()
    esp = A.KIND_EXCLUSIVE_SYNC_POINT
    off, dp = _deps([[(60, W)], [(55, esp)]])
    u = _upd([7, 7], [20, 30], [W, R], [A.ST_ACCEPTED, A.ST_ACCEPTED], [20, 30])
    n, applied, nadd = U.cfk_update_missing(c, u, off, dp)
    assert (applied, nadd) == (1, 1)
    assert _hlcs(n) == [10, 20, 30, 55]
    assert n.status.tolist() == [PA, CM, A.ST_ACCEPTED, A.ST_TRANSITIVELY_KNOWN]


def test_kat_same_dep_below_pruned_before_in_two_updates():
    # removePrunedAdditions (Updating.java:111-117) per update: D (W 40) ACCEPTED adds X (W 15), below
    # prunedBefore B (20) -> dropped, LoadPruned(0, key 7, X); E (W 45) ACCEPTED in the same batch with the
    # same dep: X is still absent from byId -> dropped again, LoadPruned(1, key 7, X). Nothing is inserted
    # below prunedBefore; D and E are.
    c = _miss_store()
    c.pruned_before = np.array([1])
    off, dp = _deps([[(15, W)], [(15, W)]])
    u = _upd([7, 7], [40, 45], [W, W], [A.ST_ACCEPTED, A.ST_ACCEPTED])
    lp = []
    n, applied, nadd = U.cfk_update_missing(c, u, off, dp, load_pruned=lp)
    assert (applied, nadd) == (2, 0)
    assert _hlcs(n) == [10, 20, 30, 40, 45]
    assert [(i, k, int(t[1]) >> 16) for i, k, t in lp] == [(0, 7, 15), (1, 7, 15)]


def test_kat_unwitnessed_non_esp_dep_inside_byid_throws():
    # Updating.java:243-247: C (a Read) accepted with a Read dep (17) that falls between byId entries and is
    # absent: a Read does not witness a Read and it is no ExclusiveSyncPoint -> Invariants.checkState fails
    c = _miss_store()
    off, dp = _deps([[(10, W), (17, R)]])
    u = _upd([7], [30], [R], [A.ST_ACCEPTED])
    try:
        U.cfk_update_missing(c, u, off, dp)
    except U.UnwitnessedDep as e:
        assert e.index == 0 and int(e.dep[1]) >> 16 == 17
    else:
        raise AssertionError("expected the IllegalStateException of Updating.java:247")
