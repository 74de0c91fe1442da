"""CPU restatement of CommandsForKey.update for a batch, on the CfkSnapshot SoA.

TEST INFRASTRUCTURE ONLY: imported by tests/ and bench.py's cpu_baseline leg, as the checker --
never by the product path.

Follows accord-core/src/main/java/accord/local/cfk/CommandsForKey.java:
  * update(Command) :972-980 -> update(newStatus, next, wasPruned) :992-1042, applied in batch order;
  * search: Arrays.binarySearch(byId, txnId) :1001 (byId sorted by Timestamp.compareTo,
    Timestamp.java:208-217; identity = Timestamp.equals :244-249);
  * absent -> insert at -1 - pos with (txnId, newStatus, executeAt) (:1002-1007); a key without a
    CommandsForKey gets a new one (the store creates it before the update);
  * present -> replaced (:1013-1036) iff newStatus > cur.status, or newStatus == cur.status,
    newStatus.hasInfo and the command's ballot > cur.ballot(), or newStatus is
    PREACCEPTED_OR_ACCEPTED_INVALIDATE over an ACCEPTED entry with a higher ballot (an invalidation
    outbidding an Accept); a batch without ballots carries Ballot.ZERO, which never outbids;
  * the replacing TxnInfo (TxnInfo.create :254-262): executeAt = the command's executeAt when
    newStatus.hasExecuteAt() (ACCEPTED..APPLIED), else txnId; ballot = the command's
    acceptedOrCommitted when newStatus.hasBallot (PREACCEPTED_OR_ACCEPTED_INVALIDATE..COMMITTED),
    else Ballot.ZERO (InternalStatus :495-538);
  * prunedBefore is an index into byId here: an insertion at or before it moves it by one.
Not restated (the caller's job, as the ABI documents): the shardRedundantBefore filter (:995),
loadingPruned, TxnInfo.missing() maintenance and the deps-derived additions of
Updating.computeInfoAndAdditions (insertions of TRANSITIVELY_KNOWN ids arrive as their own updates).
"""
import bisect
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "cassandra-accord_amd"))

from accord_deps.model import CfkSnapshot, Tids  # noqa: E402


def norm(msb, lsb, node):
    """Timestamp.compareTo order key (msb unsigned, lsb>>>16, lsb & IDENTITY_FLAGS, node)."""
    msb, lsb = int(msb), int(lsb)
    return (msb, ((lsb >> 16) << 4) | ((lsb >> 1) & 0xF), int(node))


HAS_EXEC = (3, 4, 5, 6)            # InternalStatus.hasExecuteAtOrDeps
HAS_BALLOT = (2, 3, 4)             # InternalStatus.hasBallot
HAS_INFO = (2, 3, 4, 5, 6)         # hasExecuteAtOrDeps | hasBallot
ZERO = (0, 0, 0)                   # Ballot.ZERO


def replaces(st, cur_st, ballot, cur_ballot):
    """CommandsForKey.update's test of whether a status/ballot replaces the entry (:1018-1034)."""
    if st > cur_st:
        return True
    if st < cur_st:
        return st == 2 and cur_st == 3 and norm(*ballot) > norm(*cur_ballot)
    return st in HAS_INFO and norm(*ballot) > norm(*cur_ballot)


def cfk_update(cfk, upd):
    """Returns (new CfkSnapshot, n_applied): `upd` (model.CfkUpdates) applied in order. Ballots:
    cfk.ballot / upd.ballot (Tids, or None = all Ballot.ZERO); the result carries ballots when
    either does."""
    keys = cfk.keys
    seg = cfk.seg.astype(np.int64)
    status = cfk.status.copy()
    em, el, en = cfk.exec.msb.copy(), cfk.exec.lsb.copy(), cfk.exec.node.copy()
    tm, tl, tn = cfk.txn.msb, cfk.txn.lsb, cfk.txn.node
    cb = getattr(cfk, "ballot", None)
    ub = getattr(upd, "ballot", None)
    with_ballots = cb is not None or ub is not None
    ne = len(status)
    bm = cb.msb.copy() if cb is not None else np.zeros(ne, np.uint64)
    bl = cb.lsb.copy() if cb is not None else np.zeros(ne, np.uint64)
    bn = cb.node.copy() if cb is not None else np.zeros(ne, np.int32)
    inserted = {}      # key -> {norm: [txn (m, l, n), exec (m, l, n), status, ballot (m, l, n)]}
    applied = 0
    for i in range(len(upd)):
        key = int(upd.keys[i])
        st = int(upd.status[i])
        t = (int(upd.txn.msb[i]), int(upd.txn.lsb[i]), int(upd.txn.node[i]))
        x = (int(upd.exec.msb[i]), int(upd.exec.lsb[i]), int(upd.exec.node[i])) if st in HAS_EXEC else t
        b = (int(ub.msb[i]), int(ub.lsb[i]), int(ub.node[i])) if ub is not None else ZERO
        sb = b if st in HAS_BALLOT else ZERO
        nt = norm(*t)
        k = int(np.searchsorted(keys, key))
        e = -1
        if k < len(keys) and keys[k] == key:
            lo, hi = int(seg[k]), int(seg[k + 1])
            while lo < hi:                                  # SortedArrays.binarySearch over byId
                m = (lo + hi) >> 1
                if norm(tm[m], tl[m], tn[m]) < nt:
                    lo = m + 1
                else:
                    hi = m
            if lo < int(seg[k + 1]) and norm(tm[lo], tl[lo], tn[lo]) == nt:
                e = lo
        if e >= 0:
            if replaces(st, int(status[e]), b, (int(bm[e]), int(bl[e]), int(bn[e]))):
                status[e] = st
                em[e], el[e], en[e] = x
                bm[e], bl[e], bn[e] = sb
                applied += 1
            continue
        ins = inserted.setdefault(key, {})
        cur = ins.get(nt)
        if cur is None:
            ins[nt] = [t, x, st, sb]
            applied += 1
        elif replaces(st, cur[2], b, cur[3]):
            cur[1], cur[2], cur[3] = x, st, sb
            applied += 1
    if not inserted:
        out = CfkSnapshot(keys.copy(), cfk.seg.copy(), cfk.txn, Tids(em, el, en), status,
                          None if cfk.pruned_before is None else cfk.pruned_before.copy(),
                          cfk.miss_off, cfk.miss)
        if with_ballots:
            out.ballot = Tids(bm, bl, bn)
        return out, applied
    # splice the insertions into byId (new keys included), keeping every key's segment sorted
    all_keys = sorted(set(keys.tolist()) | set(inserted))
    out = {f: [] for f in ("tm", "tl", "tn", "em", "el", "en", "st", "bm", "bl", "bn")}
    new_seg = [0]
    pruned = []
    for key in all_keys:
        k = int(np.searchsorted(keys, key))
        rows = []
        pb = -1
        if k < len(keys) and keys[k] == key:
            for e in range(int(seg[k]), int(seg[k + 1])):
                rows.append((norm(tm[e], tl[e], tn[e]), (tm[e], tl[e], tn[e]), (em[e], el[e], en[e]), status[e],
                             (bm[e], bl[e], bn[e])))
            if cfk.pruned_before is not None and cfk.pruned_before[k] >= 0:
                pb = rows[int(cfk.pruned_before[k])][0]
        for nt, (t, x, st, b) in sorted(inserted.get(key, {}).items()):
            bisect.insort(rows, (nt, t, x, st, b))
        for _, t, x, st, b in rows:
            out["tm"].append(t[0]), out["tl"].append(t[1]), out["tn"].append(t[2])
            out["em"].append(x[0]), out["el"].append(x[1]), out["en"].append(x[2])
            out["bm"].append(b[0]), out["bl"].append(b[1]), out["bn"].append(b[2])
            out["st"].append(st)
        pruned.append(-1 if pb == -1 else [r[0] for r in rows].index(pb))
        new_seg.append(len(out["st"]))
    txn = Tids(np.array(out["tm"], np.uint64), np.array(out["tl"], np.uint64), np.array(out["tn"], np.int32))
    exe = Tids(np.array(out["em"], np.uint64), np.array(out["el"], np.uint64), np.array(out["en"], np.int32))
    res = CfkSnapshot(np.array(all_keys, np.int64), np.array(new_seg, np.uint64), txn, exe,
                      np.array(out["st"], np.uint8),
                      None if cfk.pruned_before is None else np.array(pruned, np.int64))
    if with_ballots:
        res.ballot = Tids(np.array(out["bm"], np.uint64), np.array(out["bl"], np.uint64), np.array(out["bn"], np.int32))
    return res, applied


def dup_committed_exec(cfk):
    """True when a key holds two committed (COMMITTED..APPLIED) entries with one executeAt: the
    CommandsForKey invariant (CommandsForKey.java:1439) an update batch must not break."""
    seg = cfk.seg.astype(np.int64)
    for k in range(len(cfk.keys)):
        seen = set()
        for e in range(seg[k], seg[k + 1]):
            if 4 <= cfk.status[e] <= 6:
                x = norm(cfk.exec.msb[e], cfk.exec.lsb[e], cfk.exec.node[e])
                if x in seen:
                    return True
                seen.add(x)
    return False


# ---- Pruning.maybePrune / pruneBefore (accord-core/src/main/java/accord/local/cfk/Pruning.java) --------
KIND_WRITE = 1
APPLIED, INVALID = 6, 7


def hlc(msb, lsb):
    """Timestamp.hlc() (Timestamp.java:129-131, :328-336): highHlc(msb) | lowHlc(lsb)."""
    return ((int(msb) & 0x7FFF) << 48) | (int(lsb) >> 16)


def cfk_prune(cfk, keys=None, prune_interval=1, min_hlc_delta=0):
    """Returns (new CfkSnapshot, entries removed, keys pruned): CommandsForKey.maybePrune
    (Pruning.java:164-199) for the CommandsForKey of every key in `keys` (None: all), then
    pruneBefore (:205-331) where it applies. Every TxnInfo.missing() is NO_TXNIDS (the device model:
    the lists are not loaded), so an APPLIED entry executing before the new prunedBefore is removed
    (:239-245 with missing == NO_TXNIDS), as is every INVALID_OR_TRUNCATED entry before it (:253-254).
    prunedBefore is an index into the key's byId here (-1: none)."""
    seg = cfk.seg.astype(np.int64)
    nk = len(cfk.keys)
    want = set(int(k) for k in keys) if keys is not None else None
    pb_old = cfk.pruned_before if cfk.pruned_before is not None else np.full(nk, -1, np.int64)
    keep = np.ones(cfk.n_entries, bool)
    pruned = pb_old.copy()
    n_keys_pruned = 0
    tm, tl, tn = cfk.txn.msb, cfk.txn.lsb, cfk.txn.node
    em, el, en = cfk.exec.msb, cfk.exec.lsb, cfk.exec.node

    def tnorm(e):
        return norm(tm[e], tl[e], tn[e])

    def xnorm(e):
        return norm(em[e], el[e], en[e])

    for k in range(nk):
        if want is not None and int(cfk.keys[k]) not in want:
            continue
        lo, hi = int(seg[k]), int(seg[k + 1])
        # committedByExecuteAt (CommandsForKey.java:651-672) and maxAppliedWriteByExecuteAt (:673-679)
        committed = sorted((e for e in range(lo, hi) if 4 <= int(cfk.status[e]) <= 6), key=xnorm)
        maw = len(committed) - 1
        while maw >= 0:
            e = committed[maw]
            if int(cfk.status[e]) == APPLIED and ((int(tl[e]) >> 1) & 7) == KIND_WRITE:
                break
            maw -= 1
        # maybePrune :166-189
        if maw < prune_interval:
            continue
        max_prune_hlc = hlc(em[committed[maw]], el[committed[maw]]) - min_hlc_delta
        i = maw - 1
        while i >= 0:
            e = committed[i]
            if ((int(tl[e]) >> 1) & 7) == KIND_WRITE and hlc(em[e], el[e]) <= max_prune_hlc and int(cfk.status[e]) == APPLIED:
                break
            i -= 1
        if i < 0:
            continue
        npb = committed[i]
        if int(pb_old[k]) >= 0 and tnorm(npb) <= tnorm(lo + int(pb_old[k])):
            continue
        pos = npb - lo                              # insertPos: npb is in byId
        if pos == 0:
            continue
        # pruneBefore :205-260: entries before pos that are INVALID, or APPLIED executing before npb
        removed = []
        for e in range(lo, lo + pos):
            st = int(cfk.status[e])
            if st == INVALID or (st == APPLIED and xnorm(e) < xnorm(npb)):
                removed.append(e)
        if not removed:
            continue                                # pos == retainCount: the CommandsForKey as it was
        keep[removed] = False
        pruned[k] = pos - len(removed)             # npb's index in the new byId
        n_keys_pruned += 1
    idx = np.nonzero(keep)[0]
    new_seg = np.zeros(nk + 1, np.uint64)
    new_seg[1:] = np.cumsum([int(keep[int(seg[k]):int(seg[k + 1])].sum()) for k in range(nk)])
    # prunedBefore indices of keys not pruned here shift by the removals before them (none: a key's
    # removals are all below its new prunedBefore, and other keys' removals are in other segments)
    out = CfkSnapshot(cfk.keys.copy(), new_seg, cfk.txn.take(idx), cfk.exec.take(idx), cfk.status[idx].copy(),
                      pruned if (cfk.pruned_before is not None or n_keys_pruned) else None)
    if getattr(cfk, "ballot", None) is not None:
        out.ballot = cfk.ballot.take(idx)
    return out, int((~keep).sum()), n_keys_pruned
