"""Pure-Python mirror of the reference semantics, written independently of oracle/refcpu.c,
used only to cross-check the C restatement on small inputs (test infrastructure).

Canonical-model style of the reference's own tests: the deps of a request are computed as
pair SETS (like KeyDepsTest's Map<Key, NavigableSet<TxnId>> model, KeyDepsTest.java:337-346,
and RangeDepsTest's brute-force overlap model, RangeDepsTest.java:95-169), then encoded into
the RelationMultiMap CSR (RelationMultiMap.java:245-257).
"""
import numpy as np

IDENT = 0xFFFFFFFFFFFF001E


def key(t):
    """Timestamp.compareTo as a sort key (Timestamp.java:208-217)."""
    msb, lsb, node = t
    return (msb, lsb >> 16, lsb & 0x1E, node)


def eq(a, b):
    return a[0] == b[0] and ((a[1] ^ b[1]) & IDENT) == 0 and a[2] == b[2]


def kind(t):
    return (t[1] >> 1) & 7


def domain(t):
    return t[1] & 1


WITNESSES = {0: {1}, 2: {1}, 1: {0, 1}, 3: {0, 1}, 4: {0, 1, 3, 4}}


def contains(start_inclusive, s, e, k):
    return (s <= k < e) if start_inclusive else (s < k <= e)


def cfk_active(entries, S, kinds, elide=True, pruned=None):
    """CommandsForKey.mapReduceActive (CommandsForKey.java:910-968) over entries
    [(txnId, status, executeAt)] sorted by txnId."""
    end = sum(1 for t, _, _ in entries if key(t) < key(S))
    committed = sorted([e for e in entries if 4 <= e[1] <= 6], key=lambda e: key(e[2]))
    writes_before = [e for e in committed if kind(e[0]) == 1 and key(e[2]) < key(S)]
    M = writes_before[-1][2] if writes_before else None
    out = []
    for t, st, ex in entries[:end]:
        if kind(t) not in kinds:
            continue
        if st in (0, 7):
            continue
        if st in (4, 5, 6) and elide and M is not None and key(ex) < key(M) and kind(t) in (0, 1):
            continue
        out.append(t)
    if pruned is not None and key(S) <= key(pruned):
        maw = max([i for i, e in enumerate(committed) if e[1] == 6 and kind(e[0]) == 1])
        cand = [i for i in range(maw) if key(committed[i][2]) >= key(S)]
        i = cand[0] if cand else maw
        while kind(committed[i][0]) != 1:
            i += 1
        out.append(committed[i][0])
    return out


def shard_redundant_before(w, k):
    """The shardRedundantBefore of the RedundantBefore entry holding key k (RedundantBefore.get: epochs not read),
    or None."""
    rb, si = w.redundant, w.range_start_inclusive
    for i in range(len(rb.range_start)):
        if contains(si, int(rb.range_start[i]), int(rb.range_end[i]), k):
            wm = (int(rb.wm.msb[i]), int(rb.wm.lsb[i]), int(rb.wm.node[i]))
            return wm if key(wm) > key((0, 0, 0)) else None
    return None


def truncate(w, k, lo, hi):
    """SafeCommandStore.maybeTruncate before key k's CommandsForKey is read (SafeCommandStore.java:165-171,
    CommandsForKey.withRedundantBeforeAtLeast :1317-1341): (first entry index kept, shardRedundantBefore or None).
    Entries below the key's shardRedundantBefore leave; prunedBefore at or below it becomes NO_INFO."""
    wm = shard_redundant_before(w, k)
    if wm is None:
        return lo, None
    c = w.cfk
    e = lo
    while e < hi and key((int(c.txn.msb[e]), int(c.txn.lsb[e]), int(c.txn.node[e]))) < key(wm):
        e += 1
    return e, wm


def slices_of(w, qi):
    """The slice request qi's scan reads (SafeCommandStore.mapReduceActive's `slice`, SafeCommandStore.java:292):
    its slice set (Queries.slice_set into Workload.slice_sets: RangesForEpoch.allBetween results) or the store's
    slices; None = every key."""
    q = w.queries
    k = None if getattr(q, "slice_set", None) is None else int(q.slice_set[qi])
    if k is None or k == 0xFFFFFFFF:
        return None if w.slices is None else [(int(a), int(b)) for a, b in w.slices]
    return [(int(a), int(b)) for a, b in np.asarray(w.slice_sets[k], np.int64).reshape(-1, 2)]


def request_pairs(w, qi, elide=True):
    """(keyDeps, rangeDeps, directKeyDeps) pair sets of PreAccept.calculatePartialDeps."""
    q = w.queries
    txn = (int(q.txn.msb[qi]), int(q.txn.lsb[qi]), int(q.txn.node[qi]))
    ex = (int(q.exec.msb[qi]), int(q.exec.lsb[qi]), int(q.exec.node[qi]))
    keys = [int(k) for k in q.keys[int(q.key_off[qi]):int(q.key_off[qi + 1])]]
    min_epoch = 0 if q.min_epoch is None else int(q.min_epoch[qi])
    kinds = WITNESSES[kind(txn)]
    p1 = None if eq(ex, txn) else txn
    si = w.range_start_inclusive

    own = slices_of(w, qi)

    def in_slice(k):
        if own is None:
            return True
        return any(contains(si, a, b, k) for a, b in own)

    # a Range-domain request (ranges_of non-empty): its keys are every CommandsForKey key inside one of
    # its ranges and inside the request's slices (InMemoryCommandStore.mapReduceForKey, case Range,
    # InMemoryCommandStore.java:289-304) -- a key is in a sliced range iff it is in both
    ranges = q.ranges_of(qi)
    slices = [(None, None)] if own is None else own
    kd, rd, dd = set(), set(), set()
    cfk = w.cfk
    kidx = {int(k): i for i, k in enumerate(cfk.keys)}
    if ranges:
        keys = [int(k) for k in cfk.keys if any(contains(si, a, b, int(k)) for a, b in ranges)]
    for k in keys:
        if not in_slice(k) or k not in kidx:
            continue
        i = kidx[k]
        s0, s1 = int(cfk.seg[i]), int(cfk.seg[i + 1])
        t0, wm = truncate(w, k, s0, s1)
        pruned = None
        if cfk.pruned_before is not None and cfk.pruned_before[i] >= 0:
            e = s0 + int(cfk.pruned_before[i])
            pruned = (int(cfk.txn.msb[e]), int(cfk.txn.lsb[e]), int(cfk.txn.node[e]))
            if wm is not None and key(wm) >= key(pruned):
                pruned = None
        ents = [((int(cfk.txn.msb[e]), int(cfk.txn.lsb[e]), int(cfk.txn.node[e])), int(cfk.status[e]),
                 (int(cfk.exec.msb[e]), int(cfk.exec.lsb[e]), int(cfk.exec.node[e]))) for e in range(t0, s1)]
        for t in cfk_active(ents, ex, kinds, elide, pruned):
            if p1 is not None and eq(t, p1):
                continue
            (kd if kind(t) in (0, 1) else dd).add((k, key(t), t))
    sliced = [k for k in keys if in_slice(k)]
    c = w.cmds
    for ci in range(len(c.txn)):
        t = (int(c.txn.msb[ci]), int(c.txn.lsb[ci]), int(c.txn.node[ci]))
        hist = c.historical is not None and c.historical[ci]
        if not hist and c.erased is not None and c.erased[ci]:
            continue
        if key(t) >= key(ex) or kind(t) not in kinds:
            continue
        if p1 is not None and eq(t, p1):
            continue
        for r in range(int(c.range_off[ci]), int(c.range_off[ci + 1])):
            s, e = int(c.range_start[r]), int(c.range_end[r])
            if ranges:
                # the command's range meets a request range inside a slice: three half-open intervals
                # of one kind share a point iff the largest start is below the smallest end
                hit = any(max(s, a, s if sa is None else sa) < min(e, b, e if sb is None else sb)
                          for a, b in ranges for sa, sb in slices)
            else:
                hit = any(contains(si, s, e, k) for k in sliced)
            if hit:
                rd.add(((s, e), key(t), t))
    rb = w.redundant
    ep = ex[0] >> 15
    for i in range(len(rb.range_start)):
        s, e = int(rb.range_start[i]), int(rb.range_end[i])
        wm = (int(rb.wm.msb[i]), int(rb.wm.lsb[i]), int(rb.wm.node[i]))
        if ranges:
            if not any(max(s, a) < min(e, b) for a, b in ranges):      # unsliced request ranges
                continue
        elif not any(contains(si, s, e, k) for k in keys):
            continue
        if ep < int(rb.start_epoch[i]) or min_epoch >= int(rb.end_epoch[i]):
            continue
        if key(wm) > key((0, 0, 0)):
            rd.add(((s, e), key(wm), wm))
    return kd, rd, dd


def csr(pairs):
    """RelationMultiMap CSR of a pair set: sorted keys with >= 1 value, sorted unique values,
    keysToValues = [absolute end offsets starting at nKeys] + value indices."""
    keys = sorted({p[0] for p in pairs})
    vals = sorted({(p[1], p[2]) for p in pairs})
    vindex = {v[0]: i for i, v in enumerate(vals)}
    out = []
    body = []
    for k in keys:
        idx = sorted(vindex[p[1]] for p in pairs if p[0] == k)
        body.extend(idx)
        out.append(len(keys) + len(body))
    return keys, [v[1] for v in vals], out + body


def levels_by_rounds(g):
    """Apply rounds of a waitingOn graph, by direct simulation (independent of rc_levels): in
    round r every txn applies whose waits (every earlier-executing txn on a shared key whose kind
    it witnesses, Txn.java:221-235, and every earlier-executing direct dep) all applied before r."""
    import numpy as np
    n = len(g.kind)
    order = np.lexsort(g.exec.order_key())
    pos = np.empty(n, np.int64)
    pos[order] = np.arange(n)
    waits = [set() for _ in range(n)]
    by_key = {}
    for t in range(n):
        for k in g.keys[int(g.key_off[t]):int(g.key_off[t + 1])]:
            by_key.setdefault(int(k), []).append(t)
    for ts in by_key.values():
        ts.sort(key=lambda t: pos[t])
        for j, t in enumerate(ts):
            w = WITNESSES.get(int(g.kind[t]), set())
            for p in ts[:j]:
                if int(g.kind[p]) in w:
                    waits[t].add(p)
    if g.dep_off is not None:
        for t in range(n):
            for d in g.deps[int(g.dep_off[t]):int(g.dep_off[t + 1])]:
                if pos[int(d)] < pos[t]:
                    waits[t].add(int(d))
    level = np.full(n, -1)
    r = 0
    done = 0
    while done < n:
        ready = [t for t in range(n) if level[t] < 0 and all(0 <= level[p] < r for p in waits[t])]
        for t in ready:
            level[t] = r
        done += len(ready)
        r += 1
    return level


def rmap_value(m, k):
    """The value of ReducingRangeMap m at key k (ReducingIntervalMap.find, ReducingIntervalMap.java:
    176-182): interval i = #starts <= k minus one ([s_i, s_i+1) intervals) or #starts < k minus
    one ((s_i, s_i+1] intervals); None outside the map or for a null value."""
    if m is None or len(m) == 0:
        return None
    st = [int(x) for x in m.starts]
    i = sum(1 for s in st if (s < k if m.inclusive_ends else s <= k)) - 1
    if i < 0 or i >= len(m):
        return None
    if m.present is not None and not m.present[i]:
        return None
    return (int(m.values.msb[i]), int(m.values.lsb[i]), int(m.values.node[i]))


def preaccept_model(mc, rb, q, permit_fast_path=1, node_epoch=0):
    """CommandStore.preaccept (CommandStore.java:322-347) without the clock, key by key:
    -> list of (minNonConflicting (msb, lsb, node), AD_PA_* flags)."""
    out = []
    for t in range(len(q)):
        txn = (int(q.txn.msb[t]), int(q.txn.lsb[t]), int(q.txn.node[t]))
        ks = [int(k) for k in q.keys[int(q.key_off[t]):int(q.key_off[t + 1])]]
        if any(v is not None and key(v) > key(txn) for v in (rmap_value(rb, k) for k in ks)):
            out.append(((0, 0, 0), 2))
            continue
        if kind(txn) == 4:
            out.append(((0, 0, 0), 4))
            continue
        acc = (0, 0, 0)
        for k in ks:
            v = rmap_value(mc, k)
            if v is not None and key(v) >= key(acc):       # Timestamp::max(value, accumulator)
                acc = v
        fast = permit_fast_path and key(txn) >= key(acc) and (txn[0] >> 15) >= node_epoch
        out.append((acc, 1 if fast else 0))
    return out


WITNESSED_BY = {2: set(), 0: {1, 3, 4}, 1: {0, 1, 3, 4}, 3: {4}, 4: {4}}   # Txn.Kind.witnessedBy, Txn.java:247-262
RECOVER = {0: ("before", False, (3, 4)), 1: ("before", True, (5, 6)),      # BeginRecovery.java:334,348,365,378
           2: ("after", False, (3, 4)), 3: ("any", False, (5, 6))}


def recovery_pairs(w, qi, scan):
    """(keyDeps, directKeyDeps) pair sets of BeginRecovery scan `scan` for request qi: the entries
    CommandsForKey.mapReduceFull (CommandsForKey.java:809-908) visits, from a flat reading of its
    predicates (empty loadingPruned)."""
    q, c = w.queries, w.cfk
    T = (int(q.txn.msb[qi]), int(q.txn.lsb[qi]), int(q.txn.node[qi]))
    keys = [int(k) for k in q.keys[int(q.key_off[qi]):int(q.key_off[qi + 1])]]
    started, with_dep, statuses = RECOVER[scan]
    kinds = WITNESSED_BY[kind(T)]
    si = w.range_start_inclusive
    # a Range-domain request visits every CommandsForKey key inside one of its ranges (and the store's
    # slices, tested below): InMemoryCommandStore.mapReduceForKey, case Range (:289-304)
    ranges = q.ranges_of(qi)
    if ranges:
        keys = [int(k) for k in c.keys if any(contains(si, a, b, int(k)) for a, b in ranges)]
    own = slices_of(w, qi)
    kd, dd = set(), set()
    for k in keys:
        if own is not None and not any(contains(si, a, b, k) for a, b in own):
            continue
        pos = np.searchsorted(c.keys, k)
        if pos >= len(c.keys) or c.keys[pos] != k:
            continue
        t0, wm = truncate(w, k, int(c.seg[pos]), int(c.seg[pos + 1]))
        cut = t0 > int(c.seg[pos])
        ents = range(t0, int(c.seg[pos + 1]))
        tid = lambda e: (int(c.txn.msb[e]), int(c.txn.lsb[e]), int(c.txn.node[e]))  # noqa: E731
        known = any(eq(tid(e), T) for e in ents)
        if with_dep and not known:
            pb = None
            if c.pruned_before is not None and c.pruned_before[pos] >= 0:
                pb = tid(int(c.seg[pos]) + int(c.pruned_before[pos]))
                if wm is not None and key(wm) >= key(pb):
                    pb = None
            if pb is None or not key(T) < key(pb):
                continue
        for e in ents:
            t = tid(e)
            if started == "before" and not key(t) < key(T):
                continue
            if started == "after" and key(t) < key(T):
                continue
            if kind(t) not in kinds or int(c.status[e]) not in statuses:
                continue
            ex = (int(c.exec.msb[e]), int(c.exec.lsb[e]), int(c.exec.node[e]))
            if not key(ex) > key(T):
                continue
            miss = []
            if c.miss_off is not None:
                m0, m1 = int(c.miss_off[e]), int(c.miss_off[e + 1])
                miss = [(int(c.miss.msb[j]), int(c.miss.lsb[j]), int(c.miss.node[j])) for j in range(m0, m1)]
                if cut:                                      # Utils.removeRedundantMissing (Utils.java:265-275)
                    miss = [m for m in miss if key(m) >= key(wm)]
            has_as_dep = known and not any(eq(m, T) for m in miss)
            if has_as_dep != with_dep:
                continue
            (kd if kind(t) in (0, 1) else dd).add((k, key(t), t))
    return kd, dd


def recovery_range_pairs(w, qi, scan):
    """rangeDeps pairs of BeginRecovery scan `scan` for request qi from the store's live range commands,
    a flat reading of mapReduceRangesInternal's predicates (InMemoryCommandStore.java:884-958) and the
    scan's lambda (BeginRecovery.java:334-380): ((start, end), order key, txnId)."""
    q, cm = w.queries, w.cmds
    out = set()
    if len(cm.txn) == 0:
        return out
    T = (int(q.txn.msb[qi]), int(q.txn.lsb[qi]), int(q.txn.node[qi]))
    keys = [int(k) for k in q.keys[int(q.key_off[qi]):int(q.key_off[qi + 1])]]
    si = w.range_start_inclusive
    own = slices_of(w, qi)
    if own is not None:
        keys = [k for k in keys if any(contains(si, a, b, k) for a, b in own)]
    ranges = q.ranges_of(qi)
    slices = [(None, None)] if own is None else own
    started, with_dep, statuses = RECOVER[scan]
    need = 1 if statuses == (3, 4) else 2                  # AD_RS_PROPOSED / AD_RS_STABLE
    kinds = WITNESSED_BY[kind(T)]
    for i in range(len(cm.txn)):
        if (cm.historical is not None and cm.historical[i]) or (cm.erased is not None and cm.erased[i]):
            continue
        t = (int(cm.txn.msb[i]), int(cm.txn.lsb[i]), int(cm.txn.node[i]))
        ex = (int(cm.rec_exec.msb[i]), int(cm.rec_exec.lsb[i]), int(cm.rec_exec.node[i]))
        if started == "after" and not key(t) > key(T):
            continue
        if started == "before" and not key(t) < key(T):
            continue
        if started in ("before", "any") and key(ex) < key(T):
            continue
        if not int(cm.rec_status[i]) & need or kind(t) not in kinds or not cm.rec_has_deps[i]:
            continue
        d0, d1 = int(cm.rec_dep_off[i]), int(cm.rec_dep_off[i + 1])
        inter = any(eq((int(cm.rec_deps.msb[j]), int(cm.rec_deps.lsb[j]), int(cm.rec_deps.node[j])), T)
                    for j in range(d0, d1))
        if inter != with_dep:
            continue
        if scan == 0 and not key(ex) > key(T):
            continue
        for r in range(int(cm.range_off[i]), int(cm.range_off[i + 1])):
            a, b = int(cm.range_start[r]), int(cm.range_end[r])
            if ranges:
                # the command's range meets a request range inside a slice (three half-open intervals)
                hit = any(max(a, x, a if sa is None else sa) < min(b, y, b if sb is None else sb)
                          for x, y in ranges for sa, sb in slices)
            else:
                hit = any(contains(si, a, b, k) for k in keys)
            if hit:
                out.add(((a, b), key(t), t))
    return out


def sequential_augmented(w):
    """SEQUENTIAL PreAccept semantics as a SNAPSHOT store (extended to Range-domain
    txns): every request, in ascending TxnId order, is registered before its deps are computed
    (PreAccept.java:116-132) -- a key-domain txn CommandsForKey manages goes into each of its keys' byId
    in the store's slices as PREACCEPTED (executeAt = txnId; a present entry below PREACCEPTED is raised,
    CommandsForKey.update :972-1042), a Range-domain txn becomes a live range command over its ranges
    intersected with the slices, less the ranges of the RedundantBefore entries in its epoch bounds whose
    shardAppliedOrInvalidatedBefore is above it (InMemoryCommandStore.java:740-763,
    RedundantBefore.java:216-225). A request only sees registered txns below it (STARTED_BEFORE), so
    registering the whole batch first answers the same. Returns the augmented workload (SNAPSHOT)."""
    from accord_deps.model import CfkSnapshot, RangeCommands, Tids, Workload
    q, c, si = w.queries, w.cfk, w.range_start_inclusive
    slices = None if w.slices is None else [(int(a), int(b)) for a, b in w.slices]
    tup = lambda T, i: (int(T.msb[i]), int(T.lsb[i]), int(T.node[i]))  # noqa: E731
    by_key = {}
    for i, k in enumerate(c.keys):
        s0, s1 = int(c.seg[i]), int(c.seg[i + 1])
        pb = int(c.pruned_before[i]) if c.pruned_before is not None else -1
        ents = [[tup(c.txn, e), int(c.status[e]), tup(c.exec, e), e - s0 == pb] for e in range(s0, s1)]
        by_key[int(k)] = ents
    new_cmds = []
    for qi in range(len(q)):
        t = tup(q.txn, qi)
        ranges = q.ranges_of(qi)
        if ranges:
            rs = []
            for a, b in ranges:
                for sa, sb in (slices or [(a, b)]):
                    lo, hi = max(a, sa), min(b, sb)
                    if lo < hi:
                        rs.append((lo, hi))
            rb = w.redundant
            for j in range(len(rb.range_start)):
                wm = (int(rb.wm.msb[j]), int(rb.wm.lsb[j]), int(rb.wm.node[j]))
                ep = t[0] >> 15
                if ep < int(rb.start_epoch[j]) or ep >= int(rb.end_epoch[j]) or not key(t) < key(wm):
                    continue
                x0, x1 = int(rb.range_start[j]), int(rb.range_end[j])
                out = []
                for a, b in rs:
                    if not (a < x1 and b > x0):
                        out.append((a, b))
                        continue
                    if a < x0:
                        out.append((a, x0))
                    if x1 < b:
                        out.append((x1, b))
                rs = out
            new_cmds.append((t, rs))
            continue
        if domain(t) != 0 or kind(t) not in (0, 1, 3, 4):
            continue
        for k in q.keys[int(q.key_off[qi]):int(q.key_off[qi + 1])]:
            k = int(k)
            if slices is not None and not any(contains(si, a, b, k) for a, b in slices):
                continue
            wm = shard_redundant_before(w, k)
            if wm is not None and key(t) < key(wm):      # CommandsForKey.update ignores it (:997)
                continue
            ents = by_key.setdefault(k, [])
            hit = [e for e in ents if eq(e[0], t)]
            if hit:
                if hit[0][1] < 2:
                    hit[0][1], hit[0][2] = 2, t
            else:
                ents.append([t, 2, t, False])
                ents.sort(key=lambda e: key(e[0]))
    keys = sorted(by_key)
    seg, tx, ex, st, pb = [0], [], [], [], []
    for k in keys:
        ents = by_key[k]
        p = -1
        for j, e in enumerate(ents):
            tx.append(e[0]); st.append(e[1]); ex.append(e[2])
            if e[3]:
                p = j
        pb.append(p)
        seg.append(len(tx))
    T = lambda xs: Tids(np.array([x[0] for x in xs], np.uint64), np.array([x[1] for x in xs], np.uint64),  # noqa: E731
                        np.array([x[2] for x in xs], np.int32))
    cfk = CfkSnapshot(np.array(keys, np.int64), np.array(seg, np.uint64), T(tx), T(ex), np.array(st, np.uint8),
                      np.array(pb, np.int64) if c.pruned_before is not None else None)
    cm = w.cmds
    n0 = len(cm.txn)
    txn = Tids.concat([cm.txn, T([t for t, _ in new_cmds])]) if new_cmds else cm.txn
    off = list(int(x) for x in cm.range_off)
    rs_, re_ = list(int(x) for x in cm.range_start), list(int(x) for x in cm.range_end)
    for _, rs in new_cmds:
        for a, b in rs:
            rs_.append(a); re_.append(b)
        off.append(len(rs_))
    pad = lambda a: None if a is None else np.concatenate([np.asarray(a, np.uint8), np.zeros(len(new_cmds), np.uint8)])  # noqa: E731
    cmds = RangeCommands(txn, np.array(off, np.uint64), np.array(rs_, np.int64), np.array(re_, np.int64),
                         pad(cm.erased) if cm.erased is not None or n0 == 0 else None,
                         pad(cm.historical) if cm.historical is not None or n0 == 0 else None)
    return Workload(w.name + "_aug", cfk, cmds, w.redundant, q, 0, w.params, si, w.slices)


def ranges_with(left, right):
    """Ranges.with (Ranges.java:136-139): AbstractRanges.union(MERGE_OVERLAPPING, left, right) (:486-574) after
    supersetLinearMerge (:429-474), over [(start, end)] lists; touching ranges join only a run that already
    merged an intersection (the Java's `min.start().compareTo(end) > 0` test)."""
    def inter(a, b):
        return 1 if a[0] >= b[1] else (-1 if a[1] <= b[0] else 0)
    if not right or not left:
        return list(left or right)
    A_, B_ = list(left), list(right)
    if A_[0][0] > B_[0][0] or (A_[0][0] == B_[0][0] and A_[-1][1] < B_[-1][1]):
        A_, B_ = B_, A_
    ai = bi = 0
    while ai < len(A_) and bi < len(B_):                    # supersetLinearMerge
        a, b = A_[ai], B_[bi]
        c = inter(a, b)
        if c < 0:
            ai += 1
        elif c > 0 or b[0] < a[0]:
            break
        elif b[1] <= a[1]:
            bi += 1
            ai += b[1] == a[1]
        else:
            t, ok = ai, True
            while True:
                t += 1
                if t == len(A_) or a[1] != A_[t][0]:
                    ok = False
                    break
                a = A_[t]
                if not a[1] < b[1]:
                    break
            if not ok:
                break
            bi, ai = bi + 1, t
    if bi == len(B_):
        return A_
    out = A_[:ai]
    while ai < len(A_) and bi < len(B_):
        a, b = A_[ai], B_[bi]
        c = inter(a, b)
        if c < 0:
            out.append(a)
            ai += 1
        elif c > 0:
            out.append(b)
            bi += 1
        else:
            start, end = min(a[0], b[0]), max(a[1], b[1])
            ai, bi = ai + 1, bi + 1
            while ai < len(A_) or bi < len(B_):
                if ai == len(A_) or (bi < len(B_) and not A_[ai][0] < B_[bi][0]):
                    m, from_a = B_[bi], False
                else:
                    m, from_a = A_[ai], True
                if m[0] > end:
                    break
                end = max(end, m[1])
                if from_a:
                    ai += 1
                else:
                    bi += 1
            out.append((start, end))
    return out + A_[ai:] + B_[bi:]


def range_cmds_update(cmds, upd):
    """The registry after upkeep rows (rc_range_cmds_update's rules: historical merge unless live, erase of a live
    command, update = register or union) as a new RangeCommands, commands in (live, historical) TxnId order."""
    from accord_deps.model import RangeCommands, Tids
    tup = lambda T, i: (int(T.msb[i]), int(T.lsb[i]), int(T.node[i]))  # noqa: E731
    live, hist = {}, {}
    for i in range(len(cmds.txn.msb)):
        rs = [(int(cmds.range_start[j]), int(cmds.range_end[j])) for j in range(int(cmds.range_off[i]), int(cmds.range_off[i + 1]))]
        t = tup(cmds.txn, i)
        if cmds.historical is not None and cmds.historical[i]:
            hist[t] = rs
        else:
            live[t] = [rs, bool(cmds.erased is not None and cmds.erased[i])]
    for i in range(len(upd.txn.msb)):
        t = tup(upd.txn, i)
        rs = [(int(upd.range_start[j]), int(upd.range_end[j])) for j in range(int(upd.range_off[i]), int(upd.range_off[i + 1]))]
        if upd.historical is not None and upd.historical[i]:
            if t not in live:
                hist[t] = ranges_with(hist[t], rs) if t in hist else rs
        elif upd.erased is not None and upd.erased[i]:
            if t in live:
                live[t][1] = True
        else:
            live[t] = [ranges_with(live[t][0], rs), live[t][1]] if t in live else [rs, False]
    rows = [(t, v[0], v[1], False) for t, v in sorted(live.items(), key=lambda x: key(x[0]))] + \
           [(t, v, False, True) for t, v in sorted(hist.items(), key=lambda x: key(x[0]))]
    off = [0]
    st, en = [], []
    for _, rs, _, _ in rows:
        st += [a for a, _ in rs]
        en += [b for _, b in rs]
        off.append(len(st))
    ids = Tids(np.array([r[0][0] for r in rows], np.uint64), np.array([r[0][1] for r in rows], np.uint64),
               np.array([r[0][2] for r in rows], np.int32))
    return RangeCommands(ids, np.array(off, np.uint64), np.array(st, np.int64), np.array(en, np.int64),
                         erased=np.array([r[2] for r in rows], np.uint8), historical=np.array([r[3] for r in rows], np.uint8))
