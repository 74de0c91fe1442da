"""Update batches for the CommandsForKey maintenance tests: status transitions of
entries already in a store, with executeAts the store already knows (the txn's own id or the
executeAt its entries carry), some entries updated several times in one batch."""
import numpy as np

from accord_deps.model import CfkUpdates, Tids


def entry_keys(cfk):
    return np.repeat(cfk.keys, np.diff(cfk.seg.astype(np.int64)))


def transitions(cfk, rng, n, repeat_frac=0.25, statuses=range(8)):
    ne = cfk.n_entries
    e = rng.integers(0, ne, n)
    rep = rng.random(n) < repeat_frac
    if n > 1:
        e[rep] = e[rng.integers(0, n, int(rep.sum()))]
    st = rng.choice(np.array(list(statuses), np.uint8), n)
    # a range-domain id may sit in a CommandsForKey only as TRANSITIVELY_KNOWN / INVALID
    rd = (cfk.txn.lsb[e] & np.uint64(1)) == 1
    st[rd] = np.where(rng.random(int(rd.sum())) < 0.5, 0, 7).astype(np.uint8)
    own = rng.random(n) < 0.5
    ex = Tids(np.where(own, cfk.txn.msb[e], cfk.exec.msb[e]), np.where(own, cfk.txn.lsb[e], cfk.exec.lsb[e]),
              np.where(own, cfk.txn.node[e], cfk.exec.node[e]))
    return CfkUpdates(entry_keys(cfk)[e], cfk.txn.take(e), ex, st), e


def fresh_preaccepts(cfk, rng, n_txns, max_keys=4, epoch=9, hlc0=1, statuses=(2,), new_exec_frac=0.0,
                     kinds=(0, 1, 3), new_keys=None):
    """PreAccepts of txnIds newer than every id of the store (epoch above the store's): each new txn
    on 1..max_keys existing keys, inserted with a status from `statuses`; executeAt = txnId or, for
    `new_exec_frac` of them, a later new Timestamp."""
    from accord_deps.model import make_timestamps, make_txn_ids
    kind = rng.choice(np.array(kinds, np.uint8), n_txns)
    t = make_txn_ids(epoch, hlc0 + np.arange(n_txns) * 3, kind, rng.integers(1, 17, n_txns))
    x = make_timestamps(epoch, hlc0 + np.arange(n_txns) * 3 + 1, t.lsb & np.uint64(0xFFFF), 1 << 25)
    use_x = rng.random(n_txns) < new_exec_frac
    ex = Tids(np.where(use_x, x.msb, t.msb), np.where(use_x, x.lsb, t.lsb), np.where(use_x, x.node, t.node))
    keys, rows = [], []
    pool = cfk.keys if new_keys is None else np.union1d(cfk.keys, np.asarray(new_keys, np.int64))
    for i in range(n_txns):
        kk = rng.choice(pool, min(len(pool), rng.integers(1, max_keys + 1)), replace=False)
        keys.extend(kk.tolist())
        rows.extend([i] * len(kk))
    rows = np.array(rows)
    st = rng.choice(np.array(statuses, np.uint8), len(rows))
    return CfkUpdates(np.array(keys, np.int64), t.take(rows), ex.take(rows), st)


def concat(*us):
    b = None
    if any(u.ballot is not None for u in us):
        z = [Tids(np.zeros(len(u), np.uint64), np.zeros(len(u), np.uint64), np.zeros(len(u), np.int32)) for u in us]
        b = Tids.concat([u.ballot if u.ballot is not None else zz for u, zz in zip(us, z)])
    return CfkUpdates(np.concatenate([u.keys for u in us]), Tids.concat([u.txn for u in us]),
                      Tids.concat([u.exec for u in us]), np.concatenate([u.status for u in us]), b)


def ballots(rng, n, epoch=1, zero_frac=0.2, hlc_span=20):
    """Random Ballots (Timestamp layout; a few equal, some Ballot.ZERO)."""
    from accord_deps.model import make_timestamps
    b = make_timestamps(epoch, rng.integers(1, hlc_span, n), np.zeros(n, np.uint64), rng.integers(1, 4, n))
    z = rng.random(n) < zero_frac
    return Tids(np.where(z, 0, b.msb).astype(np.uint64), np.where(z, 0, b.lsb).astype(np.uint64),
                np.where(z, 0, b.node).astype(np.int32))


def ballot_transitions(cfk, rng, n, statuses=(2, 3, 4, 5, 6)):
    """Transitions that exercise the ballot rules (CommandsForKey.java:1018-1034): many updates of
    few entries with equal statuses, PREACCEPTED_OR_ACCEPTED_INVALIDATE over ACCEPTED, random
    ballots."""
    u, e = transitions(cfk, rng, n, repeat_frac=0.6, statuses=statuses)
    u.ballot = ballots(rng, n)
    return u, e


def below_redundant(keys, t, w):
    """Rows whose txnId is below its key's shardRedundantBefore in workload w's RedundantBefore: the updates
    CommandsForKey.update ignores (CommandsForKey.java:997), which ad_cfk_update leaves to its caller."""
    red, si = w.redundant, bool(w.range_start_inclusive)
    out = np.zeros(len(keys), bool)
    for j in range(len(red.range_start)):
        a, b = int(red.range_start[j]), int(red.range_end[j])
        wm = (int(red.wm.msb[j]), int(red.wm.lsb[j]), int(red.wm.node[j]))
        if wm == (0, 0, 0):
            continue
        inr = ((keys >= a) & (keys < b)) if si else ((keys > a) & (keys <= b))
        for i in np.nonzero(inr)[0]:
            x = (int(t.msb[i]), int(t.lsb[i]), int(t.node[i]))
            out[i] = (x[0], x[1] >> 16, x[1] & 0x1E, x[2]) < (wm[0], wm[1] >> 16, wm[1] & 0x1E, wm[2])
    return out


def older_inserts(cfk, rng, n, known_frac=0.3, new_exec_frac=0.3, statuses=range(8), w=None):
    """Insertions below the newest id of the store: txnIds next to existing ones (same msb and
    flags, another node: ids the dictionary does not hold, landing mid-segment), and for
    `known_frac` of them ids the store holds under another key. executeAt = txnId or, for
    `new_exec_frac`, an unknown Timestamp next to an existing one. With w, the rows below their key's
    shardRedundantBefore are left out, as a caller of ad_cfk_update does (below_redundant)."""
    ne = cfk.n_entries
    e = rng.integers(0, ne, n)
    ek = entry_keys(cfk)
    keys = rng.choice(cfk.keys, n)
    known = rng.random(n) < known_frac
    node = cfk.txn.node[e].astype(np.int64) + np.where(known, 0, 1000 + rng.integers(0, 50, n))
    t = Tids(cfk.txn.msb[e].copy(), cfk.txn.lsb[e].copy(), node.astype(np.int32))
    # a known id goes to a key that does not hold it (else it is an update of that entry)
    keys = np.where(known & (keys == ek[e]), cfk.keys[(np.searchsorted(cfk.keys, ek[e]) + 1) % len(cfk.keys)], keys)
    st = rng.choice(np.array(list(statuses), np.uint8), n)
    rd = (t.lsb & np.uint64(1)) == 1
    st[rd] = np.where(rng.random(int(rd.sum())) < 0.5, 0, 7).astype(np.uint8)
    f = rng.integers(0, ne, n)
    use_x = (rng.random(n) < new_exec_frac) & ~rd
    x = Tids(np.where(use_x, cfk.exec.msb[f], t.msb), np.where(use_x, cfk.exec.lsb[f], t.lsb),
             np.where(use_x, cfk.exec.node[f].astype(np.int64) + 3000 + np.arange(n), t.node).astype(np.int32))
    u = CfkUpdates(keys.astype(np.int64), t, x, st)
    if w is not None:
        keep = np.nonzero(~below_redundant(u.keys, u.txn, w))[0]
        u = CfkUpdates(u.keys[keep], u.txn.take(keep), u.exec.take(keep), u.status[keep])
    return u


def unused_keys(cfk, rng, n, lo=-500, hi=500):
    """n key values in [lo, hi) the store holds no CommandsForKey for."""
    free = np.setdiff1d(np.arange(lo, hi, dtype=np.int64), cfk.keys)
    return np.sort(rng.choice(free, min(n, len(free)), replace=False))
