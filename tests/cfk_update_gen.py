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
