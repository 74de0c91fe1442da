"""Seeded synthetic workloads for the five BASELINE.json configs.

Every generator is deterministic in its seed (numpy PCG64) and honours the invariants the
reference relies on:
  * byId strictly increasing per key (CommandsForKey.java:1438);
  * executeAts of committed entries unique per key (:1439) and never equal to another txnId
    (executeAt node ids live in a range disjoint from txnId node ids, as
    CommandsForKeyTest.java:418-424,449-455 arranges);
  * ids equal under Timestamp.equals are bit-identical;
  * prunedBefore, when set, names an APPLIED Write of the key.
All data is synthetic; key ordinals stand for Key.compareTo order (IntKey-like tokens).
"""
import numpy as np

from . import _abi as A
from .model import (CfkSnapshot, Graph, Queries, RangeCommands, Redundant, Tids, Workload,
                    make_timestamps, make_txn_ids)

EXEC_NODE_BASE = 1 << 24        # executeAt node ids never collide with txnId node ids (1..16)


def splitmix64(x):
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def key_tokens(n_keys, salt):
    """rank r -> i64 token (a bijection, so distinct ranks give distinct keys)."""
    return splitmix64(np.arange(n_keys, dtype=np.uint64) + np.uint64(salt)).view(np.int64)


class Zipf:
    def __init__(self, n, s):
        w = 1.0 / np.power(np.arange(1, n + 1, dtype=np.float64), s)
        self.cdf = np.cumsum(w)
        self.cdf /= self.cdf[-1]
        self.p = w / w.sum()

    def sample(self, rng, size):
        return np.minimum(np.searchsorted(self.cdf, rng.random(size), side="right"), len(self.cdf) - 1)


def distinct_rows(rng, sampler, n_rows, k):
    """n_rows x k samples, each row without duplicates (rejection on dup, SURVEY §8d cfg 2)."""
    out = sampler(rng, (n_rows, k))
    while True:
        s = np.sort(out, axis=1)
        bad = np.nonzero((s[:, 1:] == s[:, :-1]).any(axis=1))[0]
        if len(bad) == 0:
            return out
        out[bad] = sampler(rng, (len(bad), k))


def _segments(key_rank, txn_idx, n_keys_total):
    """Sort (key, txn) entries; return order, per-entry position-from-end, unique keys, seg offsets."""
    order = np.lexsort((txn_idx, key_rank))
    kr = key_rank[order]
    uniq, start, counts = np.unique(kr, return_index=True, return_counts=True)
    seg = np.zeros(len(uniq) + 1, dtype=np.uint64)
    seg[1:] = np.cumsum(counts)
    pos = np.arange(len(kr)) - np.repeat(start, counts)
    from_end = np.repeat(counts, counts) - 1 - pos
    return order, from_end, uniq, seg


def build_history(rng, n_hist_txns, keys_of_txn, token_of_rank, hist_kind, tail_unapplied,
                  epoch=1, hlc0=1, node_base=0):
    """CFK snapshot for history txns j (txnId hlc = hlc0 + j, node 1..16, kind hist_kind[j]):
    every entry APPLIED with executeAt = txnId except the last `tail_unapplied` entries per key,
    drawn from {PREACCEPTED, ACCEPTED, COMMITTED, STABLE}; ACCEPTED/COMMITTED/STABLE carry an
    executeAt bumped by 1..1000 hlc ticks (CommandsForKey.TxnInfo.create, :272-279)."""
    j = np.arange(n_hist_txns, dtype=np.int64)
    txn_node = (rng.integers(1, 17, n_hist_txns) + node_base).astype(np.int32)
    bump = rng.integers(1, 1001, n_hist_txns).astype(np.uint64)
    txn = make_txn_ids(epoch, hlc0 + j.astype(np.uint64), hist_kind, txn_node)
    k = keys_of_txn.shape[1]
    key_rank = keys_of_txn.reshape(-1)
    txn_idx = np.repeat(j, k)
    tok = token_of_rank[key_rank]
    order, from_end, uniq_tok, seg = _segments(tok, txn_idx, None)
    e_txn = txn_idx[order]
    status = np.full(len(e_txn), A.ST_APPLIED, dtype=np.uint8)
    tail = from_end < tail_unapplied
    status[tail] = rng.integers(A.ST_PREACCEPTED, A.ST_STABLE + 1, int(tail.sum())).astype(np.uint8)
    has_exec = (status >= A.ST_ACCEPTED) & (status <= A.ST_STABLE)
    et = txn.take(e_txn)
    flags = et.lsb & np.uint64(0xFFFF)
    hlc = (et.lsb >> np.uint64(16)) | ((et.msb & np.uint64(0x7FFF)) << np.uint64(48))
    bumped = make_timestamps(epoch, hlc + bump[e_txn], flags, EXEC_NODE_BASE + e_txn.astype(np.int64))
    ex = Tids(np.where(has_exec, bumped.msb, et.msb), np.where(has_exec, bumped.lsb, et.lsb),
              np.where(has_exec, bumped.node, et.node))
    return CfkSnapshot(uniq_tok, seg, et, ex, status), txn


def _queries(rng, n_txns, keys_rank, token_of_rank, kinds, hlc0, epoch=1, exec_bump=None):
    node = rng.integers(1, 17, n_txns).astype(np.int32)
    i = np.arange(n_txns, dtype=np.uint64)
    txn = make_txn_ids(epoch, hlc0 + i, kinds, node)
    if exec_bump is None:
        ex = Tids(txn.msb.copy(), txn.lsb.copy(), txn.node.copy())
    else:
        flags = txn.lsb & np.uint64(0xFFFF)
        bumped = make_timestamps(epoch, hlc0 + i + exec_bump.astype(np.uint64), flags,
                                 EXEC_NODE_BASE + (1 << 22) + np.arange(n_txns))
        sel = exec_bump > 0
        ex = Tids(np.where(sel, bumped.msb, txn.msb), np.where(sel, bumped.lsb, txn.lsb),
                  np.where(sel, bumped.node, txn.node))
    tok = token_of_rank[keys_rank]
    tok.sort(axis=1)
    k = tok.shape[1]
    key_off = np.arange(n_txns + 1, dtype=np.uint64) * np.uint64(k)
    return Queries(txn, ex, key_off, tok.reshape(-1))


def _rw_kinds(rng, n, esp_frac=0.0, sync_frac=0.0):
    u = rng.random(n)
    kinds = np.where(u < 0.5, A.KIND_READ, A.KIND_WRITE).astype(np.uint8)
    r = rng.random(n)
    kinds[r < sync_frac] = A.KIND_SYNC_POINT
    kinds[(r >= sync_frac) & (r < sync_frac + esp_frac)] = A.KIND_EXCLUSIVE_SYNC_POINT
    return kinds


def config1(n_txns=10_000, keys_per_txn=4, n_keys=1_000, seed=0xACC0D001):
    """Config 1: 10k txns x 4 keys over 1k uniform keys, single CommandStore, SEQUENTIAL
    (each txn is PreAccepted -- inserted as PREACCEPTED -- before its deps are computed)."""
    rng = np.random.default_rng(seed)
    keys = distinct_rows(rng, lambda r, s: r.integers(0, n_keys, s), n_txns, keys_per_txn)
    kinds = _rw_kinds(rng, n_txns)
    token = np.arange(n_keys, dtype=np.int64)          # IntKey k -> ordinal k
    q = _queries(rng, n_txns, keys, token, kinds, hlc0=1000)
    return Workload("config1", CfkSnapshot.empty(), RangeCommands.empty(), Redundant.empty(), q,
                    flags=A.AD_SEQUENTIAL,
                    params=dict(n_txns=n_txns, keys_per_txn=keys_per_txn, n_keys=n_keys, seed=seed,
                                semantics="SEQUENTIAL"))


def config2(n_txns=1_000_000, keys_per_txn=8, n_keys=1_000_000, n_hist_entries=16_000_000, zipf_s=0.99,
            seed=0xACC0D002, sync_frac=0.02, esp_frac=0.0, tail_unapplied=4):
    """Config 2: 1M txns x 8 Zipf(0.99) keys over 1M keys, 16M-entry CFK history (2M history txns x 8
    keys), SNAPSHOT, Read/Write requests 50/50. 2% of history is SyncPoint; only key-domain
    ExclusiveSyncPoint requests witness SyncPoints (Txn.java:221-235), so `esp_frac` > 0 adds those
    (directKeyDeps; each one returns every SyncPoint of its keys). Default 0: BASELINE config 2
    specifies Read/Write requests only."""
    rng = np.random.default_rng(seed)
    z = Zipf(n_keys, zipf_s)
    token = key_tokens(n_keys, seed)
    n_hist = n_hist_entries // keys_per_txn
    hk = distinct_rows(rng, z.sample, n_hist, keys_per_txn)
    hist_kind = _rw_kinds(rng, n_hist, sync_frac=sync_frac)
    cfk, _ = build_history(rng, n_hist, hk, token, hist_kind, tail_unapplied)
    qk = distinct_rows(rng, z.sample, n_txns, keys_per_txn)
    q = _queries(rng, n_txns, qk, token, _rw_kinds(rng, n_txns, esp_frac=esp_frac), hlc0=n_hist + 2000)
    w = Workload("config2", cfk, RangeCommands.empty(), Redundant.empty(), q,
                 params=dict(n_txns=n_txns, keys_per_txn=keys_per_txn, n_keys=n_keys,
                             n_hist_entries=n_hist * keys_per_txn, zipf_s=zipf_s, seed=seed,
                             sync_frac=sync_frac, esp_frac=esp_frac, semantics="SNAPSHOT"))
    return w


def config2_stream(w, n_batches, n_txns, seed=0xACC0D5EE, held_keys_only=False):
    """Successive config-2 request batches for a steady-state run on the config-2 store `w`: batch b
    holds n_txns fresh PreAccepts (8 Zipf keys each, Read/Write 50/50) whose txnIds follow every id
    of batches < b (hlc ranges after the config's own request batch). `held_keys_only`: Zipf over
    the keys the store holds a CommandsForKey for (same ranks order)."""
    p = w.params
    n_keys, k = int(p["n_keys"]), int(p["keys_per_txn"])
    rng = np.random.default_rng(seed)
    token = key_tokens(n_keys, int(p["seed"]))
    if held_keys_only:
        token = token[np.isin(token, w.cfk.keys)]
        n_keys = len(token)
    z = Zipf(n_keys, float(p["zipf_s"]))
    n_hist = int(p["n_hist_entries"]) // k
    hlc = n_hist + 2000 + int(p["n_txns"]) + 4096
    out = []
    for _ in range(n_batches):
        qk = distinct_rows(rng, z.sample, n_txns, k)
        out.append(_queries(rng, n_txns, qk, token, _rw_kinds(rng, n_txns), hlc0=hlc))
        hlc += n_txns + 16
    return out


def with_range_requests(w, frac, max_keys=8, seed=0xACC0D0A6):
    """The workload `w` with a random `frac` of its requests turned into Range-domain txns (TxnId and
    executeAt domain bit set, TxnId.java:154-157; kind unchanged): each gets one normalised Range
    (keys[i] - 1, keys[i + m]] over the store's sorted keys (m + 1 CommandsForKey, m uniform in
    [0, max_keys)), EndInclusive, in place of its keys -- the shape of a sync point or range read in a
    replica's batch (SafeCommandStore.mapReduceActive over Ranges, SafeCommandStore.java:292)."""
    q = w.queries
    n = len(q)
    rng = np.random.default_rng(seed)
    isr = rng.random(n) < frac
    keys_sorted = np.sort(w.cfk.keys)
    nk = len(keys_sorted)
    key_cnt = np.diff(q.key_off.astype(np.int64))
    keep = np.repeat(~isr, key_cnt)
    new_cnt = np.where(isr, 0, key_cnt)
    key_off = np.zeros(n + 1, np.uint64)
    key_off[1:] = np.cumsum(new_cnt)
    ri = np.nonzero(isr)[0]
    a = rng.integers(0, max(nk - max_keys, 1), len(ri))
    m = rng.integers(0, max_keys, len(ri))
    rs = keys_sorted[a] - 1
    re_ = keys_sorted[np.minimum(a + m, nk - 1)]
    range_off = np.zeros(n + 1, np.uint64)
    range_off[1:] = np.cumsum(isr.astype(np.uint64))
    dom = isr.astype(np.uint64)
    txn = Tids(q.txn.msb, q.txn.lsb | dom, q.txn.node)
    ex = Tids(q.exec.msb, q.exec.lsb | dom, q.exec.node)
    w.queries = Queries(txn, ex, key_off, q.keys[keep], q.min_epoch, range_off, rs.astype(np.int64), re_.astype(np.int64))
    w.name = w.name + "+ranges"
    return w


def with_request_mix(w, accept_frac=0.0, unordered_frac=0.0, unordered_window=2000, seed=0xACC0D0A5):
    """The config-2 workload `w` (history txn j has txnId hlc 1 + j) turned into a replica's mix of
    deps requests (SNAPSHOT semantics), so that the paths besides the newest-request one run:
      * Accept (Accept.java:84-117): Commands.accept ran first, so the txn -- one of the history's
        in-flight txns (an entry PREACCEPTED or ACCEPTED) -- sits in its keys' CommandsForKey as
        ACCEPTED with the proposed executeAt E, newer than every id of the store; the request is
        that txnId over all of its keys, deps computed at S = E with the txnId itself excluded
        (PreAccept.java:261; Accept.calculatePartialDeps, Accept.java:113-117).
      * out-of-order PreAccept: txnId (= executeAt) inside the last `unordered_window` hlc ticks of
        the history, older than the newest entries of busy keys (a coordinator whose clock lags);
        keys and kind unchanged.
      * the rest: fresh PreAccepts newer than everything (config 2 as generated).
    The fractions pick disjoint random subsets of the requests (Accepts capped by the number of
    in-flight history txns)."""
    q = w.queries
    n = len(q)
    rng = np.random.default_rng(seed)
    u = rng.random(n)
    cfk = w.cfk
    n_hist = int(w.params.get("n_hist_entries", w.params.get("n_hist_entries_per_gpu"))) // int(w.params["keys_per_txn"])
    ent_j = (cfk.txn.lsb >> np.uint64(16)).astype(np.int64) - 1
    ent_key = np.repeat(cfk.keys, np.diff(cfk.seg.astype(np.int64)))
    inflight = (cfk.status == A.ST_PREACCEPTED) | (cfk.status == A.ST_ACCEPTED)
    cand = np.unique(ent_j[inflight])
    want = np.nonzero(u < accept_frac)[0]
    n_acc = min(len(want), len(cand))
    ai = np.sort(rng.choice(want, n_acc, replace=False)) if n_acc else np.zeros(0, np.int64)
    acc = np.zeros(n, bool)
    acc[ai] = True
    uno = (u >= accept_frac) & (u < accept_frac + unordered_frac)
    js = rng.choice(cand, n_acc, replace=False) if n_acc else np.zeros(0, np.int64)
    # the accepted txns' entries, grouped by request (ascending keys: entries are in key order)
    req_of_j = np.full(n_hist, -1, np.int64)
    req_of_j[js] = np.arange(n_acc)
    ej = req_of_j[ent_j]
    sel = np.nonzero(ej >= 0)[0]
    sel = sel[np.lexsort((ent_key[sel], ej[sel]))]
    a_cnt = np.bincount(ej[sel], minlength=n_acc)
    a_first = np.zeros(n_acc, np.int64)
    if n_acc:
        a_first[1:] = np.cumsum(a_cnt)[:-1]
    # request ids and keys
    flags = q.txn.lsb & np.uint64(0xFFFF)
    node = q.txn.node.copy()
    msb, lsb = q.txn.msb.copy(), q.txn.lsb.copy()
    ui = np.nonzero(uno)[0]
    win = max(1, int(unordered_window))
    k = np.arange(len(ui), dtype=np.uint64)
    late = make_timestamps(1, np.uint64(max(1, n_hist - win)) + (k % np.uint64(win)), flags[ui],
                           17 + (k // np.uint64(win)).astype(np.int32))
    msb[ui], lsb[ui], node[ui] = late.msb, late.lsb, late.node
    jt = cfk.txn.take(sel[a_first]) if n_acc else cfk.txn.take(np.zeros(0, np.int64))
    msb[ai], lsb[ai], node[ai] = jt.msb, jt.lsb, jt.node
    txn = Tids(msb, lsb, node)
    E = make_timestamps(1, np.uint64(n_hist + 2000 + n + 1000) + np.arange(n_acc, dtype=np.uint64),
                        jt.lsb & np.uint64(0xFFFF), EXEC_NODE_BASE + (1 << 22) + np.arange(n_acc))
    ex = Tids(msb.copy(), lsb.copy(), node.copy())
    ex.msb[ai], ex.lsb[ai], ex.node[ai] = E.msb, E.lsb, E.node
    ko = q.key_off.astype(np.int64)
    cnt = np.diff(ko)
    cnt[ai] = a_cnt
    key_off = np.zeros(n + 1, np.uint64)
    key_off[1:] = np.cumsum(cnt)
    keep_old = ~np.repeat(acc, np.diff(ko))
    dst_old = np.repeat(~acc, cnt)
    keys = np.zeros(int(key_off[-1]), np.int64)
    keys[dst_old] = q.keys[keep_old]
    keys[~dst_old] = ent_key[sel]
    q2 = Queries(txn, ex, key_off, keys, q.min_epoch)
    # Commands.accept: the in-flight entries of an accepted txn become ACCEPTED at E
    st = cfk.status.copy()
    e_msb, e_lsb, e_node = cfk.exec.msb.copy(), cfk.exec.lsb.copy(), cfk.exec.node.copy()
    up = sel[inflight[sel]]
    r = ej[up]
    st[up] = A.ST_ACCEPTED
    e_msb[up], e_lsb[up], e_node[up] = E.msb[r], E.lsb[r], E.node[r]
    cfk2 = CfkSnapshot(cfk.keys, cfk.seg, cfk.txn, Tids(e_msb, e_lsb, e_node), st, cfk.pruned_before)
    p = dict(w.params)
    p.update(accept_frac=accept_frac, unordered_frac=unordered_frac, unordered_window=unordered_window,
             n_accept=int(n_acc), n_unordered=int(len(ui)))
    return Workload(w.name + "_mix", cfk2, w.cmds, w.redundant, q2, w.flags, p, w.range_start_inclusive, w.slices)


def _uniform(h):
    """u64 hash -> float64 in [0, 1)."""
    return (h >> np.uint64(11)).astype(np.float64) * (1.0 / (1 << 53))


def slice_tokens(lo, hi, n, salt):
    """n distinct i64 tokens inside the slice (lo, hi]: one per equal sub-interval, jittered."""
    width = int(hi) - int(lo) - 1
    step = width // n
    off = np.arange(n, dtype=np.uint64) * np.uint64(step) + splitmix64(np.arange(n, dtype=np.uint64) + np.uint64(salt)) % np.uint64(step)
    with np.errstate(over="ignore"):
        return (np.uint64((int(lo) + 1) % (1 << 64)) + off).view(np.int64)


TIMESTAMP_MAX = (0x7FFFFFFFFFFFFFFF, 0x7FFFFFFFFFFFFFFF, 0x7FFFFFFF)   # Timestamp.MAX (Timestamp.java:29)


def with_ephemeral_reads(w, frac=0.3, seed=0xACC0DE4D):
    """GetEphemeralReadDeps requests (GetEphemeralReadDeps.java:76): a share of the batch becomes
    EphemeralRead txns whose deps are computed at executeAt = Timestamp.MAX (msb = lsb = Long.MAX_VALUE,
    node Id.MAX: the flag bits read as kind 7), i.e. every started txn of a key it witnesses."""
    import copy
    rng = np.random.default_rng(seed)
    q = w.queries
    sel = rng.random(len(q)) < frac
    lsb = q.txn.lsb.copy()
    lsb[sel] = (lsb[sel] & ~np.uint64(0xE)) | np.uint64(A.KIND_EPHEMERAL_READ << 1)
    txn = Tids(q.txn.msb.copy(), lsb, q.txn.node.copy())
    em, el, en = q.exec.msb.copy(), q.exec.lsb.copy(), q.exec.node.copy()
    em[sel], el[sel], en[sel] = np.uint64(TIMESTAMP_MAX[0]), np.uint64(TIMESTAMP_MAX[1]), np.int32(TIMESTAMP_MAX[2])
    out = copy.copy(w)
    out.queries = Queries(txn, Tids(em, el, en), q.key_off.copy(), q.keys.copy(), q.min_epoch)
    out.name = w.name + "+ephemeral"
    return out


def config2_sharded(rank, world, n_txns_per_gpu=1_000_000, keys_per_txn=8, n_keys_per_gpu=1_000_000,
                    n_hist_entries_per_gpu=16_000_000, zipf_s=0.99, seed=0xACC0D002, sync_frac=0.02,
                    tail_unapplied=4):
    """Config 2 weak-scaled over `world` GPUs (one CommandStore per GPU, EvenSplit token slices):
    store g owns n_keys_per_gpu keys inside slice g and a config-2 history of its own
    (n_hist_entries_per_gpu entries, 8 Zipf(0.99) keys per history txn, txnIds node-disjoint
    across stores); the batch holds world * n_txns_per_gpu Read/Write requests x 8 distinct keys,
    each key on a uniformly chosen store and Zipf(0.99)-ranked within it, so every store sees the
    config-2 key distribution and ~8 x n_txns_per_gpu probes. At world == 1 this is config 2.
    Returns (Workload of `rank` holding only the requests routed to it, their global indices,
    total number of requests). Deterministic in (seed, world): every rank derives the same batch."""
    lo, hi = shard_bounds(world)
    z = Zipf(n_keys_per_gpu, zipf_s)
    # store `rank`: keys and history
    tok = slice_tokens(lo[rank], hi[rank], n_keys_per_gpu, seed + 7919 * rank)
    rng = np.random.default_rng([seed, world, rank])
    token_of_rank = tok[rng.permutation(n_keys_per_gpu)]
    n_hist = n_hist_entries_per_gpu // keys_per_txn
    hk = distinct_rows(rng, z.sample, n_hist, keys_per_txn)
    cfk, _ = build_history(rng, n_hist, hk, token_of_rank, _rw_kinds(rng, n_hist, sync_frac=sync_frac),
                           tail_unapplied, node_base=16 * rank)
    # the global batch (same on every rank)
    T = world * n_txns_per_gpu
    K = keys_per_txn
    slot = np.arange(T * K, dtype=np.uint64)
    salt = np.uint64(seed * 1000003 + world)
    shard = (splitmix64(slot ^ salt) % np.uint64(world)).reshape(T, K) if world > 1 else np.zeros((T, K), np.uint64)
    rows, cols = np.nonzero(shard == rank)
    loc = rows.astype(np.uint64) * np.uint64(K) + cols.astype(np.uint64)
    zr = np.minimum(np.searchsorted(z.cdf, _uniform(splitmix64(loc + salt * np.uint64(3)))), n_keys_per_gpu - 1)
    # distinct keys per request: re-draw a slot that repeats a key already drawn in its row
    rows = rows.astype(np.int64)
    row_start = np.searchsorted(rows, np.arange(T + 1))        # slots of a row are contiguous
    cand = np.arange(len(rows))
    for rnd in range(1, 64):
        kk = rows[cand] * n_keys_per_gpu + zr[cand]
        o = np.argsort(kk, kind="stable")                      # equal keys: earlier slot first
        ks = kk[o]
        dup = np.zeros(len(o), bool)
        dup[1:] = ks[1:] == ks[:-1]
        if not dup.any():
            break
        bad = cand[o[dup]]
        zr[bad] = np.minimum(np.searchsorted(z.cdf, _uniform(splitmix64(loc[bad] + salt * np.uint64(3 + 2 * rnd)))),
                             n_keys_per_gpu - 1)
        br = np.unique(rows[bad])
        cand = np.concatenate([np.arange(row_start[r], row_start[r + 1]) for r in br]) if len(br) < 4096 else \
            np.nonzero(np.isin(rows, br))[0]
    qrng = np.random.default_rng([seed, world, 1 << 20])
    kinds = _rw_kinds(qrng, T)
    node = qrng.integers(1, 17, T).astype(np.int32)
    hlc0 = n_hist + 2000
    idx = np.unique(rows).astype(np.int64)
    txn = make_txn_ids(1, np.uint64(hlc0) + idx.astype(np.uint64), kinds[idx], node[idx])
    order = np.lexsort((token_of_rank[zr], rows))
    keys = token_of_rank[zr][order]
    counts = np.bincount(rows, minlength=T)[idx]
    key_off = np.zeros(len(idx) + 1, np.uint64)
    key_off[1:] = np.cumsum(counts)
    q = Queries(txn, Tids(txn.msb.copy(), txn.lsb.copy(), txn.node.copy()), key_off, keys)
    w = Workload("config2_sharded", cfk, RangeCommands.empty(), Redundant.empty(), q,
                 params=dict(rank=rank, world=world, n_txns_per_gpu=n_txns_per_gpu, keys_per_txn=K,
                             n_keys_per_gpu=n_keys_per_gpu, n_hist_entries_per_gpu=n_hist * K, zipf_s=zipf_s,
                             seed=seed, sync_frac=sync_frac, semantics="SNAPSHOT"),
                 slices=np.array([[lo[rank], hi[rank]]], dtype=np.int64))
    return w, idx, T


def shard_bounds(n_shards):
    """EvenSplit of the i64 token space (ShardDistributor.EvenSplit, ShardDistributor.java:106-156):
    shard g owns (lo_g, hi_g] in EndInclusive terms; returned as (lo, hi) arrays."""
    lo = [-(1 << 63) + (g * (1 << 64)) // n_shards for g in range(n_shards)]
    hi = [-(1 << 63) + ((g + 1) * (1 << 64)) // n_shards for g in range(n_shards)]
    lo[0] = -(1 << 63)
    hi[-1] = (1 << 63) - 1
    return np.array(lo, dtype=object), np.array(hi, dtype=object)


def cut_bounds(cuts):
    """Slices of the i64 token space cut at the given ascending points: slice g runs from lo_g to hi_g
    (the same shape as shard_bounds, for small workloads whose keys sit near 0)."""
    lo = [-(1 << 63)] + [int(c) for c in cuts]
    hi = [int(c) for c in cuts] + [(1 << 63) - 1]
    return np.array(lo, dtype=object), np.array(hi, dtype=object)


def config3(n_txns=64_000_000, keys_per_txn=4, n_keys=10_000_000, hist_frac=0.75, seed=0xACC0D003,
            tail_unapplied=2):
    """Config 3 (whole job): 64M txns over 10M uniform keys; first 75% are history (APPLIED except the
    last 2 per key), the rest probes, SNAPSHOT. Shard with `slice_workload`."""
    rng = np.random.default_rng(seed)
    token = key_tokens(n_keys, seed)
    n_hist = int(n_txns * hist_frac)
    hk = distinct_rows(rng, lambda r, s: r.integers(0, n_keys, s), n_hist, keys_per_txn)
    cfk, _ = build_history(rng, n_hist, hk, token, _rw_kinds(rng, n_hist), tail_unapplied)
    nq = n_txns - n_hist
    qk = distinct_rows(rng, lambda r, s: r.integers(0, n_keys, s), nq, keys_per_txn)
    q = _queries(rng, nq, qk, token, _rw_kinds(rng, nq), hlc0=n_hist + 2000)
    return Workload("config3", cfk, RangeCommands.empty(), Redundant.empty(), q,
                    params=dict(n_txns=n_txns, keys_per_txn=keys_per_txn, n_keys=n_keys, seed=seed,
                                n_hist_txns=n_hist, semantics="SNAPSHOT"))


def _h(x, salt):
    return splitmix64(np.asarray(x, np.uint64) ^ np.uint64(salt & 0xFFFFFFFFFFFFFFFF))


def _txn_keys(j, n_keys, keys_per_txn, salt):
    """Key ranks of txns j (uint64 array), keys_per_txn distinct uniform draws each, from hashes of
    (j, slot): every rank derives the same keys for the same txn without sharing a random stream."""
    ks = np.empty((len(j), keys_per_txn), np.int64)
    for i in range(keys_per_txn):
        ks[:, i] = (_h(j * np.uint64(keys_per_txn) + np.uint64(i), salt) % np.uint64(n_keys)).astype(np.int64)
    for rnd in range(1, 32):
        srt = np.sort(ks, axis=1)
        rows = np.nonzero((srt[:, 1:] == srt[:, :-1]).any(axis=1))[0]
        if not len(rows):
            break
        sub = ks[rows]
        for i in range(1, keys_per_txn):
            d = (sub[:, i:i + 1] == sub[:, :i]).any(axis=1)
            if d.any():
                jj = j[rows[d]]
                sub[d, i] = (_h(jj * np.uint64(keys_per_txn) + np.uint64(i), salt + 0x9E37 * rnd) % np.uint64(n_keys)).astype(np.int64)
        ks[rows] = sub
    return ks


def config3_shard(rank, world, txns_per_gpu=8_000_000, keys_per_gpu=1_250_000, keys_per_txn=4, hist_frac=0.75,
                  seed=0xACC0D003, tail_unapplied=2, chunk=4_000_000):
    """BASELINE config 3 -- 64M txns over 10M uniform keys, token-range sharded across 8 GPUs, SNAPSHOT --
    weak-scaled to `world` GPUs: world/8 of it (world x 8M txns over world x 1.25M keys), exactly config 3
    at world = 8. The first 75 % of the txns form the history (APPLIED except the last 2 entries per key,
    drawn from PREACCEPTED..STABLE, the proposed/committed ones at an executeAt 1..1000 hlc ticks later),
    the rest is the probe batch. Store `rank` owns EvenSplit token slice `rank` (ShardDistributor.EvenSplit,
    ShardDistributor.java:106-156). Every rank derives the same global txns from hashes (txn j: hlc 1 + j,
    kind and node from its hash, keys from _txn_keys) and keeps only what touches its slice, so no rank
    materialises the whole job. Returns (Workload of this store: its CommandsForKey and the requests
    touching it with their keys restricted to the slice, global request indices, number of requests,
    this store's proposed/committed executeAts for the node's global dictionary)."""
    T = int(txns_per_gpu) * world
    K = int(keys_per_gpu) * world
    H = int(T * hist_frac)
    Q = T - H
    salt = seed * 0x100000001B3 + world
    token = key_tokens(K, seed)
    lo, hi = shard_bounds(world)
    lo_r, hi_r = int(lo[rank]), int(hi[rank])

    def in_slice(tok):     # EndInclusive (lo, hi], as the store's slice (synth.route, slice_workload)
        return (tok > lo_r) & (tok <= hi_r)

    # ---- history entries of this slice
    e_tok, e_j = [], []
    for j0 in range(0, H, chunk):
        j = np.arange(j0, min(H, j0 + chunk), dtype=np.uint64)
        tk = token[_txn_keys(j, K, keys_per_txn, salt)]
        m = in_slice(tk)
        rows, cols = np.nonzero(m)
        e_tok.append(tk[rows, cols])
        e_j.append(j[rows].astype(np.int64))
    e_tok = np.concatenate(e_tok) if e_tok else np.zeros(0, np.int64)
    e_j = np.concatenate(e_j) if e_j else np.zeros(0, np.int64)
    order = np.argsort(e_tok, kind="stable")          # j ascending within a key (generation order)
    e_tok, e_j = e_tok[order], e_j[order]
    uk, start, counts = np.unique(e_tok, return_index=True, return_counts=True)
    seg = np.zeros(len(uk) + 1, np.uint64)
    seg[1:] = np.cumsum(counts)
    pos = np.arange(len(e_tok)) - np.repeat(start, counts)
    from_end = np.repeat(counts, counts) - 1 - pos
    hj = _h(e_j.astype(np.uint64), salt + 1)
    kind = (hj & np.uint64(1)).astype(np.uint8)                      # Read / Write 50/50 (per txn)
    node = (1 + (hj >> np.uint64(8)) % np.uint64(16)).astype(np.int32)
    bump = (1 + (hj >> np.uint64(16)) % np.uint64(1000)).astype(np.uint64)
    txn = make_txn_ids(1, 1 + e_j.astype(np.uint64), kind, node)
    status = np.full(len(e_j), A.ST_APPLIED, np.uint8)
    tail = from_end < tail_unapplied
    he = _h(e_j.astype(np.uint64) * np.uint64(0x10001) + (e_tok.view(np.uint64) & np.uint64(0xFFFF)), salt + 2)
    status[tail] = (A.ST_PREACCEPTED + (he[tail] % np.uint64(4))).astype(np.uint8)
    has_exec = (status >= A.ST_ACCEPTED) & (status <= A.ST_STABLE)
    bumped = make_timestamps(1, 1 + e_j.astype(np.uint64) + bump, kind.astype(np.uint64) << np.uint64(1),
                             EXEC_NODE_BASE + e_j)
    ex = Tids(np.where(has_exec, bumped.msb, txn.msb), np.where(has_exec, bumped.lsb, txn.lsb),
              np.where(has_exec, bumped.node, txn.node))
    cfk = CfkSnapshot(uk, seg, txn, ex, status)
    exec_ids = Tids(bumped.msb[has_exec], bumped.lsb[has_exec], bumped.node[has_exec])
    # ---- the probe batch: requests touching this slice, keys restricted to it (ascending)
    q_tok, q_row = [], []
    for j0 in range(H, T, chunk):
        j = np.arange(j0, min(T, j0 + chunk), dtype=np.uint64)
        tk = token[_txn_keys(j, K, keys_per_txn, salt)]
        m = in_slice(tk)
        rows, cols = np.nonzero(m)
        q_tok.append(tk[rows, cols])
        q_row.append(j[rows].astype(np.int64) - H)
    q_tok = np.concatenate(q_tok) if q_tok else np.zeros(0, np.int64)
    q_row = np.concatenate(q_row) if q_row else np.zeros(0, np.int64)
    o = np.lexsort((q_tok, q_row))
    q_tok, q_row = q_tok[o], q_row[o]
    idx, cnt = np.unique(q_row, return_counts=True)
    key_off = np.zeros(len(idx) + 1, np.uint64)
    key_off[1:] = np.cumsum(cnt)
    jq = (idx + H).astype(np.uint64)
    hq = _h(jq, salt + 1)
    qtxn = make_txn_ids(1, np.uint64(H + 2000) + idx.astype(np.uint64), (hq & np.uint64(1)).astype(np.uint8),
                        (1 + (hq >> np.uint64(8)) % np.uint64(16)).astype(np.int32))
    q = Queries(qtxn, Tids(qtxn.msb.copy(), qtxn.lsb.copy(), qtxn.node.copy()), key_off, q_tok)
    w = Workload("config3_shard", cfk, RangeCommands.empty(), Redundant.empty(), q,
                 params=dict(rank=rank, world=world, n_txns=T, n_keys=K, n_hist_txns=H, keys_per_txn=keys_per_txn,
                             seed=seed, semantics="SNAPSHOT", salt=salt),
                 slices=np.array([[lo_r, hi_r]], dtype=np.int64))
    return w, idx.astype(np.int64), Q, exec_ids


def _pack_c3(t):
    """Order-preserving u64 of config3_shard's ids (epoch 1, hlc < 2^32, identity flags, node < 2^27):
    Timestamp.compareTo order (Timestamp.java:208-217) on these ids."""
    hlc = t.lsb >> np.uint64(16)
    return (hlc << np.uint64(32)) | ((t.lsb & np.uint64(0x1E)) << np.uint64(27)) | t.node.astype(np.uint64)


def config3_global_dict(params, exec_ids):
    """The node's global TxnId dictionary for config3_shard (ShardExchange.install_global_dict's union of
    every store's dictionary, built without gathering the txnIds): every history txnId (all appear in
    some store) and the proposed/committed executeAts every store reported (`exec_ids`: list of Tids),
    ascending and unique. Valid for config3_shard's ids only (_pack_c3)."""
    H = int(params["n_hist_txns"])
    salt = int(params["salt"])
    j = np.arange(H, dtype=np.uint64)
    hj = _h(j, salt + 1)
    txn = make_txn_ids(1, 1 + j, (hj & np.uint64(1)).astype(np.uint8), (1 + (hj >> np.uint64(8)) % np.uint64(16)).astype(np.int32))
    packed = np.concatenate([_pack_c3(txn)] + [_pack_c3(e) for e in exec_ids])
    u = np.unique(packed)
    hlc = u >> np.uint64(32)
    flags = (u >> np.uint64(27)) & np.uint64(0x1E)
    node = (u & np.uint64((1 << 27) - 1)).astype(np.int32)
    return make_timestamps(1, hlc, flags, node)


def config4(n_txns=1_000_000, keys_per_txn=4, n_keys=1_000_000, n_ranges=100_000, n_hist_txns=1_000_000,
            seed=0xACC0D004, log2_min=8, log2_max=20):
    """Config 4: 100k Range-domain Write commands (EndInclusive (s, s+w], s uniform i32, w log-uniform
    in [2^8, 2^20]) older than 1M key txns x 4 uniform keys over 1M i32 key tokens; plus a 1M-txn x 4
    key CFK history (APPLIED except the last 2 per key) so keyDeps and rangeDeps merge. SNAPSHOT."""
    rng = np.random.default_rng(seed)
    token = np.unique(rng.integers(-(1 << 31), (1 << 31) - 1, int(n_keys * 1.1)))
    token = rng.permutation(token)[:n_keys].astype(np.int64)
    start = rng.integers(-(1 << 31), (1 << 31) - 1, n_ranges).astype(np.int64)
    width = np.floor(np.exp2(rng.uniform(log2_min, log2_max, n_ranges))).astype(np.int64)
    node = rng.integers(1, 17, n_ranges).astype(np.int32)
    rtx = make_txn_ids(1, 1 + np.arange(n_ranges, dtype=np.uint64), A.KIND_WRITE, node, domain=1)
    cmds = RangeCommands(rtx, np.arange(n_ranges + 1, dtype=np.uint64), start, start + width)
    hk = distinct_rows(rng, lambda r, s: r.integers(0, n_keys, s), n_hist_txns, keys_per_txn)
    cfk, _ = build_history(rng, n_hist_txns, hk, token, _rw_kinds(rng, n_hist_txns), 2,
                           hlc0=n_ranges + 10)
    qk = distinct_rows(rng, lambda r, s: r.integers(0, n_keys, s), n_txns, keys_per_txn)
    q = _queries(rng, n_txns, qk, token, _rw_kinds(rng, n_txns), hlc0=n_ranges + n_hist_txns + 2000)
    return Workload("config4", cfk, cmds, Redundant.empty(), q,
                    params=dict(n_txns=n_txns, keys_per_txn=keys_per_txn, n_keys=n_keys, n_ranges=n_ranges,
                                n_hist_txns=n_hist_txns, seed=seed, semantics="SNAPSHOT"))


def config5(n_txns=1_000_000, keys_per_txn=4, n_keys=100_000, direct_frac=0.01, seed=0xACC0D005):
    """Config 5: 1M committed key txns x 4 keys over 100k keys, 50/50 R/W, executeAt = txnId + a
    unique random 0..999 hlc ticks; 1% of txns carry one direct dep on an earlier-executing txn."""
    rng = np.random.default_rng(seed)
    keys = distinct_rows(rng, lambda r, s: r.integers(0, n_keys, s), n_txns, keys_per_txn)
    keys.sort(axis=1)
    kind = _rw_kinds(rng, n_txns)
    i = np.arange(n_txns, dtype=np.uint64)
    hlc = np.uint64(1000) + i + rng.integers(0, 1000, n_txns).astype(np.uint64)   # txnId hlc = 1000 + i
    ex = make_timestamps(1, hlc, (kind.astype(np.uint64) << np.uint64(1)), EXEC_NODE_BASE + np.arange(n_txns))
    order = np.lexsort(ex.order_key())
    rank = np.empty(n_txns, np.int64)
    rank[order] = np.arange(n_txns)
    has = rng.random(n_txns) < direct_frac
    dep_off = np.zeros(n_txns + 1, np.uint64)
    dep_off[1:] = np.cumsum(has)
    src = np.nonzero(has)[0]
    # a direct dep on a txn executing earlier (Commands.updateWaitingOn keeps only those)
    tgt_rank = (rng.random(len(src)) * np.maximum(rank[src], 1)).astype(np.int64)
    deps = order[tgt_rank].astype(np.uint32)
    deps = np.where(rank[src] > 0, deps, src.astype(np.uint32))     # self-dep of the first is dropped
    key_off = np.arange(n_txns + 1, dtype=np.uint64) * np.uint64(keys_per_txn)
    g = Graph(ex, kind, key_off, keys.reshape(-1).astype(np.int64), dep_off, deps)
    return g, dict(n_txns=n_txns, keys_per_txn=keys_per_txn, n_keys=n_keys, direct_frac=direct_frac, seed=seed)


def random_graph(seed, n_txns=400, n_keys=30, max_keys=4, direct_frac=0.1, kinds=(0, 1, 2, 3, 4, 5),
                 long_runs=False):
    """A waitingOn graph with every Txn.Kind (Read, Write, EphemeralRead, SyncPoint,
    ExclusiveSyncPoint, LocalOnly), 0..max_keys keys per txn, executeAt order unrelated to the
    txn index, node ids with both signs, a few epochs, and direct deps pointing both ways in
    executeAt order (later-executing ones must be ignored) -- for K5 parity tests."""
    rng = np.random.default_rng(seed)
    kind = rng.choice(np.asarray(kinds, np.uint8), n_txns).astype(np.uint8)
    if long_runs:   # long runs of reads on a hot key: the chain walk's worst case
        kind = np.where(rng.random(n_txns) < 0.9, A.KIND_READ, kind).astype(np.uint8)
    nk = rng.integers(0, max_keys + 1, n_txns)
    key_space = rng.choice(np.arange(-1000, 1000), n_keys, replace=False).astype(np.int64)
    rows = [np.sort(rng.choice(key_space, k, replace=False)) for k in nk]
    key_off = np.zeros(n_txns + 1, np.uint64)
    key_off[1:] = np.cumsum(nk)
    keys = np.concatenate(rows + [np.zeros(0, np.int64)]).astype(np.int64)
    epoch = rng.integers(1, 4, n_txns).astype(np.uint64)
    hlc = rng.choice(np.arange(1, 50 * n_txns), n_txns, replace=False).astype(np.uint64)
    node = rng.integers(-3, 4, n_txns).astype(np.int32)
    ex = make_timestamps(epoch, hlc, (kind.astype(np.uint64) << np.uint64(1)), node)
    has = rng.random(n_txns) < direct_frac
    cnt = np.where(has, rng.integers(1, 4, n_txns), 0)
    dep_off = np.zeros(n_txns + 1, np.uint64)
    dep_off[1:] = np.cumsum(cnt)
    deps = rng.integers(0, n_txns, int(cnt.sum())).astype(np.uint32)
    return Graph(ex, kind, key_off, keys, dep_off, deps)


def slice_workload(w, lo, hi):
    """The part of workload `w` a CommandStore owning the token range from lo to hi sees
    ((lo, hi] for EndInclusive ranges, [lo, hi) for StartInclusive): the CommandsForKey of its
    keys; every request, with its keys restricted to the slice (mapReduceForKey skips keys the
    store does not own, InMemoryCommandStore.java:280); range commands with their ranges sliced
    to the store (Ranges.slice(..., Minimal) at registration, InMemoryCommandStore.java:758-761;
    commands left without ranges are not registered) and RedundantBefore sliced likewise."""
    if w.slices is not None:
        raise ValueError("slice_workload: workload already restricted to slices")
    inc = bool(w.range_start_inclusive)

    def inside(x):
        return ((x >= lo) & (x < hi)) if inc else ((x > lo) & (x <= hi))

    def clip(s0, e0):
        s1 = np.maximum(s0, np.int64(lo))
        e1 = np.minimum(e0, np.int64(hi))
        return s1, e1, s1 < e1

    keys = w.cfk.keys
    sel = inside(keys)
    ki = np.nonzero(sel)[0]
    if len(ki):
        e0, e1 = int(w.cfk.seg[ki[0]]), int(w.cfk.seg[ki[-1] + 1])
        seg = w.cfk.seg[ki[0]:ki[-1] + 2] - np.uint64(e0)
    else:
        e0 = e1 = 0
        seg = np.zeros(1, np.uint64)
    cfk = CfkSnapshot(keys[sel], seg, w.cfk.txn.take(slice(e0, e1)), w.cfk.exec.take(slice(e0, e1)),
                      w.cfk.status[e0:e1],
                      None if w.cfk.pruned_before is None else w.cfk.pruned_before[sel])
    q = w.queries
    qsel = inside(q.keys)
    cs = np.zeros(len(q.keys) + 1, np.int64)
    np.cumsum(qsel, out=cs[1:])
    ko = q.key_off.astype(np.int64)
    counts = cs[ko[1:]] - cs[ko[:-1]]
    key_off = np.zeros(len(q) + 1, np.uint64)
    key_off[1:] = np.cumsum(counts)
    # Range-domain requests keep their ranges: the store slices them itself (ad_config slices)
    qq = Queries(q.txn, q.exec, key_off, q.keys[qsel], q.min_epoch, q.range_off, q.range_start, q.range_end)

    c = w.cmds
    rs, re_, keep = clip(c.range_start, c.range_end)
    cmd_of = np.repeat(np.arange(len(c.txn)), np.diff(c.range_off.astype(np.int64)))
    per_cmd = np.bincount(cmd_of[keep], minlength=len(c.txn))
    live = np.nonzero(per_cmd)[0]
    roff = np.zeros(len(live) + 1, np.uint64)
    roff[1:] = np.cumsum(per_cmd[live])
    cmds = RangeCommands(c.txn.take(live), roff, rs[keep], re_[keep],
                         None if c.erased is None else c.erased[live],
                         None if c.historical is None else c.historical[live])
    r = w.redundant
    bs, be, bk = clip(r.range_start, r.range_end)
    bi = np.nonzero(bk)[0]
    red = Redundant(bs[bi], be[bi], r.start_epoch[bi], r.end_epoch[bi], r.wm.take(bi))
    out = Workload(w.name, cfk, cmds, red, qq, w.flags, dict(w.params), w.range_start_inclusive,
                   np.array([[lo, hi]], dtype=np.int64))
    out.params.update(slice=(int(lo), int(hi)))
    return out


def shard_local(w, lo, hi):
    """What the store owning slice (lo, hi] is given in the multi-GPU path: its slice of the
    snapshot (slice_workload) and only the requests that touch it (exchange.route), with their
    global request indices."""
    from .exchange import route
    s = slice_workload(w, lo, hi)
    q, idx = route(w.queries, lo, hi, bool(w.range_start_inclusive))
    s.queries = q
    return s, idx


# ------------------------------------------------------------------------------------------
# Small randomised workloads exercising every branch of the reference path (parity tests)
# ------------------------------------------------------------------------------------------
def random_small(seed, n_keys=24, n_hist_txns=120, n_txns=60, max_keys=4, n_range_cmds=12,
                 n_redundant=3, with_pruned=True, accept_frac=0.3, start_inclusive=False,
                 with_slices=False, exec_below_frac=0.05, range_frac=0.0, truncated=True):
    """All statuses (incl. TRANSITIVELY_KNOWN / INVALID), all globally visible kinds, prunedBefore,
    Accept-style executeAt > txnId (so PreAccept.java:261's self exclusion matters), requests whose
    txnId is in the CFK, range commands (erased / historical / multi-range), RedundantBefore.
    range_frac: that share of the requests (none of them in a CommandsForKey) are Range-domain txns
    (TxnId domain bit set) with 1-3 normalised ranges, from a few keys wide to most of the key space,
    some touching or crossing slice, command and redundant-before boundaries.
    truncated: the CommandsForKeys as every read of the store sees them, truncated to its RedundantBefore
    (truncate_to_redundant); False keeps the entries below the watermarks (the load-time truncation's cases)."""
    rng = np.random.default_rng(seed)
    key_space = np.sort(rng.choice(np.arange(-500, 500), n_keys, replace=False)).astype(np.int64)
    hist_kinds = rng.choice([A.KIND_READ, A.KIND_WRITE, A.KIND_SYNC_POINT, A.KIND_EXCLUSIVE_SYNC_POINT],
                            n_hist_txns, p=[0.4, 0.4, 0.1, 0.1]).astype(np.uint8)
    hist_hlc = np.sort(rng.choice(np.arange(10, 10 * (n_hist_txns + n_txns) + 10), n_hist_txns + n_txns,
                                  replace=False)).astype(np.uint64)
    all_node = rng.integers(1, 17, n_hist_txns + n_txns).astype(np.int32)
    perm = rng.permutation(n_hist_txns + n_txns)
    h_idx, q_idx = np.sort(perm[:n_hist_txns]), np.sort(perm[n_hist_txns:])
    q_kinds = rng.choice([A.KIND_READ, A.KIND_WRITE, A.KIND_EPHEMERAL_READ, A.KIND_SYNC_POINT,
                          A.KIND_EXCLUSIVE_SYNC_POINT], n_txns, p=[0.3, 0.3, 0.1, 0.15, 0.15]).astype(np.uint8)
    kinds = np.zeros(n_hist_txns + n_txns, np.uint8)
    kinds[h_idx] = hist_kinds
    kinds[q_idx] = q_kinds
    epochs = np.where(rng.random(n_hist_txns + n_txns) < 0.2, 2, 1).astype(np.uint64)
    epochs = np.maximum.accumulate(epochs)
    all_txn = make_txn_ids(epochs, hist_hlc, kinds, all_node)
    bump = rng.integers(1, 40, n_hist_txns + n_txns).astype(np.uint64)
    below = rng.random(n_hist_txns + n_txns) < exec_below_frac
    ex_hlc = np.where(below, np.maximum(hist_hlc.astype(np.int64) - bump.astype(np.int64), 1).astype(np.uint64),
                      hist_hlc + bump)
    all_exec_bumped = make_timestamps(epochs, ex_hlc, all_txn.lsb & np.uint64(0xFFFF),
                                      EXEC_NODE_BASE + np.arange(n_hist_txns + n_txns))

    # CFK: every history txn on 1..max_keys keys; queries that are "already known" also appear
    entries = []
    for j in h_idx:
        nk = rng.integers(1, max_keys + 1)
        for kr in rng.choice(n_keys, nk, replace=False):
            entries.append((kr, j))
    known_q = [j for j in q_idx if rng.random() < 0.25]
    rng_q = set(j for j in q_idx if j not in known_q and rng.random() < range_frac) if range_frac else set()
    q_keys = {}
    for j in q_idx:
        nk = rng.integers(0, max_keys + 1)
        q_keys[j] = np.sort(rng.choice(n_keys, nk, replace=False))
        if j in rng_q:
            q_keys[j] = np.zeros(0, np.int64)
        if j in known_q:
            for kr in q_keys[j]:
                entries.append((kr, j))
    entries = sorted(set(entries))
    e_key = np.array([e[0] for e in entries], np.int64)
    e_txn = np.array([e[1] for e in entries], np.int64)
    status = rng.choice(8, len(entries), p=[0.05, 0.05, 0.15, 0.1, 0.1, 0.1, 0.4, 0.05]).astype(np.uint8)
    has_exec = (status >= A.ST_ACCEPTED) & (status <= A.ST_APPLIED)
    # some APPLIED/committed at executeAt == txnId
    same = rng.random(len(entries)) < 0.5
    use_b = has_exec & ~same
    t = all_txn.take(e_txn)
    b = all_exec_bumped.take(e_txn)
    ex = Tids(np.where(use_b, b.msb, t.msb), np.where(use_b, b.lsb, t.lsb), np.where(use_b, b.node, t.node))
    uniq, start, counts = np.unique(e_key, return_index=True, return_counts=True)
    seg = np.zeros(len(uniq) + 1, np.uint64)
    seg[1:] = np.cumsum(counts)
    pruned = None
    if with_pruned:
        pruned = np.full(len(uniq), -1, np.int64)
        for i in range(len(uniq)):
            s0, s1 = int(seg[i]), int(seg[i + 1])
            cand = [p for p in range(s0, s1) if status[p] == A.ST_APPLIED and kinds[e_txn[p]] == A.KIND_WRITE]
            if cand and rng.random() < 0.3:
                pruned[i] = rng.choice(cand) - s0
    cfk = CfkSnapshot(key_space[uniq], seg, t, ex, status, pruned)

    # range commands: Range-domain txnIds below/around the queries
    rc_hlc = np.sort(rng.choice(np.arange(1, 10 * (n_hist_txns + n_txns)), n_range_cmds, replace=False) * 10 + 5)
    rc_kind = rng.choice([A.KIND_READ, A.KIND_WRITE, A.KIND_SYNC_POINT, A.KIND_EXCLUSIVE_SYNC_POINT],
                         n_range_cmds).astype(np.uint8)
    rc_txn = make_txn_ids(1, rc_hlc.astype(np.uint64), rc_kind, rng.integers(1, 17, n_range_cmds), domain=1)
    r_off = [0]
    r_s, r_e = [], []
    for i in range(n_range_cmds):
        nr = rng.integers(1, 4)
        pts = np.sort(rng.choice(np.arange(-520, 520), 2 * nr, replace=False))
        for a in range(nr):
            r_s.append(pts[2 * a])
            r_e.append(pts[2 * a + 1])
        r_off.append(len(r_s))
    # duplicate a range across commands so Range::compare-equal keys merge
    if n_range_cmds >= 2:
        r_s[r_off[1]] = r_s[0]
        r_e[r_off[1]] = r_e[0]
        # keep per-command ranges sorted & disjoint
        seg1 = list(zip(r_s[r_off[1]:r_off[2]], r_e[r_off[1]:r_off[2]]))
        seg1 = sorted(set(seg1))
        merged = []
        for s_, e_ in seg1:
            if merged and s_ <= merged[-1][1]:
                merged[-1] = (merged[-1][0], max(merged[-1][1], e_))
            else:
                merged.append((s_, e_))
        new_s = r_s[:r_off[1]] + [m[0] for m in merged] + r_s[r_off[2]:]
        new_e = r_e[:r_off[1]] + [m[1] for m in merged] + r_e[r_off[2]:]
        delta = len(merged) - (r_off[2] - r_off[1])
        r_off = r_off[:2] + [o + delta for o in r_off[2:]]
        r_s, r_e = new_s, new_e
    cmds = RangeCommands(rc_txn, np.array(r_off, np.uint64), np.array(r_s, np.int64), np.array(r_e, np.int64),
                         erased=(rng.random(n_range_cmds) < 0.15).astype(np.uint8),
                         historical=(rng.random(n_range_cmds) < 0.25).astype(np.uint8))

    # redundant-before: disjoint ranges with range-domain watermarks
    pts = np.sort(rng.choice(np.arange(-520, 520), 2 * n_redundant, replace=False))
    # watermarks across the history's epochs and hlcs, so that truncation (SafeCommandStore.maybeTruncate) cuts
    # into the CommandsForKeys their ranges hold
    rb_ep = np.where(rng.random(n_redundant) < 0.6, 2, 1).astype(np.uint64)
    rb_wm = make_txn_ids(rb_ep, rng.integers(1, (n_hist_txns + n_txns) * 10 // 7 + 2, n_redundant).astype(np.uint64) * 7 + 3,
                         A.KIND_EXCLUSIVE_SYNC_POINT, rng.integers(1, 17, n_redundant), domain=1)
    none = rng.random(n_redundant) < 0.2
    rb_wm = Tids(np.where(none, 0, rb_wm.msb), np.where(none, 0, rb_wm.lsb), np.where(none, 0, rb_wm.node))
    red = Redundant(pts[0::2], pts[1::2], rng.integers(0, 3, n_redundant), rng.integers(2, 5, n_redundant), rb_wm)

    # queries
    qt = all_txn.take(q_idx)
    accept = rng.random(n_txns) < accept_frac
    qb = all_exec_bumped.take(q_idx)
    qe = Tids(np.where(accept, qb.msb, qt.msb), np.where(accept, qb.lsb, qt.lsb), np.where(accept, qb.node, qt.node))
    key_off = np.zeros(n_txns + 1, np.uint64)
    key_off[1:] = np.cumsum([len(q_keys[j]) for j in q_idx])
    keys = np.concatenate([key_space[q_keys[j]] for j in q_idx] + [np.zeros(0, np.int64)])
    min_epoch = rng.integers(0, 3, n_txns).astype(np.int64)
    ro = rs = re_ = None
    if rng_q:
        isr = np.array([j in rng_q for j in q_idx])
        dom = isr.astype(np.uint64)
        qt = Tids(qt.msb, qt.lsb | dom, qt.node)          # Range-domain TxnIds (TxnId.java:154-157)
        qe = Tids(qe.msb, qe.lsb | dom, qe.node)
        # ranges over the key line (endpoints may fall on keys, slice or command bounds)
        bounds = np.concatenate([key_space, [-400, -100, 0, 300], r_s, r_e, pts]).astype(np.int64)
        ro, rs, re_ = [0], [], []
        for i in range(n_txns):
            if isr[i]:
                nr = int(rng.integers(1, 4))
                wide = rng.random() < 0.3
                cand = (np.sort(rng.choice(np.arange(-560, 560), 2 * nr, replace=False)) if wide else
                        np.sort(np.unique(rng.choice(bounds, 2 * nr) + rng.integers(-1, 2, 2 * nr))))
                for a in range(len(cand) // 2):
                    if cand[2 * a] < cand[2 * a + 1]:
                        rs.append(int(cand[2 * a]))
                        re_.append(int(cand[2 * a + 1]))
                if len(rs) == ro[-1]:                      # at least one range
                    lo_ = int(rng.integers(-550, 500))
                    rs.append(lo_)
                    re_.append(lo_ + int(rng.integers(1, 60)))
            ro.append(len(rs))
        ro, rs, re_ = np.array(ro, np.uint64), np.array(rs, np.int64), np.array(re_, np.int64)
    q = Queries(qt, qe, key_off, keys, min_epoch, ro, rs, re_)
    slices = None
    if with_slices:
        slices = np.array([[-400, -100], [0, 300]], np.int64)
    if truncated:
        cfk = truncate_to_redundant(cfk, red, start_inclusive)
    return Workload("random_small", cfk, cmds, red, q, params=dict(seed=seed), range_start_inclusive=int(start_inclusive),
                    slices=slices)


def truncate_to_redundant(cfk, red, start_inclusive=False):
    """The CommandsForKeys truncated to the RedundantBefore `red`, as SafeCommandStore.maybeTruncate leaves them
    (SafeCommandStore.java:165-171 -> CommandsForKey.withRedundantBeforeAtLeast, CommandsForKey.java:1317-1341):
    per key, byId below its entry's shardRedundantBefore leaves and the rest's missing() lose the ids below it
    (Utils.removeRedundantMissing) -- both only where something left -- and a prunedBefore at or below it goes."""
    def contains(s, e, k):
        return (s <= k < e) if start_inclusive else (s < k <= e)
    ne = cfk.n_entries
    keep = np.ones(ne, bool)
    pruned = None if cfk.pruned_before is None else cfk.pruned_before.copy()
    lb = [None] * ne                       # per kept entry: the watermark its missing() is trimmed to
    tid = lambda t, e: (int(t.msb[e]), int(t.lsb[e]), int(t.node[e]))  # noqa: E731
    for k, key in enumerate(cfk.keys.tolist()):
        wm = None
        for i in range(len(red.range_start)):
            if contains(int(red.range_start[i]), int(red.range_end[i]), key):
                w = tid(red.wm, i)
                wm = w if _tid_key(w) > (0, 0, 0, 0) else None
                break
        if wm is None:
            continue
        s0, s1 = int(cfk.seg[k]), int(cfk.seg[k + 1])
        pos = 0
        while s0 + pos < s1 and _tid_key(tid(cfk.txn, s0 + pos)) < _tid_key(wm):
            pos += 1
        keep[s0:s0 + pos] = False
        if pos:
            for e in range(s0 + pos, s1):
                lb[e] = wm
        if pruned is not None and pruned[k] >= 0:
            pruned[k] = -1 if _tid_key(wm) >= _tid_key(tid(cfk.txn, s0 + int(pruned[k]))) else pruned[k] - pos
    idx = np.nonzero(keep)[0]
    e_key = np.repeat(np.arange(len(cfk.keys)), np.diff(cfk.seg.astype(np.int64)))
    seg = np.zeros(len(cfk.keys) + 1, np.uint64)
    seg[1:] = np.cumsum(np.bincount(e_key[idx], minlength=len(cfk.keys)))
    off = miss = None
    if cfk.miss_off is not None:
        off, mi = [0], []
        for e in idx.tolist():
            for j in range(int(cfk.miss_off[e]), int(cfk.miss_off[e + 1])):
                if lb[e] is None or _tid_key(tid(cfk.miss, j)) >= _tid_key(lb[e]):
                    mi.append(j)
            off.append(len(mi))
        off = np.array(off, np.uint64)
        miss = cfk.miss.take(np.array(mi, np.int64))
    out = CfkSnapshot(cfk.keys, seg, cfk.txn.take(idx), cfk.exec.take(idx), cfk.status[idx], pruned, off, miss)
    if getattr(cfk, "ballot", None) is not None:
        out.ballot = cfk.ballot.take(idx)
    return out


def _hlc(t):
    """Timestamp.hlc() (Timestamp.java:129-131) of a Tids."""
    return (t.lsb >> np.uint64(16)) | ((t.msb & np.uint64(0x7FFF)) << np.uint64(48))


def with_redundant_ranges(w, n_entries=16, seed=0xACC0D0B0, covered=0.8, wm_frac=0.3, none_frac=0.1):
    """w with a RedundantBefore over its key line: up to n_entries disjoint ranges (about half the line) whose
    shardAppliedOrInvalidatedBefore are range-domain ExclusiveSyncPoints at up to `wm_frac` of the history's
    hlcs (epoch 1), `none_frac` of them NONE -- the GC watermark of a store whose oldest history is redundant."""
    from dataclasses import replace
    rng = np.random.default_rng(seed)
    keys = w.cfk.keys if len(w.cfk.keys) else np.array([0, 1], np.int64)
    lo, hi = int(keys.min()) - 1, int(keys.max()) + 1
    # consecutive cut pairs [c0, c1), [c2, c3), ... each kept with probability `covered`: disjoint, ascending
    cuts = np.unique(rng.integers(lo, hi, 2 * n_entries).astype(np.int64))
    starts, ends = [], []
    for i in range(0, len(cuts) - 1, 2):
        if rng.random() < covered:
            starts.append(int(cuts[i]))
            ends.append(int(cuts[i + 1]))
    n = len(starts)
    hist_hlc = int(_hlc(w.cfk.txn).max()) if w.cfk.n_entries else 1000
    wm = make_txn_ids(1, rng.integers(1, max(2, int(hist_hlc * wm_frac)), n).astype(np.uint64), A.KIND_EXCLUSIVE_SYNC_POINT,
                      rng.integers(1, 17, n), domain=1)
    none = rng.random(n) < none_frac
    wm = Tids(np.where(none, 0, wm.msb), np.where(none, 0, wm.lsb), np.where(none, 0, wm.node).astype(np.int32))
    red = Redundant(np.array(starts, np.int64), np.array(ends, np.int64), np.zeros(n, np.int64), np.full(n, 1 << 40, np.int64),
                    wm)
    return replace(w, redundant=red)


def advance_redundant(red, seed, step_frac=0.15, hist_hlc=None, frac=0.7):
    """The same RedundantBefore entries with `frac` of the watermarks moved forward by up to step_frac of
    hist_hlc hlc ticks (NONE ones given one): GC progress, for ad_redundant_advance."""
    rng = np.random.default_rng(seed)
    n = len(red.range_start)
    hlc = _hlc(red.wm)
    span = max(2, int((hist_hlc or int(hlc.max()) + 1000) * step_frac))
    move = rng.random(n) < frac
    nh = hlc + rng.integers(1, span, n).astype(np.uint64)
    ep = np.maximum(red.wm.msb >> np.uint64(15), np.uint64(1))          # each watermark keeps its epoch
    new = make_txn_ids(ep, nh, A.KIND_EXCLUSIVE_SYNC_POINT, rng.integers(1, 17, n), domain=1)
    pick = lambda a, b: np.where(move, b, a)  # noqa: E731
    wm = Tids(pick(red.wm.msb, new.msb), pick(red.wm.lsb, new.lsb), pick(red.wm.node, new.node).astype(np.int32))
    return Redundant(red.range_start, red.range_end, red.start_epoch, red.end_epoch, wm)


def range_cmd_updates(cmds, seed, n, lo=-520, hi=520, epoch=1, hlc_hi=500, frac=(0.35, 0.25, 0.15, 0.25), max_width=120):
    """Registry upkeep rows for ad_range_cmds_update (a RangeCommands whose flags say what each row is): shares
    `frac` of (a) updates of registered live commands with more ranges (overlapping, touching or apart), (b) new
    registrations (fresh Range-domain txnIds), (c) erasures of live commands, (d) historical merges (of historical
    commands, of live ones -- ignored -- and new ones). Ranges normalised, within [lo, hi)."""
    rng = np.random.default_rng(seed)
    live = [i for i in range(len(cmds.txn.msb)) if cmds.historical is None or not cmds.historical[i]]
    hist = [i for i in range(len(cmds.txn.msb)) if cmds.historical is not None and cmds.historical[i]]
    kinds = rng.choice(4, n, p=np.asarray(frac) / np.sum(frac))
    fresh = make_txn_ids(epoch, np.sort(rng.choice(np.arange(1, hlc_hi), n, replace=False)).astype(np.uint64) * 10 + 7,
                         rng.choice([A.KIND_READ, A.KIND_WRITE, A.KIND_SYNC_POINT, A.KIND_EXCLUSIVE_SYNC_POINT], n),
                         rng.integers(100, 116, n), domain=1)      # nodes no history id carries: no equal ids
    rows_t, er, hi_f, off, st, en = [], [], [], [0], [], []
    made = []
    for i in range(n):
        k = int(kinds[i])
        if k == 0 and live:
            j = int(rng.choice(live))
            t = (cmds.txn.msb[j], cmds.txn.lsb[j], cmds.txn.node[j])
            base = [(int(cmds.range_start[x]), int(cmds.range_end[x])) for x in range(int(cmds.range_off[j]), int(cmds.range_off[j + 1]))]
        elif k == 3 and (hist or live) and rng.random() < 0.7:
            pool = hist if (hist and rng.random() < 0.7) else (live or hist)
            j = int(rng.choice(pool))
            t = (cmds.txn.msb[j], cmds.txn.lsb[j], cmds.txn.node[j])
            base = [(int(cmds.range_start[x]), int(cmds.range_end[x])) for x in range(int(cmds.range_off[j]), int(cmds.range_off[j + 1]))]
        elif k == 2 and live:
            j = int(rng.choice(live))
            t = (cmds.txn.msb[j], cmds.txn.lsb[j], cmds.txn.node[j])
            base = []
        elif made and rng.random() < 0.3:
            t, base = made[int(rng.integers(0, len(made)))]        # a command this batch registered, again
        else:
            t = (fresh.msb[i], fresh.lsb[i], fresh.node[i])
            base = []
            made.append((t, base))
        rs = []
        if k != 2:
            nr = int(rng.integers(1, 4))
            pts = []
            for _ in range(nr):
                if base and rng.random() < 0.6:                       # near an existing range: overlap / touch / apart
                    a, b = base[int(rng.integers(0, len(base)))]
                    d = int(rng.integers(-3, 4))
                    x = b + d if rng.random() < 0.5 else a - int(rng.integers(1, max(2, max_width // 4))) + d
                    pts.append((x, x + int(rng.integers(1, max(2, max_width // 3)))))
                else:
                    x = int(rng.integers(lo, hi - 1))
                    pts.append((x, min(hi, x + int(rng.integers(1, max_width)))))
            pts.sort()
            for a, b in pts:                                          # normalise (merge overlapping)
                if rs and a < rs[-1][1]:
                    rs[-1] = (rs[-1][0], max(rs[-1][1], b))
                elif a < b:
                    rs.append((a, b))
        rows_t.append(t)
        er.append(1 if k == 2 else 0)
        hi_f.append(1 if k == 3 else 0)
        st += [a for a, _ in rs]
        en += [b for _, b in rs]
        off.append(len(st))
    ids = Tids(np.array([x[0] for x in rows_t], np.uint64), np.array([x[1] for x in rows_t], np.uint64),
               np.array([x[2] for x in rows_t], np.int32))
    return RangeCommands(ids, np.array(off, np.uint64), np.array(st, np.int64), np.array(en, np.int64),
                         erased=np.array(er, np.uint8), historical=np.array(hi_f, np.uint8))


def sequential_ranges(seed, range_frac=0.4, **kw):
    """A SEQUENTIAL PreAccept batch (config 1's semantics) mixing key-domain and Range-domain txns (sync
    points, range reads/writes) over a random_small store with range commands and RedundantBefore: the
    requests in ascending TxnId order with executeAt == txnId; each registers before its deps are
    computed (PreAccept.java:116-132) -- a Range-domain one as a range command
    (InMemoryCommandStore.java:740-763) that every later request of the batch sees."""
    kw.setdefault("accept_frac", 0.0)
    w = random_small(seed, range_frac=range_frac, **kw)
    cm, q = w.cmds, w.queries
    ident = lambda t: set(zip(t.msb.tolist(), (t.lsb >> np.uint64(16)).tolist(),  # noqa: E731
                              (t.lsb & np.uint64(0x1E)).tolist(), t.node.tolist()))
    clash = ident(cm.txn) & ident(q.txn)
    if clash:                          # a batch txn that is already a range command: not a fresh PreAccept
        keep = np.array([x not in clash for x in zip(cm.txn.msb.tolist(), (cm.txn.lsb >> np.uint64(16)).tolist(),
                                                     (cm.txn.lsb & np.uint64(0x1E)).tolist(), cm.txn.node.tolist())])
        w.cmds = RangeCommands.empty() if not keep.any() else cm.take(np.nonzero(keep)[0])
    w.flags = A.AD_SEQUENTIAL
    w.name = "sequential_ranges"
    return w


def range_map(rng, n_values, key_lo, key_hi, hlc_lo, hlc_hi, null_frac=0.1, inclusive_ends=0, epochs=(1, 2),
              node_max=16, flag_noise=True):
    """A random ReducingRangeMap<Timestamp> over key ordinals [key_lo, key_hi): distinct ascending
    starts, Timestamps with random epoch / hlc / node (and, with flag_noise, non-identity lsb
    flag bits such as REJECTED 0x8000 so ties between equal Timestamps are observable), some null."""
    from .model import RangeMap
    n_values = int(n_values)
    if n_values == 0:
        return RangeMap.empty(inclusive_ends)
    starts = np.sort(rng.choice(np.arange(key_lo, key_hi, dtype=np.int64), n_values + 1, replace=False))
    ep = rng.choice(np.asarray(epochs, np.uint64), n_values)
    hlc = rng.integers(hlc_lo, hlc_hi, n_values).astype(np.uint64)
    flags = (rng.integers(0, 5, n_values).astype(np.uint64) << np.uint64(1))
    if flag_noise:
        flags |= np.where(rng.random(n_values) < 0.3, np.uint64(0x8000), np.uint64(0))
    v = make_timestamps(ep, hlc, flags, rng.integers(1, node_max + 1, n_values).astype(np.int32))
    present = (rng.random(n_values) >= null_frac).astype(np.uint8)
    return RangeMap(starts.astype(np.int64), v, present, int(inclusive_ends))


def preaccept_workload(seed, n_txns=300, n_values=40, key_space=600, max_keys=6, inclusive_ends=0, with_reject=True,
                       esp_frac=0.1):
    """Requests (ascending keys) plus maxConflicts / rejectBefore maps with overlapping ranges of
    keys and Timestamps around the requests' txnIds, so every branch of preaccept is taken."""
    from .model import Queries
    rng = np.random.default_rng(seed)
    mc = range_map(rng, n_values, -key_space // 2, key_space // 2, 50, 150, inclusive_ends=inclusive_ends)
    rb = range_map(rng, max(1, n_values // 4), -key_space // 2, key_space // 2, 20, 120,
                   inclusive_ends=inclusive_ends) if with_reject else None
    nk = rng.integers(0, max_keys + 1, n_txns)
    key_off = np.zeros(n_txns + 1, np.uint64)
    key_off[1:] = np.cumsum(nk)
    keys = np.concatenate([np.sort(rng.choice(np.arange(-key_space // 2 - 20, key_space // 2 + 20), k,
                                              replace=False)) for k in nk] + [np.zeros(0, np.int64)]).astype(np.int64)
    # keys exactly on interval starts exercise both end conventions
    on_start = rng.random(len(keys)) < 0.15
    if len(mc) and on_start.any():
        keys[on_start] = rng.choice(mc.starts, int(on_start.sum()))
        for t in range(n_txns):
            seg = keys[int(key_off[t]):int(key_off[t + 1])]
            u = np.unique(seg)
            keys[int(key_off[t]):int(key_off[t]) + len(u)] = u
            nk[t] = len(u)
        # re-pack after de-duplication
        keys = np.concatenate([keys[int(key_off[t]):int(key_off[t]) + int(nk[t])] for t in range(n_txns)]
                              + [np.zeros(0, np.int64)]).astype(np.int64)
        key_off[1:] = np.cumsum(nk)
    kinds = np.where(rng.random(n_txns) < esp_frac, A.KIND_EXCLUSIVE_SYNC_POINT,
                     rng.choice([A.KIND_READ, A.KIND_WRITE, A.KIND_SYNC_POINT], n_txns)).astype(np.uint8)
    txn = make_txn_ids(rng.choice(np.asarray([1, 2], np.uint64), n_txns), rng.integers(40, 160, n_txns).astype(np.uint64),
                       kinds, rng.integers(1, 17, n_txns).astype(np.int32))
    return Queries(txn, txn, key_off, keys, None), mc, rb


def max_conflicts_from_cfk(cfk):
    """The maxConflicts a store holds after every CommandsForKey entry updated it with its executeAt
    (CommandStore.updateMaxConflicts, CommandStore.java:282-291): per key, the max executeAt of its
    entries on the point interval (key - 1, key] (EndInclusive), null between keys."""
    from .model import RangeMap, Tids
    keys = np.asarray(cfk.keys, np.int64)
    if len(keys) == 0:
        return RangeMap.empty(1)
    seg = cfk.seg.astype(np.int64)
    order = np.lexsort(cfk.exec.order_key())            # ascending Timestamp order
    rank = np.empty(len(order), np.int64)
    rank[order] = np.arange(len(order))
    key_of = np.repeat(np.arange(len(keys)), np.diff(seg))
    best = np.full(len(keys), -1, np.int64)
    np.maximum.at(best, key_of, rank)
    best_e = order[best]
    starts = np.unique(np.concatenate([keys - 1, keys]))
    n = len(starts) - 1
    hit = np.isin(starts[1:], keys) & (starts[:-1] == starts[1:] - 1)
    kidx = np.searchsorted(keys, starts[1:])
    kidx = np.minimum(kidx, len(keys) - 1)
    e = best_e[kidx]
    z = np.zeros(n, np.uint64)
    v = Tids(np.where(hit, cfk.exec.msb[e], z), np.where(hit, cfk.exec.lsb[e], z),
             np.where(hit, cfk.exec.node[e], 0).astype(np.int32))
    return RangeMap(starts, v, hit.astype(np.uint8), 1)


def _order(t):
    """Timestamp.compareTo sort keys (Timestamp.java:208-217) of a Tids, for np.lexsort."""
    return (t.node.astype(np.int64), (t.lsb & np.uint64(0x1E)), (t.lsb >> np.uint64(16)), t.msb)


def with_missing(cfk, seed, frac=0.5, max_missing=3, extra=None):
    """A copy of `cfk` whose entries with deps (ACCEPTED..APPLIED) carry TxnInfo.missing() lists
    (CommandsForKey.java:332-341) with probability `frac`: 1..max_missing ids drawn from the same key's
    byId (and from `extra` ids, e.g. txnIds unknown to the store), ascending and duplicate-free."""
    rng = np.random.default_rng(seed)
    ne = cfk.n_entries
    off = np.zeros(ne + 1, np.uint64)
    pick = []
    has_deps = (cfk.status >= A.ST_ACCEPTED) & (cfk.status <= A.ST_APPLIED)
    for k in range(len(cfk.keys)):
        s0, s1 = int(cfk.seg[k]), int(cfk.seg[k + 1])
        for e in range(s0, s1):
            ids = []
            if has_deps[e] and rng.random() < frac:
                n = int(rng.integers(1, max_missing + 1))
                ids = [("e", int(i)) for i in rng.choice(np.arange(s0, s1), min(n, s1 - s0), replace=False)]
                if extra is not None and len(extra) and rng.random() < 0.3:
                    ids.append(("x", int(rng.integers(0, len(extra)))))
            pick.append(ids)
    cols = []
    for e, ids in enumerate(pick):
        t = Tids.concat([cfk.txn.take(np.array([i for s, i in ids if s == "e"], np.int64)),
                         (extra.take(np.array([i for s, i in ids if s == "x"], np.int64)) if extra is not None
                          else cfk.txn.take(np.zeros(0, np.int64)))])
        o = np.lexsort(_order(t)) if len(t) else np.zeros(0, np.int64)
        t = t.take(o)
        keep = np.ones(len(t), bool)          # duplicate-free under Timestamp.equals
        for j in range(1, len(t)):
            keep[j] = not (t.msb[j] == t.msb[j - 1] and ((t.lsb[j] ^ t.lsb[j - 1]) & np.uint64(0xFFFFFFFFFFFF001E)) == 0
                           and t.node[j] == t.node[j - 1])
        cols.append(t.take(np.nonzero(keep)[0]))
        off[e + 1] = off[e] + int(keep.sum())
    miss = Tids.concat(cols) if cols else cfk.txn.take(np.zeros(0, np.int64))
    return CfkSnapshot(cfk.keys, cfk.seg, cfk.txn, cfk.exec, cfk.status, cfk.pruned_before, off, miss)


def recovery_workload(seed, n_known=40, **kw):
    """BeginRecovery scans on a random_small store without range commands: its
    requests (a quarter of them already in the CommandsForKey) plus `n_known` requests recovering a
    txnId of the history over (a superset of) its keys; entries carry missing() lists. With
    range_frac (random_small's) that share of its own requests are Range-domain txns over Ranges."""
    kw.setdefault("n_range_cmds", 0)
    w = random_small(seed, **kw)
    rng = np.random.default_rng(seed ^ 0x5EC0)
    cfk = w.cfk
    e_key = np.repeat(np.arange(len(cfk.keys)), np.diff(cfk.seg.astype(np.int64)))
    qs_t, qs_k = [], []
    if cfk.n_entries:
        for e in rng.choice(cfk.n_entries, min(n_known, cfk.n_entries), replace=False):
            t = cfk.txn.take(np.array([e]))
            same = np.nonzero((cfk.txn.msb == t.msb[0]) & (cfk.txn.lsb == t.lsb[0]) & (cfk.txn.node == t.node[0]))[0]
            ks = set(int(cfk.keys[e_key[i]]) for i in same)
            ks |= set(int(x) for x in rng.choice(cfk.keys, min(2, len(cfk.keys)), replace=False))
            qs_t.append(t)
            qs_k.append(np.array(sorted(ks), np.int64))
    q = w.queries
    txn = Tids.concat([q.txn] + qs_t)
    keys = [q.keys[int(q.key_off[i]):int(q.key_off[i + 1])] for i in range(len(q))] + qs_k
    key_off = np.zeros(len(keys) + 1, np.uint64)
    key_off[1:] = np.cumsum([len(k) for k in keys])
    ro = rs = re_ = None
    if q.range_off is not None:
        # Range-domain requests (range_frac: recovering sync points and range txns over Ranges) keep
        # their ranges; the appended history requests are key-domain
        ro = np.concatenate([q.range_off, np.full(len(qs_k), q.range_off[-1], np.uint64)])
        rs, re_ = q.range_start, q.range_end
    w.queries = Queries(txn, txn, key_off, np.concatenate(keys + [np.zeros(0, np.int64)]), None, ro, rs, re_)
    # stretch some proposed/committed executeAts far past their txnIds (Accept-style), so that earlier
    # txns executing after the recovering one (the STARTED_BEFORE scans) are common
    stretch = ((cfk.status >= A.ST_ACCEPTED) & (cfk.status <= A.ST_APPLIED) & (cfk.exec.node >= EXEC_NODE_BASE)
               & (rng.random(cfk.n_entries) < 0.5))
    bump = (rng.integers(0, 600, cfk.n_entries).astype(np.uint64) << np.uint64(16)) * stretch.astype(np.uint64)
    cfk = CfkSnapshot(cfk.keys, cfk.seg, cfk.txn, Tids(cfk.exec.msb, cfk.exec.lsb + bump, cfk.exec.node), cfk.status,
                      cfk.pruned_before)
    w.cfk = with_missing(cfk, seed, extra=q.txn)
    w.cmds = with_range_recovery(w.cmds, seed, pool=txn)
    w.name = "recovery_small"
    return w


def with_range_recovery(cmds, seed, pool):
    """Recovery facts for every range command (ad_range_cmds_recovery_soa): a status class (proposed,
    stable or neither), deps known or not, executeAtOrTxnId at or up to 4000 hlc ticks past the txnId,
    and a deps id list drawn from `pool` (the recovering ids the scans test) -- so WITH and WITHOUT,
    both status classes and executeAt on either side of a recovering txnId all occur."""
    n = len(cmds.txn)
    rng = np.random.default_rng(seed ^ 0xDE95)
    # range-command txnIds spread over the pool's hlc span, so that commands start before and after
    # the recovering txns
    if n and len(pool):
        hlc_of = (pool.msb.astype(np.uint64) & np.uint64(0x7FFF)) << np.uint64(48) | (pool.lsb >> np.uint64(16))
        lo_h, hi_h = int(hlc_of.min()), int(hlc_of.max())
        h = np.sort(rng.choice(np.arange(max(1, lo_h - 50), hi_h + 50), n, replace=False)).astype(np.uint64)
        kinds = ((cmds.txn.lsb >> np.uint64(1)) & np.uint64(7)).astype(np.uint8)
        epochs = (pool.msb >> np.uint64(15))[rng.integers(0, len(pool), n)]
        cmds = RangeCommands(make_txn_ids(epochs, h, kinds, cmds.txn.node, domain=1), cmds.range_off,
                             cmds.range_start, cmds.range_end, cmds.erased, cmds.historical)
    status = rng.choice([0, A.AD_RS_PROPOSED, A.AD_RS_STABLE], n, p=[0.2, 0.4, 0.4]).astype(np.uint8)
    has_deps = (rng.random(n) < 0.85).astype(np.uint8)
    bump = (rng.integers(0, 4000, n).astype(np.uint64) << np.uint64(16)) * (rng.random(n) < 0.8)
    up = (rng.random(n) < 0.3).astype(np.uint64) << np.uint64(15)          # a later epoch now and then
    ex = Tids(cmds.txn.msb + up, cmds.txn.lsb + bump.astype(np.uint64), cmds.txn.node.copy())
    off = [0]
    parts = []
    npool = len(pool)
    for i in range(n):
        pick = np.nonzero(rng.random(npool) < 0.2)[0] if npool else np.zeros(0, np.int64)
        k = len(pick)
        t = pool.take(np.asarray(pick, np.int64))
        o = np.lexsort((t.node, t.lsb, t.msb)) if k else np.zeros(0, np.int64)
        t = t.take(o)
        # ascending and unique under Timestamp order (msb, lsb >> 16 ... as the oracle compares)
        keep = []
        for j in range(len(t.msb)):
            cur = (int(t.msb[j]), int(t.lsb[j]), int(t.node[j]))
            if keep and _tid_key(keep[-1]) >= _tid_key(cur):
                continue
            keep.append(cur)
        parts.append(keep)
        off.append(off[-1] + len(keep))
    flat = [x for p in parts for x in p]
    deps = Tids(np.array([x[0] for x in flat], np.uint64), np.array([x[1] for x in flat], np.uint64),
                np.array([x[2] for x in flat], np.int32))
    return RangeCommands(cmds.txn, cmds.range_off, cmds.range_start, cmds.range_end, cmds.erased, cmds.historical,
                         rec_status=status, rec_has_deps=has_deps, rec_exec=ex, rec_dep_off=np.array(off, np.uint64),
                         rec_deps=deps)


def _tid_key(t):
    """Timestamp.compareTo order of an (msb, lsb, node) triple (Timestamp.java:209-217)."""
    return (t[0], t[1] >> 16, t[1] & 0x1E, t[2])


def with_missing_fast(cfk, seed, frac=0.2, back=8):
    """Vectorised with_missing for large snapshots: a chosen entry with deps gets one missing id,
    the txnId of an entry up to `back` positions before it in the same key's byId."""
    rng = np.random.default_rng(seed)
    ne = cfk.n_entries
    key_lo = np.repeat(cfk.seg[:-1].astype(np.int64), np.diff(cfk.seg.astype(np.int64)))
    has_deps = (cfk.status >= A.ST_ACCEPTED) & (cfk.status <= A.ST_APPLIED)
    pick = has_deps & (rng.random(ne) < frac)
    src = np.maximum(np.arange(ne) - rng.integers(1, back + 1, ne), key_lo)
    off = np.zeros(ne + 1, np.uint64)
    off[1:] = np.cumsum(pick)
    return CfkSnapshot(cfk.keys, cfk.seg, cfk.txn, cfk.exec, cfk.status, cfk.pruned_before, off,
                       cfk.txn.take(src[pick]))


def with_epoch_slices(w, seed, store_every=0, n_epochs=3):
    """The batch of a store whose ownership changed over epochs 1..n_epochs (a topology change in flight): each
    request's minUnsyncedEpoch is drawn in [1, its executeAt's epoch] and its scan is sliced to
    RangesForEpoch.allBetween(minUnsyncedEpoch, executeAt.epoch()) (PreAccept.java:100,130, Accept.java:115,
    CommandStores.java:233-242) of epochs that own different random parts of the key space, the last one all of
    it; every `store_every`-th request (0: none) reads the store's own slices instead (epochs.py)."""
    from .epochs import RangesForEpoch, with_slice_sets
    rng = np.random.default_rng(seed)
    ks = np.concatenate([np.asarray(w.cfk.keys, np.int64), np.asarray(w.queries.keys, np.int64)])
    if w.queries.range_off is not None and w.queries.n_ranges:
        ks = np.concatenate([ks, w.queries.range_start, w.queries.range_end])
    lo, hi = (int(ks.min()) - 3, int(ks.max()) + 3) if len(ks) else (-1000, 1000)

    def random_ranges(n):
        cuts = np.unique(rng.integers(lo, hi, 2 * n + 8, dtype=np.int64))
        while len(cuts) < 2 * n:
            cuts = np.unique(np.concatenate([cuts, rng.integers(lo, hi, 8, dtype=np.int64)]))
        cuts = np.sort(rng.choice(cuts, 2 * n, replace=False))
        return [(int(cuts[2 * i]), int(cuts[2 * i + 1])) for i in range(n)]
    epochs = list(range(1, n_epochs + 1))
    rfe = RangesForEpoch(epochs, [random_ranges(1 + e % 3) for e in epochs[:-1]] + [[(lo, hi)]])
    q = w.queries.take(np.arange(len(w.queries)))
    ex_ep = (q.exec.msb >> np.uint64(15)).astype(np.int64)
    q.min_epoch = np.array([rng.integers(1, max(1, e) + 1) for e in ex_ep], np.int64)
    from dataclasses import replace
    return with_slice_sets(replace(w, queries=q), rfe, store_every)
