"""Host-side data model: structure-of-arrays forms of the reference's inputs and outputs.

Mirrors the Java types the hot path consumes/produces:
  Tids            accord.primitives.Timestamp / TxnId  {msb, lsb, node}  (Timestamp.java:77-79)
  CfkSnapshot     CommandsForKey.SerializerSupport.create(key, TxnInfo[] byId, ..., prunedBefore)
                  for every key of a CommandStore (CommandsForKey.java:226-232)
  RangeCommands   InMemoryCommandStore.rangeCommands / historicalRangeCommands (:103-104)
  Redundant       RedundantBefore entries (RedundantBefore.java:59-120)
  Queries         a batch of PreAccept.calculatePartialDeps requests (PreAccept.java:245)
  PartialDepsBatch  per request the three RelationMultiMaps of PartialDeps (Deps.java:59-119):
                  keys, txnIds and the exact keysToTxnIds int[] (RelationMultiMap.java:245-257)
"""
from dataclasses import dataclass, field
from typing import Optional

import numpy as np

from . import _abi as A

MASK64 = (1 << 64) - 1


@dataclass
class Tids:
    msb: np.ndarray
    lsb: np.ndarray
    node: np.ndarray

    def __post_init__(self):
        self.msb = A.as_u64(self.msb)
        self.lsb = A.as_u64(self.lsb)
        self.node = A.as_i32(self.node)

    def __len__(self):
        return len(self.msb)

    def take(self, idx):
        return Tids(self.msb[idx], self.lsb[idx], self.node[idx])

    @staticmethod
    def concat(parts):
        parts = list(parts)
        return Tids(np.concatenate([p.msb for p in parts]), np.concatenate([p.lsb for p in parts]),
                    np.concatenate([p.node for p in parts]))

    def kind(self):
        return ((self.lsb >> np.uint64(1)) & np.uint64(7)).astype(np.uint8)

    def domain(self):
        return (self.lsb & np.uint64(1)).astype(np.uint8)

    def epoch(self):
        return (self.msb >> np.uint64(15)).astype(np.int64)

    def order_key(self):
        """Columns for np.lexsort reproducing Timestamp.compareTo (Timestamp.java:208-217);
        last column is the primary key."""
        return (self.node.astype(np.int64), self.lsb & np.uint64(0x1E), self.lsb >> np.uint64(16), self.msb)

    def tuples(self):
        return list(zip(self.msb.tolist(), self.lsb.tolist(), self.node.tolist()))


def make_timestamps(epoch, hlc, flags, node):
    """Timestamp(epoch, hlc, flags, node): msb = epoch<<15 | hlc>>>48, lsb = hlc<<16 | flags
    (Timestamp.java:81-89)."""
    epoch = np.asarray(epoch, dtype=np.uint64)
    hlc = np.asarray(hlc, dtype=np.uint64)
    flags = np.asarray(flags, dtype=np.uint64)
    msb = (epoch << np.uint64(15)) | (hlc >> np.uint64(48))
    lsb = (hlc << np.uint64(16)) | flags
    msb, lsb, node = np.broadcast_arrays(msb, lsb, np.asarray(node, dtype=np.int32))
    return Tids(msb.copy(), lsb.copy(), node.copy())


def make_txn_ids(epoch, hlc, kind, node, domain=0):
    """TxnId(epoch, hlc, kind, domain, node): flags = kind<<1 | domain (TxnId.java:124-137)."""
    kind = np.asarray(kind, dtype=np.uint64)
    domain = np.asarray(domain, dtype=np.uint64)
    return make_timestamps(epoch, hlc, (kind << np.uint64(1)) | domain, node)


@dataclass
class CfkSnapshot:
    keys: np.ndarray          # i64 [n_keys] strictly ascending
    seg: np.ndarray           # u64 [n_keys+1]
    txn: Tids
    exec: Tids
    status: np.ndarray        # u8
    pruned_before: Optional[np.ndarray] = None   # i64 [n_keys], -1 = none
    # TxnInfo.missing() (CommandsForKey.java:332-341): ids of entry e are miss[miss_off[e]:miss_off[e+1]]
    miss_off: Optional[np.ndarray] = None        # u64 [n_entries+1]; None = every entry NO_TXNIDS
    miss: Optional[Tids] = None
    # TxnInfo.ballot() per entry (TxnInfoExtra, CommandsForKey.java:273-283); None = Ballot.ZERO
    ballot: Optional[Tids] = None

    def __post_init__(self):
        self.keys = A.as_i64(self.keys)
        if self.miss_off is not None:
            self.miss_off = A.as_u64(self.miss_off)
        self.seg = A.as_u64(self.seg)
        self.status = A.as_u8(self.status)
        if self.pruned_before is not None:
            self.pruned_before = A.as_i64(self.pruned_before)

    @property
    def n_entries(self):
        return len(self.status)

    def soa(self):
        s = A.AdCfkSoa()
        s.n_keys = len(self.keys)
        s.keys = A.ptr(self.keys)
        s.seg = A.ptr(self.seg)
        s.n_entries = len(self.status)
        s.txn_msb, s.txn_lsb, s.txn_node = A.ptr(self.txn.msb), A.ptr(self.txn.lsb), A.ptr(self.txn.node)
        s.exec_msb, s.exec_lsb, s.exec_node = A.ptr(self.exec.msb), A.ptr(self.exec.lsb), A.ptr(self.exec.node)
        s.status = A.ptr(self.status)
        s.pruned_before = A.ptr(self.pruned_before)
        return s

    def ballot_arrays(self):
        """(msb, lsb, node) of the ballots for ad_cfk_ballots_load, or None."""
        if self.ballot is None:
            return None
        return (np.ascontiguousarray(self.ballot.msb, np.uint64), np.ascontiguousarray(self.ballot.lsb, np.uint64),
                np.ascontiguousarray(self.ballot.node, np.int32))

    def missing_soa(self):
        """AdCfkMissingSoa of the missing lists, or None when there are none."""
        if self.miss_off is None:
            return None
        s = A.AdCfkMissingSoa()
        s.n_entries = len(self.status)
        s.off = A.ptr(self.miss_off)
        s.msb, s.lsb, s.node = A.ptr(self.miss.msb), A.ptr(self.miss.lsb), A.ptr(self.miss.node)
        return s

    @staticmethod
    def empty():
        z64 = np.zeros(0, np.uint64)
        return CfkSnapshot(np.zeros(0, np.int64), np.zeros(1, np.uint64), Tids(z64, z64, np.zeros(0, np.int32)),
                           Tids(z64, z64, np.zeros(0, np.int32)), np.zeros(0, np.uint8))


@dataclass
class CfkUpdates:
    """A batch of CommandsForKey.update calls (ad_cfk_update_soa): update i raises txn[i] in the
    CommandsForKey of keys[i] to status[i] with executeAt exec[i] and the command's ballot
    (acceptedOrCommitted; None = Ballot.ZERO)."""
    keys: np.ndarray          # i64
    txn: Tids
    exec: Tids
    status: np.ndarray        # u8 InternalStatus
    ballot: Optional[Tids] = None
    # the command's deps on the key per update (ascending): deps[dep_off[i]:dep_off[i+1]]; None = none
    dep_off: Optional[np.ndarray] = None
    deps: Optional[Tids] = None

    def __post_init__(self):
        self.keys = A.as_i64(self.keys)
        self.status = A.as_u8(self.status)
        if self.dep_off is not None:
            self.dep_off = A.as_u64(self.dep_off)

    def __len__(self):
        return len(self.keys)

    def soa(self):
        s = A.AdCfkUpdateSoa()
        s.n = len(self.keys)
        s.keys = A.ptr(self.keys)
        s.txn_msb, s.txn_lsb, s.txn_node = A.ptr(self.txn.msb), A.ptr(self.txn.lsb), A.ptr(self.txn.node)
        s.exec_msb, s.exec_lsb, s.exec_node = A.ptr(self.exec.msb), A.ptr(self.exec.lsb), A.ptr(self.exec.node)
        s.status = A.ptr(self.status)
        if self.ballot is not None:
            s.ballot_msb, s.ballot_lsb, s.ballot_node = A.ptr(self.ballot.msb), A.ptr(self.ballot.lsb), A.ptr(self.ballot.node)
        if self.dep_off is not None:
            s.dep_off = A.ptr(self.dep_off)
            s.dep_msb, s.dep_lsb, s.dep_node = A.ptr(self.deps.msb), A.ptr(self.deps.lsb), A.ptr(self.deps.node)
        return s


@dataclass
class RangeCommands:
    txn: Tids
    range_off: np.ndarray
    range_start: np.ndarray
    range_end: np.ndarray
    erased: Optional[np.ndarray] = None
    historical: Optional[np.ndarray] = None
    # recovery facts (ad_range_cmds_recovery_soa): AD_RS_* status class, deps known, executeAtOrTxnId,
    # and per command the ids t with partialDeps().intersects(t, its ranges), ascending
    rec_status: Optional[np.ndarray] = None
    rec_has_deps: Optional[np.ndarray] = None
    rec_exec: Optional[Tids] = None
    rec_dep_off: Optional[np.ndarray] = None
    rec_deps: Optional[Tids] = None

    def __post_init__(self):
        self.range_off = A.as_u64(self.range_off)
        self.range_start = A.as_i64(self.range_start)
        self.range_end = A.as_i64(self.range_end)
        if self.erased is not None:
            self.erased = A.as_u8(self.erased)
        if self.historical is not None:
            self.historical = A.as_u8(self.historical)
        if self.rec_status is not None:
            self.rec_status = A.as_u8(self.rec_status)
            self.rec_has_deps = A.as_u8(self.rec_has_deps)
            self.rec_dep_off = A.as_u64(self.rec_dep_off)

    def recovery_soa(self):
        """AdRangeCmdsRecoverySoa of the recovery facts, or None when there are none."""
        if self.rec_status is None:
            return None
        s = A.AdRangeCmdsRecoverySoa()
        s.n_cmds = len(self.txn)
        s.status, s.has_deps = A.ptr(self.rec_status), A.ptr(self.rec_has_deps)
        s.exec_msb, s.exec_lsb, s.exec_node = A.ptr(self.rec_exec.msb), A.ptr(self.rec_exec.lsb), A.ptr(self.rec_exec.node)
        s.dep_off = A.ptr(self.rec_dep_off)
        s.dep_msb, s.dep_lsb, s.dep_node = A.ptr(self.rec_deps.msb), A.ptr(self.rec_deps.lsb), A.ptr(self.rec_deps.node)
        return s

    def soa(self):
        s = A.AdRangeCmdsSoa()
        s.n_cmds = len(self.txn)
        s.txn_msb, s.txn_lsb, s.txn_node = A.ptr(self.txn.msb), A.ptr(self.txn.lsb), A.ptr(self.txn.node)
        s.erased = A.ptr(self.erased)
        s.historical = A.ptr(self.historical)
        s.range_off = A.ptr(self.range_off)
        s.range_start = A.ptr(self.range_start)
        s.range_end = A.ptr(self.range_end)
        return s

    @staticmethod
    def empty():
        z64 = np.zeros(0, np.uint64)
        return RangeCommands(Tids(z64, z64, np.zeros(0, np.int32)), np.zeros(1, np.uint64),
                             np.zeros(0, np.int64), np.zeros(0, np.int64))

    def take(self, idx):
        """The commands idx (ascending), their ranges with them (recovery facts dropped)."""
        idx = np.asarray(idx, np.int64)
        o = self.range_off.astype(np.int64)
        cnt = o[idx + 1] - o[idx]
        off = np.zeros(len(idx) + 1, np.uint64)
        off[1:] = np.cumsum(cnt)
        src = np.repeat(o[idx] - off[:-1].astype(np.int64), cnt) + np.arange(int(off[-1]))
        sel = lambda a: None if a is None else a[idx]  # noqa: E731
        return RangeCommands(self.txn.take(idx), off, self.range_start[src], self.range_end[src], sel(self.erased),
                             sel(self.historical))


@dataclass
class Redundant:
    range_start: np.ndarray
    range_end: np.ndarray
    start_epoch: np.ndarray
    end_epoch: np.ndarray
    wm: Tids

    def __post_init__(self):
        self.range_start = A.as_i64(self.range_start)
        self.range_end = A.as_i64(self.range_end)
        self.start_epoch = A.as_i64(self.start_epoch)
        self.end_epoch = A.as_i64(self.end_epoch)

    def soa(self):
        s = A.AdRedundantSoa()
        s.n = len(self.range_start)
        s.range_start, s.range_end = A.ptr(self.range_start), A.ptr(self.range_end)
        s.start_epoch, s.end_epoch = A.ptr(self.start_epoch), A.ptr(self.end_epoch)
        s.wm_msb, s.wm_lsb, s.wm_node = A.ptr(self.wm.msb), A.ptr(self.wm.lsb), A.ptr(self.wm.node)
        return s

    @staticmethod
    def empty():
        z = np.zeros(0, np.int64)
        z64 = np.zeros(0, np.uint64)
        return Redundant(z, z, z, z, Tids(z64, z64, np.zeros(0, np.int32)))


@dataclass
class Queries:
    """A batch of calculatePartialDeps requests (ad_query_soa). Key-domain requests carry keys
    (key_off / keys); Range-domain requests (range_off not None) carry normalised Ranges
    (range_off / range_start / range_end) and no keys."""
    txn: Tids
    exec: Tids
    key_off: np.ndarray
    keys: np.ndarray
    min_epoch: Optional[np.ndarray] = None
    range_off: Optional[np.ndarray] = None
    range_start: Optional[np.ndarray] = None
    range_end: Optional[np.ndarray] = None
    # per request its slice set (ad_query_soa.slice_set: an index into Workload.slice_sets, A.AD_SLICE_STORE = the
    # store's own slices); None = every request reads the store's slices
    slice_set: Optional[np.ndarray] = None

    def __post_init__(self):
        self.key_off = A.as_u64(self.key_off)
        self.keys = A.as_i64(self.keys)
        if self.min_epoch is not None:
            self.min_epoch = A.as_i64(self.min_epoch)
        if self.slice_set is not None:
            self.slice_set = A.as_u32(self.slice_set)
        if self.range_off is not None:
            self.range_off = A.as_u64(self.range_off)
            self.range_start = A.as_i64(self.range_start)
            self.range_end = A.as_i64(self.range_end)

    def __len__(self):
        return len(self.txn)

    @property
    def n_probes(self):
        return int(self.key_off[-1]) if len(self.key_off) else 0

    @property
    def n_ranges(self):
        return int(self.range_off[-1]) if self.range_off is not None and len(self.range_off) else 0

    def ranges_of(self, i):
        """[(start, end)] of request i (empty for a key-domain request)."""
        if self.range_off is None:
            return []
        a, b = int(self.range_off[i]), int(self.range_off[i + 1])
        return list(zip(self.range_start[a:b].tolist(), self.range_end[a:b].tolist()))

    def soa(self):
        s = A.AdQuerySoa()
        s.n_txns = len(self.txn)
        s.txn_msb, s.txn_lsb, s.txn_node = A.ptr(self.txn.msb), A.ptr(self.txn.lsb), A.ptr(self.txn.node)
        s.exec_msb, s.exec_lsb, s.exec_node = A.ptr(self.exec.msb), A.ptr(self.exec.lsb), A.ptr(self.exec.node)
        s.min_epoch = A.ptr(self.min_epoch)
        s.key_off = A.ptr(self.key_off)
        s.keys = A.ptr(self.keys)
        s.n_keys = self.n_probes
        if self.range_off is not None:
            s.range_off = A.ptr(self.range_off)
            s.range_start = A.ptr(self.range_start)
            s.range_end = A.ptr(self.range_end)
            s.n_ranges = self.n_ranges
        s.slice_set = A.ptr(self.slice_set)
        return s

    def window(self, lo, hi):
        return self.take(np.arange(lo, hi, dtype=np.int64))

    @staticmethod
    def _gather(off, vals, idx):
        o = off.astype(np.int64)
        cnt = o[idx + 1] - o[idx]
        noff = np.zeros(len(idx) + 1, np.uint64)
        noff[1:] = np.cumsum(cnt)
        src = np.repeat(o[idx] - noff[:-1].astype(np.int64), cnt) + np.arange(int(noff[-1]))
        return noff, [v[src] for v in vals]

    def take(self, idx):
        """The requests `idx` (ascending or not) as a batch of their own (SNAPSHOT requests are
        independent of each other, so a sample resolves to the same PartialDeps)."""
        idx = np.asarray(idx, np.int64)
        key_off, (keys,) = Queries._gather(self.key_off, [self.keys], idx)
        ro = rs = re = None
        if self.range_off is not None:
            ro, (rs, re) = Queries._gather(self.range_off, [self.range_start, self.range_end], idx)
        return Queries(self.txn.take(idx), self.exec.take(idx), key_off, keys,
                       None if self.min_epoch is None else self.min_epoch[idx], ro, rs, re,
                       None if self.slice_set is None else self.slice_set[idx])


@dataclass
class Graph:
    exec: Tids
    kind: np.ndarray
    key_off: np.ndarray
    keys: np.ndarray
    dep_off: Optional[np.ndarray] = None
    deps: Optional[np.ndarray] = None

    def __post_init__(self):
        self.kind = A.as_u8(self.kind)
        self.key_off = A.as_u64(self.key_off)
        self.keys = A.as_i64(self.keys)
        if self.dep_off is not None:
            self.dep_off = A.as_u64(self.dep_off)
            self.deps = A.as_u32(self.deps)

    def soa(self):
        s = A.AdGraphSoa()
        s.n_txns = len(self.kind)
        s.exec_msb, s.exec_lsb, s.exec_node = A.ptr(self.exec.msb), A.ptr(self.exec.lsb), A.ptr(self.exec.node)
        s.kind = A.ptr(self.kind)
        s.key_off, s.keys = A.ptr(self.key_off), A.ptr(self.keys)
        s.dep_off, s.deps = A.ptr(self.dep_off), A.ptr(self.deps)
        return s


@dataclass
class RangeMap:
    """A ReducingRangeMap<Timestamp> (ReducingIntervalMap.java: starts one longer than values):
    value i on [starts[i], starts[i+1]) or, with inclusive_ends, (starts[i], starts[i+1]]; a
    value absent where present[i] == 0 (null). MaxConflicts / rejectBefore of a CommandStore."""
    starts: np.ndarray          # i64 [n + 1] ascending, distinct
    values: Tids                # [n]
    present: np.ndarray = None  # u8 [n] (None = all present)
    inclusive_ends: int = 0

    @staticmethod
    def empty(inclusive_ends=0):
        z = np.zeros(0, np.uint64)
        return RangeMap(np.zeros(0, np.int64), Tids(z, z, np.zeros(0, np.int32)), None, inclusive_ends)

    def __len__(self):
        return len(self.values.msb)

    def soa(self):
        s = A.AdRangeMapSoa()
        s.n_values = len(self)
        if len(self):
            s.starts = A.ptr(self.starts)
            s.msb, s.lsb, s.node = A.ptr(self.values.msb), A.ptr(self.values.lsb), A.ptr(self.values.node)
            s.present = A.ptr(self.present) if self.present is not None else None
        s.inclusive_ends = self.inclusive_ends
        return s


@dataclass
class DepsMap:
    """One RelationMultiMap per request, packed: keys / txnIds / keysToTxnIds per request."""
    keys_off: np.ndarray
    keys: np.ndarray            # i64 key ordinal, or range start (rangeDeps)
    keys_end: Optional[np.ndarray]   # range end (rangeDeps only)
    txn_off: np.ndarray
    txn: Tids
    k2t_off: np.ndarray
    k2t: np.ndarray

    def request(self, i):
        ks = self.keys[self.keys_off[i]:self.keys_off[i + 1]]
        ke = None if self.keys_end is None else self.keys_end[self.keys_off[i]:self.keys_off[i + 1]]
        t = self.txn.take(slice(int(self.txn_off[i]), int(self.txn_off[i + 1])))
        return ks, ke, t, self.k2t[self.k2t_off[i]:self.k2t_off[i + 1]]


@dataclass
class PartialDepsBatch:
    maps: list                  # [keyDeps, rangeDeps, directKeyDeps] DepsMap
    scan_entries: int = 0
    stats: dict = field(default_factory=dict)

    @property
    def n_txns(self):
        return len(self.maps[0].keys_off) - 1

    def equals(self, other, detail=False):
        """Deps.equals (Deps.java:294-303): keys, txnIds and keysToTxnIds equal in all three maps."""
        for m in range(A.NMAPS):
            a, b = self.maps[m], other.maps[m]
            pairs = [("keys_off", a.keys_off, b.keys_off), ("keys", a.keys, b.keys),
                     ("txn_off", a.txn_off, b.txn_off), ("txn.msb", a.txn.msb, b.txn.msb),
                     ("txn.lsb", a.txn.lsb, b.txn.lsb), ("txn.node", a.txn.node, b.txn.node),
                     ("k2t_off", a.k2t_off, b.k2t_off), ("k2t", a.k2t, b.k2t)]
            if a.keys_end is not None or b.keys_end is not None:
                pairs.append(("keys_end", a.keys_end, b.keys_end))
            for name, x, y in pairs:
                if x is None or y is None or x.shape != y.shape or not np.array_equal(x, y):
                    if detail:
                        return False, "%s.%s differs" % (A.MAP_NAMES[m], name)
                    return False
        return (True, "") if detail else True

    def first_mismatch(self, other):
        for i in range(self.n_txns):
            for m in range(A.NMAPS):
                a = self.maps[m].request(i)
                b = other.maps[m].request(i)
                same = np.array_equal(a[0], b[0]) and np.array_equal(a[2].msb, b[2].msb) and \
                    np.array_equal(a[2].lsb, b[2].lsb) and np.array_equal(a[2].node, b[2].node) and \
                    np.array_equal(a[3], b[3])
                if a[1] is not None or b[1] is not None:
                    same = same and a[1] is not None and b[1] is not None and np.array_equal(a[1], b[1])
                if not same:
                    return i, A.MAP_NAMES[m], a, b
        return None

    def pair_count(self, m):
        mm = self.maps[m]
        return int(len(mm.k2t) - len(mm.keys))

    def take(self, idx):
        """Requests `idx` as a batch of their own (offsets rebased)."""
        idx = np.asarray(idx, np.int64)
        maps = []
        for mm in self.maps:
            def sub(off):
                o = off.astype(np.int64)
                cnt = o[idx + 1] - o[idx]
                no = np.zeros(len(idx) + 1, np.uint64)
                no[1:] = np.cumsum(cnt)
                return no, np.repeat(o[idx] - no[:-1].astype(np.int64), cnt) + np.arange(int(no[-1]))
            ko, ks = sub(mm.keys_off)
            to, ts = sub(mm.txn_off)
            oo, os_ = sub(mm.k2t_off)
            maps.append(DepsMap(ko, mm.keys[ks], None if mm.keys_end is None else mm.keys_end[ks], to, mm.txn.take(ts),
                                oo, mm.k2t[os_]))
        return PartialDepsBatch(maps)

    def window(self, first, count):
        """Requests [first, first + count) as a batch of their own (offsets rebased)."""
        maps = []
        for mm in self.maps:
            k0, k1 = int(mm.keys_off[first]), int(mm.keys_off[first + count])
            t0, t1 = int(mm.txn_off[first]), int(mm.txn_off[first + count])
            o0, o1 = int(mm.k2t_off[first]), int(mm.k2t_off[first + count])
            maps.append(DepsMap(mm.keys_off[first:first + count + 1] - np.uint64(k0), mm.keys[k0:k1],
                                None if mm.keys_end is None else mm.keys_end[k0:k1],
                                mm.txn_off[first:first + count + 1] - np.uint64(t0), mm.txn.take(slice(t0, t1)),
                                mm.k2t_off[first:first + count + 1] - np.uint64(o0), mm.k2t[o0:o1]))
        return PartialDepsBatch(maps)


@dataclass
class Workload:
    name: str
    cfk: CfkSnapshot
    cmds: RangeCommands
    redundant: Redundant
    queries: Queries
    flags: int = A.AD_SNAPSHOT
    params: dict = field(default_factory=dict)
    range_start_inclusive: int = 0
    slices: Optional[np.ndarray] = None      # (n,2) i64 owned ranges, None = all
    # the store's slice sets (ad_slice_sets_load): [(n,2) i64 normalised ranges] per set, the
    # RangesForEpoch.allBetween results Queries.slice_set names; None = none
    slice_sets: Optional[list] = None

    def slice_sets_csr(self):
        """(set_off u64, start i64, end i64) of slice_sets, or None."""
        if self.slice_sets is None:
            return None
        off = np.zeros(len(self.slice_sets) + 1, np.uint64)
        st, en = [], []
        for k, r in enumerate(self.slice_sets):
            r = np.asarray(r, np.int64).reshape(-1, 2)
            off[k + 1] = off[k] + len(r)
            st.append(r[:, 0])
            en.append(r[:, 1])
        cat = (lambda xs: np.ascontiguousarray(np.concatenate(xs) if xs else np.zeros(0, np.int64), np.int64))
        return off, cat(st), cat(en)
