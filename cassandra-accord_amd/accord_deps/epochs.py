"""Per-request slices of a store whose ownership changes by epoch (host side of ad_slice_sets_load).

During a topology change the requests of one batch slice their scan to different Ranges:
PreAccept / Accept / GetDeps pass ``safeStore.ranges().allBetween(minUnsyncedEpoch, txnId | executeAt)``
to ``SafeCommandStore.mapReduceActive`` (PreAccept.java:100,130, Accept.java:115, SafeCommandStore.java:292).
``RangesForEpoch`` mirrors ``CommandStores.RangesForEpoch`` (CommandStores.java:143-300) for that; the
distinct results a batch needs become the store's slice sets and each request names its own
(``Queries.slice_set``). A Java host does the same with its own RangesForEpoch.
"""
import numpy as np

from . import _abi as A


def ranges_with(a, b):
    """Ranges.with: the union of two normalised range lists [(start, end)] (ascending, disjoint), normalised
    (overlapping or touching ranges merged)."""
    out = []
    for s, e in sorted(list(a) + list(b)):
        if out and s <= out[-1][1]:
            out[-1] = (out[-1][0], max(out[-1][1], e))
        else:
            out.append((s, e))
    return out


def epoch_of(msb):
    """Timestamp.epoch() of the msb word (the top 48 bits)."""
    return int(msb) >> 15


class RangesForEpoch:
    """epochs ascending; ranges[i] the store's Ranges from epochs[i] on (CommandStores.java:145-146)."""

    def __init__(self, epochs, ranges):
        self.epochs = [int(e) for e in epochs]
        self.ranges = [[(int(s), int(e)) for s, e in r] for r in ranges]
        assert all(a < b for a, b in zip(self.epochs, self.epochs[1:])), "epochs must ascend"

    def _floor_index(self, epoch):                     # :269-274
        i = int(np.searchsorted(self.epochs, epoch, side="right")) - 1
        return i

    def all_at(self, epoch):                           # :190-195
        i = self._floor_index(epoch)
        return [] if i < 0 else list(self.ranges[i])

    def _all_internal(self, start, end):               # :283-291
        if start >= end:
            return []
        out = list(self.ranges[start])
        for i in range(start + 1, end):
            out = ranges_with(self.ranges[i], out)
        return out

    def all_between(self, from_inclusive, to_inclusive):   # :233-242
        if from_inclusive > to_inclusive:
            raise IndexError("allBetween(%d, %d)" % (from_inclusive, to_inclusive))
        if from_inclusive == to_inclusive:
            return self.all_at(from_inclusive)
        return self._all_internal(max(0, self._floor_index(from_inclusive)), 1 + self._floor_index(to_inclusive))


def slice_sets_for(queries, rfe):
    """(slice_sets, slice_set) of a batch: per request allBetween(minUnsyncedEpoch, executeAt.epoch()) -- the
    slice calculatePartialDeps scans with (PreAccept.java:100,130: executeAt == txnId; Accept.java:115) -- as an
    index into the distinct results. slice_sets: [(n, 2) int64 array]; slice_set: uint32 per request."""
    n = len(queries)
    me = np.zeros(n, np.int64) if queries.min_epoch is None else np.asarray(queries.min_epoch, np.int64)
    sets, index, sel = [], {}, np.zeros(n, np.uint32)
    for i in range(n):
        to = epoch_of(queries.exec.msb[i])
        r = tuple(rfe.all_between(min(int(me[i]), to), to))
        if r not in index:
            index[r] = len(sets)
            sets.append(np.asarray(r, np.int64).reshape(-1, 2))
        sel[i] = index[r]
    return sets, sel


def with_slice_sets(w, rfe, store_every=0):
    """The workload with each request sliced to its RangesForEpoch.allBetween result; every `store_every`-th
    request (0: none) names the store's own slices (A.AD_SLICE_STORE) instead."""
    from dataclasses import replace
    sets, sel = slice_sets_for(w.queries, rfe)
    if store_every:
        sel[::store_every] = A.AD_SLICE_STORE
    q = w.queries.take(np.arange(len(w.queries)))
    q.slice_set = sel
    return replace(w, queries=q, slice_sets=sets)
