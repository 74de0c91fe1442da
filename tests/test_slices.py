"""Per-request slices (ad_query_soa.slice_set, ad_slice_sets_load): during a topology change the requests of one
batch scan different Ranges -- safeStore.ranges().allBetween(minUnsyncedEpoch, txnId | executeAt) (PreAccept.java:100,
130, Accept.java:115; RangesForEpoch.allBetween, CommandStores.java:233-242). The oracle (refcpu.c slice_select)
against the independent model (refmodel.slices_of) on mixed-epoch batches: key- and Range-domain requests, range
commands, RedundantBefore (unsliced, minUnsyncedEpoch-bounded), the store's own slices beside the sets, recovery
scans; and RangesForEpoch itself against the Java's floor-index reading."""
import numpy as np
import pytest

import refmodel
from accord_deps import _abi as A
from accord_deps import synth
from accord_deps.epochs import RangesForEpoch, ranges_with


def _request(batch, i):
    out = []
    for m in range(3):
        ks, ke, t, k2t = batch.maps[m].request(i)
        keys = [int(x) for x in ks] if ke is None else [(int(a), int(b)) for a, b in zip(ks, ke)]
        out.append((keys, t.tuples(), [int(x) for x in k2t]))
    return out


def test_ranges_for_epoch_all_between():
    r = RangesForEpoch([2, 5, 9], [[(0, 10)], [(20, 30)], [(5, 25), (40, 50)]])
    assert r.all_at(1) == [] and r.all_at(2) == [(0, 10)] and r.all_at(7) == [(20, 30)]
    assert r.all_between(3, 3) == [(0, 10)]
    assert r.all_between(2, 5) == [(0, 10), (20, 30)]                 # Ranges.with of the epochs between
    assert r.all_between(6, 9) == [(5, 30), (40, 50)]                 # overlapping ranges merge
    assert r.all_between(0, 4) == [(0, 10)]                           # max(0, floorIndex(from))
    assert r.all_between(0, 1) == []
    with pytest.raises(IndexError):
        r.all_between(5, 4)
    assert ranges_with([(0, 5)], [(5, 7)]) == [(0, 7)]


@pytest.mark.parametrize("seed", range(16))
def test_crosscheck_epoch_slices(oracle, seed):
    w = synth.random_small(1300 + seed, n_keys=50, n_txns=90, range_frac=0.3 * (seed % 3 != 0),
                           with_slices=(seed % 2 == 1), start_inclusive=(seed % 4 == 2),
                           n_redundant=(0 if seed % 5 == 4 else 4), n_range_cmds=(0 if seed % 6 == 5 else 16))
    w = synth.with_epoch_slices(w, seed, store_every=(0 if seed % 4 == 0 else 5))
    assert len(w.slice_sets) >= 2
    batch = oracle.resolve(w)
    differs = 0
    for i in range(len(w.queries)):
        kd, rd, dd = refmodel.request_pairs(w, i)
        got = _request(batch, i)
        for m, pairs in ((0, kd), (1, rd), (2, dd)):
            assert got[m] == refmodel.csr(pairs), (seed, i, A.MAP_NAMES[m])
        # the request's slice matters: the store's own slices would give another answer for some requests
        own = w.queries.slice_set[i]
        if own != A.AD_SLICE_STORE:
            q = w.queries.take(np.array([i]))
            q.slice_set = None
            from dataclasses import replace
            kd2, rd2, dd2 = refmodel.request_pairs(replace(w, queries=q), 0)
            differs += (kd2, rd2, dd2) != (kd, rd, dd)
    assert differs > 0


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("scan", [0, 3])
def test_crosscheck_epoch_slices_recovery(oracle, seed, scan):
    w = synth.recovery_workload(1400 + seed, n_known=30, range_frac=0.3 * (seed % 2))
    w = synth.with_epoch_slices(w, seed + 7)
    got_batch = oracle.recover(w, scan)
    for i in range(len(w.queries)):
        kd, dd = refmodel.recovery_pairs(w, i, scan)
        rd = refmodel.recovery_range_pairs(w, i, scan)
        got = _request(got_batch, i)
        for m, pairs in ((0, kd), (1, rd), (2, dd)):
            assert got[m] == tuple(refmodel.csr(pairs)), (seed, scan, i, A.MAP_NAMES[m])


def test_slice_set_beyond_the_sets_is_rejected(oracle):
    w = synth.with_epoch_slices(synth.random_small(1500), 1)
    w.queries.slice_set[3] = len(w.slice_sets)
    with pytest.raises(Exception):
        oracle.resolve(w)
