"""RedundantBefore truncation (SafeCommandStore.maybeTruncate, SafeCommandStore.java:165-171 ->
CommandsForKey.withRedundantBeforeAtLeast, CommandsForKey.java:1317-1341; Utils.removeRedundantMissing,
Utils.java:265-275): the oracle's store_truncate (oracle/refcpu.c) against the independent model
(refmodel.truncate) on stores read before truncation, the synthetic generator's own truncation
(synth.truncate_to_redundant) against both, and the oracle's in-place advance (rc_redundant_advance).
CPU only."""
import numpy as np
import pytest

from accord_deps import _abi as A, synth
from accord_deps.model import Redundant, Tids, make_txn_ids

import refmodel
from test_oracle import _request


def _removed(w):
    t = synth.truncate_to_redundant(w.cfk, w.redundant, bool(w.range_start_inclusive))
    return w.cfk.n_entries - t.n_entries


@pytest.mark.parametrize("seed", range(16))
def test_snapshot_crosscheck_untruncated(oracle, seed):
    w = synth.random_small(3000 + seed, n_keys=40, n_hist_txns=300, n_txns=100, n_redundant=3 + seed % 4,
                           with_slices=(seed % 3 == 2), start_inclusive=(seed % 4 == 1),
                           range_frac=(0.3 if seed % 2 else 0.0), truncated=False)
    batch = oracle.resolve(w)
    for i in range(len(w.queries)):
        kd, rd, dd = refmodel.request_pairs(w, i)
        got = _request(batch, i)
        for m, pairs in ((0, kd), (1, rd), (2, dd)):
            assert got[m] == tuple(refmodel.csr(pairs)), (seed, i, A.MAP_NAMES[m])


def test_untruncated_workloads_hold_redundant_entries():
    removed = [_removed(synth.random_small(3000 + seed, n_keys=40, n_hist_txns=300, n_txns=100, n_redundant=3 + seed % 4,
                                           truncated=False)) for seed in range(16)]
    assert sum(r > 0 for r in removed) >= 12, removed


@pytest.mark.parametrize("seed", range(12))
def test_oracle_reads_truncated(oracle, seed):
    # a store read before truncation answers as the same store truncated by the generator (idempotence)
    w = synth.random_small(3100 + seed, n_keys=40, n_hist_txns=300, n_txns=100, n_redundant=5,
                           start_inclusive=(seed % 2 == 1), range_frac=0.2 * (seed % 3), truncated=False)
    t = synth.random_small(3100 + seed, n_keys=40, n_hist_txns=300, n_txns=100, n_redundant=5,
                           start_inclusive=(seed % 2 == 1), range_frac=0.2 * (seed % 3))
    assert t.cfk.n_entries < w.cfk.n_entries
    assert oracle.resolve(w).equals(oracle.resolve(t))


@pytest.mark.parametrize("seed", range(8))
def test_sequential_untruncated(oracle, seed):
    # SEQUENTIAL: a PreAccept below its key's shardRedundantBefore registers nothing (CommandsForKey.java:997)
    w = synth.sequential_ranges(3200 + seed, n_keys=30, n_txns=70, n_redundant=5, range_frac=0.3 * (seed % 2),
                                with_slices=(seed % 3 == 1), truncated=False)
    seq = oracle.resolve(w)
    aug = refmodel.sequential_augmented(w)
    for i in range(len(w.queries)):
        kd, rd, dd = refmodel.request_pairs(aug, i)
        got = _request(seq, i)
        for m, pairs in ((0, kd), (1, rd), (2, dd)):
            assert got[m] == tuple(refmodel.csr(pairs)), (seed, i, A.MAP_NAMES[m])


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("scan", A.RECOVER_SCANS)
def test_recovery_untruncated(oracle, seed, scan):
    # the recovery scans read truncated CommandsForKeys, missing() lists included
    w = synth.recovery_workload(3300 + seed, n_redundant=6, truncated=False, start_inclusive=(seed % 2 == 1))
    batch = oracle.recover(w, scan)
    for i in range(len(w.queries)):
        kd, dd = refmodel.recovery_pairs(w, i, scan)
        rd = refmodel.recovery_range_pairs(w, i, scan)
        got = _request(batch, i)
        for m, pairs in ((0, kd), (1, rd), (2, dd)):
            assert got[m] == tuple(refmodel.csr(pairs)), (seed, scan, i, A.MAP_NAMES[m])


def test_generator_truncation_trims_missing_and_pruned():
    w = synth.recovery_workload(3400, n_redundant=6, truncated=False)
    c = w.cfk
    t = synth.truncate_to_redundant(c, w.redundant, False)
    assert t.n_entries < c.n_entries
    assert int(t.miss_off[-1]) <= int(c.miss_off[-1])
    assert np.all(np.diff(t.seg.astype(np.int64)) >= 0) and int(t.seg[-1]) == t.n_entries
    # idempotent: a truncated store truncates to itself
    t2 = synth.truncate_to_redundant(t, w.redundant, False)
    assert t2.n_entries == t.n_entries and np.array_equal(t2.miss_off, t.miss_off)
    if t.pruned_before is not None:
        assert np.array_equal(t2.pruned_before, t.pruned_before)


def _advanced(red, rng, frac=0.7):
    """The same entries with watermarks moved forward (NONE ones given one), epochs widened."""
    n = len(red.range_start)
    wm = red.wm
    keep_old = rng.random(n) >= frac
    new = make_txn_ids(1, rng.integers(600, 1600, n).astype(np.uint64) * 7 + 3, A.KIND_EXCLUSIVE_SYNC_POINT,
                       rng.integers(1, 17, n), domain=1)
    pick = lambda a, b: np.where(keep_old, a, b)  # noqa: E731
    out = Tids(pick(wm.msb, new.msb), pick(wm.lsb, new.lsb), pick(wm.node, new.node).astype(np.int32))
    # never behind the old watermark
    for i in range(n):
        if refmodel.key((int(out.msb[i]), int(out.lsb[i]), int(out.node[i]))) < \
                refmodel.key((int(wm.msb[i]), int(wm.lsb[i]), int(wm.node[i]))):
            out.msb[i], out.lsb[i], out.node[i] = wm.msb[i], wm.lsb[i], wm.node[i]
    return Redundant(red.range_start, red.range_end, red.start_epoch, red.end_epoch + 1, out)


@pytest.mark.parametrize("seed", range(6))
def test_oracle_advance_equals_fresh_store(oracle, seed):
    import pyoracle
    w = synth.random_small(3500 + seed, n_keys=40, n_hist_txns=300, n_txns=100, n_redundant=5,
                           range_frac=0.2 * (seed % 2))
    rng = np.random.default_rng(seed)
    st = pyoracle.OracleStore(w.range_start_inclusive, 1, w.slices)
    try:
        st.load(w)
        red = w.redundant
        for _ in range(3):
            red = _advanced(red, rng)
            st.redundant_advance(red)
            got = st.deps_batch(w.queries, w.flags)
            w2 = type(w)(w.name, w.cfk, w.cmds, red, w.queries, w.flags, w.params, w.range_start_inclusive, w.slices)
            assert got.equals(oracle.resolve(w2))
            for i in range(0, len(w.queries), 7):
                kd, rd, dd = refmodel.request_pairs(w2, i)
                g = _request(got, i)
                for m, pairs in ((0, kd), (1, rd), (2, dd)):
                    assert g[m] == tuple(refmodel.csr(pairs))
    finally:
        st.close()


def test_oracle_advance_rejects_regress_and_ranges():
    import pyoracle
    w = synth.random_small(3600, n_redundant=4)
    st = pyoracle.OracleStore(w.range_start_inclusive, 1, w.slices)
    try:
        st.load(w)
        red = w.redundant
        live = np.nonzero(red.wm.msb != 0)[0]
        assert len(live)
        i = int(live[0])
        back = Tids(red.wm.msb.copy(), red.wm.lsb.copy(), red.wm.node.copy())
        back.msb[i] = np.uint64(0)
        back.lsb[i] = np.uint64(0)
        back.node[i] = 0
        with pytest.raises(pyoracle.OracleError):
            st.redundant_advance(Redundant(red.range_start, red.range_end, red.start_epoch, red.end_epoch, back))
        moved = red.range_start.copy()
        moved[0] -= 1
        with pytest.raises(pyoracle.OracleError):
            st.redundant_advance(Redundant(moved, red.range_end, red.start_epoch, red.end_epoch, red.wm))
    finally:
        st.close()


# ---- range-command registry upkeep (rc_range_cmds_update) ------------------------------------------------------
def test_ranges_with_cases():
    import refmodel as R
    assert R.ranges_with([(0, 5)], [(5, 10)]) == [(0, 5), (5, 10)]          # touching: apart (MERGE_OVERLAPPING)
    assert R.ranges_with([(0, 5)], [(3, 10)]) == [(0, 10)]
    assert R.ranges_with([(0, 5), (5, 9)], [(3, 6)]) == [(0, 5), (5, 9)]    # covered through a touching chain
    assert R.ranges_with([(0, 5), (6, 9)], [(3, 6)]) == [(0, 9)]            # a merge run takes the touching one
    assert R.ranges_with([(0, 10)], [(2, 3), (4, 5)]) == [(0, 10)]          # superset
    assert R.ranges_with([(2, 3)], [(0, 10)]) == [(0, 10)]
    assert R.ranges_with([(0, 2), (8, 9)], [(3, 4)]) == [(0, 2), (3, 4), (8, 9)]


@pytest.mark.parametrize("seed", range(12))
def test_range_cmds_update_matches_model(oracle, seed):
    import pyoracle
    w = synth.random_small(3700 + seed, n_keys=40, n_hist_txns=200, n_txns=80, n_range_cmds=20 + seed,
                           range_frac=0.3 * (seed % 2), with_slices=(seed % 3 == 1), start_inclusive=(seed % 4 == 2))
    st = pyoracle.OracleStore(w.range_start_inclusive, 1, w.slices)
    try:
        st.load(w)
        cmds = w.cmds
        for step in range(3):
            u = synth.range_cmd_updates(cmds, 50 * seed + step, 12)
            st.range_cmds_update(u)
            cmds = refmodel.range_cmds_update(cmds, u)
            w2 = type(w)(w.name, w.cfk, cmds, w.redundant, w.queries, w.flags, w.params, w.range_start_inclusive,
                         w.slices)
            got = st.deps_batch(w.queries, w.flags)
            assert got.equals(oracle.resolve(w2)), step
            for i in range(len(w.queries)):
                kd, rd, dd = refmodel.request_pairs(w2, i)
                g = _request(got, i)
                for m, pairs in ((0, kd), (1, rd), (2, dd)):
                    assert g[m] == tuple(refmodel.csr(pairs)), (seed, step, i, A.MAP_NAMES[m])
    finally:
        st.close()
