"""GPU parity of device-side pruning (include/accord_deps.h ad_cfk_prune):
Pruning.maybePrune (Pruning.java:164-199) -> pruneBefore (:205-331) on the device state against the
oracle's restatement (oracle/cfk_update.py cfk_prune): the CommandsForKeys left (keys, segments,
TxnIds, statuses, executeAts, prunedBefore) and the deps every later batch computes over them
(bit-exact vs the oracle's calculatePartialDeps, whose prunedBefore substitute reads the new
prunedBefore), also after further updates; the snapshot invariants hold (ad_check_snapshot)."""
import os
import sys

import numpy as np
import pytest

from accord_deps import _abi as A, native, synth
from accord_deps.model import CfkUpdates

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import cfk_update as U  # noqa: E402
import cfk_update_gen as G  # noqa: E402

pytestmark = pytest.mark.gpu


def _check(w, st, oracle, new_cfk):
    keys, seg, txn, pruned = st.cfk_byid()
    assert keys.tolist() == new_cfk.keys.tolist()
    assert seg.tolist() == new_cfk.seg.tolist()
    assert txn.msb.tolist() == new_cfk.txn.msb.tolist() and txn.lsb.tolist() == new_cfk.txn.lsb.tolist()
    assert txn.node.tolist() == new_cfk.txn.node.tolist()
    exp_pb = new_cfk.pruned_before if new_cfk.pruned_before is not None else np.full(len(keys), -1)
    assert pruned.tolist() == exp_pb.tolist()
    s, x = st.cfk_entries()
    assert s.tolist() == new_cfk.status.tolist()
    assert x.msb.tolist() == new_cfk.exec.msb.tolist() and x.lsb.tolist() == new_cfk.exec.lsb.tolist()
    assert st.check_snapshot() == (0, None)
    old = w.cfk
    w.cfk = new_cfk
    try:
        exp = oracle.resolve(w)
        got = st.calculate_partial_deps(w.queries, w.flags)
        ok, why = got.equals(exp, detail=True)
        assert ok, why
    finally:
        w.cfk = old


def _applied_wave(cfk, rng, frac=0.6):
    """Most live entries commit and apply (executeAt = txnId): APPLIED Writes to prune behind."""
    e = np.nonzero(cfk.status < A.ST_APPLIED)[0]
    e = e[rng.random(len(e)) < frac]
    rd = (cfk.txn.lsb[e] & np.uint64(1)) == 1               # range-domain ids stay as they are
    e = e[~rd]
    return CfkUpdates(G.entry_keys(cfk)[e], cfk.txn.take(e), cfk.txn.take(e), np.full(len(e), A.ST_APPLIED, np.uint8))


@pytest.mark.parametrize("seed", range(6))
def test_random_prune(oracle, seed):
    w = synth.random_small(40 + seed, n_keys=16, n_hist_txns=300, n_txns=80, with_slices=(seed % 3 == 2))
    w.flags = A.AD_SNAPSHOT
    rng = np.random.default_rng(seed)
    st = native.DeviceCommandStore(0, w.range_start_inclusive, 1, w.slices)
    try:
        st.load(w)
        cfk = w.cfk
        u = _applied_wave(cfk, rng)
        new, _ = U.cfk_update(cfk, u)
        st.cfk_update(u)
        cfk = new
        for rnd, (interval, delta, keys) in enumerate(((3, 0, None), (1, 0, cfk.keys[::2]), (1, 2, None))):
            if rnd:
                # newer txns applied (Writes and Reads): the next prune point moves forward
                f = G.fresh_preaccepts(cfk, rng, 40, statuses=(A.ST_APPLIED,), kinds=(0, 1), epoch=9 + rnd,
                                       hlc0=1 + 1000 * rnd)
                new, _ = U.cfk_update(cfk, f)
                st.cfk_update(f)
                cfk = new
            exp, removed, nkp = U.cfk_prune(cfk, keys, interval, delta)
            got_removed, stats = st.cfk_prune(keys, interval, delta)
            assert got_removed == removed and stats["n_keys"][1] == nkp
            _check(w, st, oracle, exp)
            cfk = exp
        # the pruned device state keeps serving updates
        u2, _ = G.transitions(cfk, rng, 60)
        new, _ = U.cfk_update(cfk, u2)
        st.cfk_update(u2)
        _check(w, st, oracle, new)
    finally:
        st.close()


def test_prune_removes_something():
    w = synth.random_small(41, n_keys=16, n_hist_txns=300, n_txns=80)
    rng = np.random.default_rng(1)
    cfk, _ = U.cfk_update(w.cfk, _applied_wave(w.cfk, rng, 1.0))
    exp, removed, nkp = U.cfk_prune(cfk, None, 1, 0)
    assert removed > 0 and nkp > 0         # the random tests above exercise real removals


def test_config2_scaled_apply_then_prune(oracle):
    w = synth.config2(n_txns=2000, n_keys=2000, n_hist_entries=40000, seed=11)
    w.flags = A.AD_SNAPSHOT
    st = native.DeviceCommandStore(0)
    try:
        st.load(w)
        rng = np.random.default_rng(11)
        u = _applied_wave(w.cfk, rng, 1.0)
        cfk, _ = U.cfk_update(w.cfk, u)
        st.cfk_update(u)
        exp, removed, nkp = U.cfk_prune(cfk, None, 2, 0)
        got_removed, _ = st.cfk_prune(None, 2, 0)
        assert removed > 0 and got_removed == removed
        _check(w, st, oracle, exp)
    finally:
        st.close()


@pytest.mark.parametrize("seed", range(3))
def test_prune_with_missing_lists(oracle, seed):
    # missing() lists on the device (loaded, then maintained by batches with deps): pruneBefore's
    # subset test against the merged lists (Pruning.java:239-251); lists and recovery scans after
    from test_gpu_cfk_missing import _check as check_missing, _workload, with_deps
    w = _workload(90 + seed, n_hist_txns=200)
    rng = np.random.default_rng(seed)
    st = native.DeviceCommandStore(0, w.range_start_inclusive, 1, w.slices)
    try:
        st.load(w)
        cfk = w.cfk
        u = with_deps(cfk, _applied_wave(cfk, rng, 0.8), rng, keep=0.9, n_new=0)
        cfk, _, _ = U.cfk_update_missing(cfk, u, u.dep_off, u.deps)
        st.cfk_update(u)
        exp, removed, nkp = U.cfk_prune(cfk, None, 1, 0)
        got_removed, stats = st.cfk_prune(None, 1, 0)
        assert got_removed == removed and stats["n_keys"][1] == nkp
        check_missing(w, st, oracle, exp)
        keys, seg, txn, pruned = st.cfk_byid()
        assert pruned.tolist() == (exp.pruned_before.tolist() if exp.pruned_before is not None else [-1] * len(keys))
        assert st.check_snapshot() == (0, None)
    finally:
        st.close()
