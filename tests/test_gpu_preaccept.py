"""GPU parity of the PreAccept timestamp proposal (CommandStore.preaccept minus the
clock): ad_preaccept_device vs the oracle (rc_preaccept), bit-exact minNonConflicting
{msb, lsb, node} and AD_PA_* flags per request."""
import numpy as np
import pytest

from accord_deps import native, synth
from accord_deps.model import RangeMap

pytestmark = pytest.mark.gpu


def _check(q, mc, rb, oracle, permit=1, epoch=0, snapshot=None, st=None):
    own = st is None
    if own:
        st = native.DeviceCommandStore(0)
        if snapshot is not None:
            st.load(snapshot)                 # keys of the snapshot take the per-key interval indexes
    try:
        st.load_preaccept_maps(mc, rb)
        got, fl, stats = st.preaccept(q, permit, epoch)
    finally:
        if own:
            st.close()
    exp, efl = oracle.preaccept(mc, rb, q, permit, epoch)
    assert np.array_equal(fl, efl), np.nonzero(fl != efl)[0][:5]
    for a in ("msb", "lsb", "node"):
        assert np.array_equal(getattr(got, a), getattr(exp, a)), a
    return fl, stats


@pytest.mark.parametrize("seed", range(12))
@pytest.mark.parametrize("ie", [0, 1])
def test_random_maps(oracle, seed, ie):
    q, mc, rb = synth.preaccept_workload(seed, inclusive_ends=ie, with_reject=(seed % 3 != 0))
    for permit, epoch in ((1, 0), (0, 0), (1, 2)):
        _check(q, mc, rb, oracle, permit, epoch)


def test_empty_maps_and_batch(oracle):
    q, _, _ = synth.preaccept_workload(3)
    fl, _ = _check(q, RangeMap.empty(), None, oracle)
    assert set(np.unique(fl)) <= {1, 4}
    _check(q.window(0, 0), RangeMap.empty(), None, oracle)


def test_config2_scale(oracle):
    # config-2 requests against the maxConflicts of its CommandsForKey history (point intervals),
    # with and without the snapshot loaded (per-key interval indexes vs binary search)
    w = synth.config2(n_txns=200_000, n_keys=200_000, n_hist_entries=2_000_000)
    mc = synth.max_conflicts_from_cfk(w.cfk)
    fl, stats = _check(w.queries, mc, None, oracle)
    assert (fl == 1).any() and stats["ms_device"] > 0
    _check(w.queries, mc, None, oracle, snapshot=w)


@pytest.mark.parametrize("seed", range(8))
def test_snapshot_key_index(oracle, seed):
    # a loaded snapshot whose keys cover part of the requests' keys; maps replaced after first use
    # (the per-key indexes are rebuilt for the new maps)
    from accord_deps import synth as S
    w = S.random_small(300 + seed, n_keys=200)
    q, mc, rb = S.preaccept_workload(seed, key_space=1000, inclusive_ends=seed % 2)
    st = native.DeviceCommandStore(0)
    try:
        st.load(w)
        _check(q, mc, rb, oracle, st=st)
        q2, mc2, rb2 = S.preaccept_workload(seed + 50, key_space=1000, inclusive_ends=(seed + 1) % 2)
        _check(q, mc2, rb2, oracle, st=st)
        _check(q2, mc2, None, oracle, st=st)
    finally:
        st.close()


def test_kat_witnessed_at_on_device(oracle):
    # PreAcceptTest multiKeyTimestampUpdate (:210) through the device path: ad_preaccept_device's
    # minNonConflicting + decision composed with the host node clock (accord_deps.clock)
    import test_oracle as T
    from accord_deps import _abi as A, clock
    from accord_deps.model import make_txn_ids
    t1 = make_txn_ids([1], [100], [A.KIND_WRITE], [2])
    t2 = make_txn_ids([1], [50], [A.KIND_WRITE], [3])
    clk = clock.NodeClock(1, 100, epoch=0)
    clk.set_epoch(1)
    clk.advance(10)
    q = T._single_key_queries(t2, [[10, 11]])
    st = native.DeviceCommandStore(0)
    try:
        st.load_preaccept_maps(T._maxc_after([10], t1.tuples()[0]), None)
        mn, fl, _ = st.preaccept(q, 1, 1)
    finally:
        st.close()
    w = clk.witnessed_at_batch(t2, mn, fl)
    assert w[0] == clock.make(1, 110, clock.flags_of(t2.tuples()[0]), 1)
