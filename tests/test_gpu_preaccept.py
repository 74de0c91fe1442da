"""GPU parity of the PreAccept timestamp proposal (CommandStore.preaccept minus the
clock): ad_preaccept_device vs the oracle (rc_preaccept), bit-exact minNonConflicting
{msb, lsb, node} and AD_PA_* flags per request."""
import numpy as np
import pytest

from accord_deps import native, synth
from accord_deps.model import RangeMap

pytestmark = pytest.mark.gpu


def _check(q, mc, rb, oracle, permit=1, epoch=0):
    st = native.DeviceCommandStore(0)
    try:
        st.load_preaccept_maps(mc, rb)
        got, fl, stats = st.preaccept(q, permit, epoch)
    finally:
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
    # config-2 requests against the maxConflicts of its CommandsForKey history (1M point intervals)
    w = synth.config2(n_txns=200_000, n_keys=200_000, n_hist_entries=2_000_000)
    mc = synth.max_conflicts_from_cfk(w.cfk)
    fl, stats = _check(w.queries, mc, None, oracle)
    assert (fl == 1).any() and stats["ms_device"] > 0
