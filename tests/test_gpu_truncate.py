"""GPU parity of RedundantBefore truncation (SafeCommandStore.maybeTruncate, SafeCommandStore.java:165-171 ->
CommandsForKey.withRedundantBeforeAtLeast, CommandsForKey.java:1317-1341; Utils.removeRedundantMissing,
Utils.java:265-275) and of the in-place advance (ad_redundant_advance): stores loaded before truncation are
truncated on the device when built (cfk_update.hip run_cfk_truncate), bit-exact against the oracle's
store_truncate (oracle/refcpu.c, pinned by tests/test_truncate.py) on every path; successive advances of a
config-2-shaped store match a fresh oracle store holding the advanced RedundantBefore, with no rebuild."""
import numpy as np
import pytest

from accord_deps import _abi as A
from accord_deps import native, synth
from accord_deps.model import CfkUpdates, Redundant, Tids

pytestmark = pytest.mark.gpu


def _check(w, oracle, paths=(0, 1), via="host"):
    exp = oracle.resolve(w)
    for path in paths:
        got = native.resolve(w, path=path, via=via)
        ok, why = got.equals(exp, detail=True)
        assert ok, "%s path %d via %s: %s; first mismatch %r" % (w.name, path, via, why, got.first_mismatch(exp))


@pytest.mark.parametrize("seed", range(10))
def test_snapshot_untruncated(oracle, seed):
    w = synth.random_small(4000 + seed, n_keys=50, n_hist_txns=400, n_txns=150, n_redundant=3 + seed % 5,
                           with_slices=(seed % 3 == 2), start_inclusive=(seed % 4 == 1),
                           range_frac=(0.3 if seed % 2 else 0.0), truncated=False)
    _check(w, oracle)


@pytest.mark.parametrize("via", ["device", "regions"])
@pytest.mark.parametrize("seed", range(3))
def test_device_entry_untruncated(oracle, seed, via):
    w = synth.random_small(4100 + seed, n_keys=50, n_hist_txns=400, n_txns=150, n_redundant=5, n_range_cmds=0,
                           truncated=False)
    _check(w, oracle, paths=(0,), via=via)


@pytest.mark.parametrize("seed", range(6))
def test_sequential_untruncated(oracle, seed):
    # PreAccepts below their key's shardRedundantBefore register nothing (CommandsForKey.java:997): the host route
    # (Range-domain requests) and the device route (key-domain only)
    w = synth.sequential_ranges(4200 + seed, n_keys=40, n_txns=100, n_redundant=5, range_frac=0.3 * (seed % 2),
                                with_slices=(seed % 3 == 1), truncated=False)
    _check(w, oracle, paths=(0,))


@pytest.mark.parametrize("seed", range(4))
@pytest.mark.parametrize("scan", A.RECOVER_SCANS)
def test_recovery_untruncated(oracle, seed, scan):
    # host-held missing() lists trimmed with the entries
    w = synth.recovery_workload(4300 + seed, n_redundant=6, truncated=False, range_frac=0.3 * (seed % 2))
    exp = oracle.recover(w, scan)
    got = native.recover(w, scan)
    ok, why = got.equals(exp, detail=True)
    assert ok, (seed, scan, why)


def test_store_views_after_truncation(oracle):
    # ad_cfk_entries / ad_cfk_missing after the build show the truncated store (synth.truncate_to_redundant)
    w = synth.recovery_workload(4400, n_redundant=6, truncated=False)
    t = synth.truncate_to_redundant(w.cfk, w.redundant, bool(w.range_start_inclusive))
    assert t.n_entries < w.cfk.n_entries
    st = native.DeviceCommandStore(0, w.range_start_inclusive, 1, w.slices)
    try:
        st.load(w)
        s, x = st.cfk_entries()
        assert s.tolist() == t.status.tolist()
        assert x.msb.tolist() == t.exec.msb.tolist() and x.lsb.tolist() == t.exec.lsb.tolist()
        off, m = st.cfk_missing()
        assert off.tolist() == t.miss_off.tolist()
        assert m.msb.tolist() == t.miss.msb.tolist() and m.lsb.tolist() == t.miss.lsb.tolist()
    finally:
        st.close()


def _with_red(w, red):
    return type(w)(w.name, w.cfk, w.cmds, red, w.queries, w.flags, w.params, w.range_start_inclusive, w.slices)


@pytest.mark.parametrize("path", [0, 1])
def test_config2_successive_advances(oracle, path):
    # a config-2-shaped store whose GC watermark advances three times; each advance truncates on the device
    # (no snapshot rebuild) and the next batch matches a fresh oracle store with that RedundantBefore
    w = synth.with_redundant_ranges(synth.config2(n_txns=20000, n_keys=20000, n_hist_entries=200000), 16, seed=3)
    hist = int(synth._hlc(w.cfk.txn).max())
    st = native.DeviceCommandStore(0, w.range_start_inclusive, 1, w.slices, path=path)
    try:
        st.load(w)
        got = st.calculate_partial_deps(w.queries, w.flags)
        assert got.equals(oracle.resolve(w))
        red = w.redundant
        removed = 0
        for step in range(3):
            red = synth.advance_redundant(red, 10 + step, hist_hlc=hist)
            stats = st.redundant_advance(red)
            removed += stats["n_keys"][0]
            got = st.calculate_partial_deps(w.queries, w.flags)
            exp = oracle.resolve(_with_red(w, red))
            ok, why = got.equals(exp, detail=True)
            assert ok, (step, why)
        assert removed > 0
    finally:
        st.close()


def test_advance_with_device_missing_lists(oracle):
    # missing() lists held on the device (an update batch with deps moved them there): the advance trims them on
    # the device; recovery scans and the exported lists match the store truncated by the generator
    w = synth.recovery_workload(4500, n_redundant=6)
    w.cfk = synth.with_missing(w.cfk, 4500)             # ids of byId only: the lists can move to the device
    st = native.DeviceCommandStore(0, w.range_start_inclusive, 1, w.slices)
    try:
        st.load(w)
        z = Tids(np.zeros(0, np.uint64), np.zeros(0, np.uint64), np.zeros(0, np.int32))
        st.cfk_update(CfkUpdates(np.zeros(0, np.int64), z, z, np.zeros(0, np.uint8), dep_off=np.zeros(1, np.uint64),
                                 deps=z))
        hist = int(synth._hlc(w.cfk.txn).max())
        red = synth.advance_redundant(w.redundant, 7, step_frac=0.4, hist_hlc=hist, frac=1.0)
        stats = st.redundant_advance(red)
        assert stats["n_keys"][0] > 0
        w2 = _with_red(w, red)
        t = synth.truncate_to_redundant(w.cfk, red, bool(w.range_start_inclusive))
        off, m = st.cfk_missing()
        assert off.tolist() == t.miss_off.tolist()
        assert m.msb.tolist() == t.miss.msb.tolist() and m.lsb.tolist() == t.miss.lsb.tolist()
        for scan in A.RECOVER_SCANS:
            got = st.recovery_scan(w2.queries, scan)
            ok, why = got.equals(oracle.recover(w2, scan), detail=True)
            assert ok, (scan, why)
    finally:
        st.close()


def test_advance_errors():
    w = synth.random_small(4600, n_redundant=4)
    st = native.DeviceCommandStore(0, w.range_start_inclusive, 1, w.slices)
    try:
        st.load(w)
        red = w.redundant
        live = np.nonzero(red.wm.msb != 0)[0]
        i = int(live[0])
        back = Tids(red.wm.msb.copy(), red.wm.lsb.copy(), red.wm.node.copy())
        back.msb[i], back.lsb[i], back.node[i] = 0, 0, 0
        for bad in (Redundant(red.range_start, red.range_end, red.start_epoch, red.end_epoch, back),
                    Redundant(red.range_start[:-1], red.range_end[:-1], red.start_epoch[:-1], red.end_epoch[:-1],
                              red.wm.take(np.arange(len(red.range_start) - 1)))):
            with pytest.raises(native.AccordDepsError) as e:
                st.redundant_advance(bad)
            assert e.value.code == A.AD_E_INVAL
        # the store still answers as loaded
        got = st.calculate_partial_deps(w.queries, w.flags)
        assert got.equals(native.resolve(w))
    finally:
        st.close()


@pytest.mark.parametrize("path", [0, 1])
def test_advance_merging_without_removals(oracle, path):
    # new watermarks older than the dictionary's newest id but below every entry: the dictionary merges (every
    # stored rank moves), nothing is truncated -- the derived arrays must follow the merge alone
    from accord_deps.model import make_txn_ids
    w = synth.with_redundant_ranges(synth.config2(n_txns=4000, n_keys=4000, n_hist_entries=40000), 12, seed=4,
                                    none_frac=1.0)
    st = native.DeviceCommandStore(0, w.range_start_inclusive, 1, w.slices, path=path)
    try:
        st.load(w)
        red = w.redundant
        n = len(red.range_start)
        low = make_txn_ids(1, np.zeros(n, np.uint64), A.KIND_EXCLUSIVE_SYNC_POINT, np.arange(n) + 1, domain=1)
        red2 = Redundant(red.range_start, red.range_end, red.start_epoch, red.end_epoch, low)
        stats = st.redundant_advance(red2)
        assert stats["n_keys"][0] == 0 and stats["n_keys"][2] == n
        got = st.calculate_partial_deps(w.queries, w.flags)
        ok, why = got.equals(oracle.resolve(_with_red(w, red2)), detail=True)
        assert ok, why
    finally:
        st.close()
