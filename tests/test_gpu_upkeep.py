"""GPU parity of the range-command registry's upkeep without a snapshot rebuild (ad_range_cmds_update:
InMemorySafeStore.update, InMemoryCommandStore.java:740-763; RangeCommand.update :547-551 with Ranges.with,
AbstractRanges.java:486-574; historicalRangeCommands.merge :814-828; erased commands skipped :892): successive
upkeep batches on a loaded store -- registrations, unions with more ranges, erasures, historical merges -- then
batches bit-exact against the oracle store given the same rows (rc_range_cmds_update, pinned by
tests/test_truncate.py against the model refmodel.range_cmds_update)."""
import numpy as np
import pytest

from accord_deps import _abi as A
from accord_deps import native, synth
from accord_deps.model import RangeCommands, Tids

pytestmark = pytest.mark.gpu


def _run(w, oracle, steps, rows, path=0, seed=0, via="host"):
    import pyoracle
    st = native.DeviceCommandStore(0, w.range_start_inclusive, 1, w.slices, path=path)
    orc = pyoracle.OracleStore(w.range_start_inclusive, 1, w.slices)
    try:
        st.load(w)
        orc.load(w)
        cmds = w.cmds
        import refmodel
        for step in range(steps):
            u = synth.range_cmd_updates(cmds, 1000 * seed + step, rows)
            stats = st.range_cmds_update(u)
            orc.range_cmds_update(u)
            cmds = refmodel.range_cmds_update(cmds, u)
            exp = orc.deps_batch(w.queries, w.flags)
            if via == "host":
                got = st.calculate_partial_deps(w.queries, w.flags)
            else:
                import torch
                qdev, keep = native.device_queries(w.queries, torch.device("cuda", 0))
                res, _ = st.deps_batch_device(qdev)
                torch.cuda.synchronize()
                got = st.device_result_to_host(res)
            ok, why = got.equals(exp, detail=True)
            assert ok, (step, why, got.first_mismatch(exp))
        return stats
    finally:
        st.close()
        orc.close()


@pytest.mark.parametrize("path", [0, 1])
@pytest.mark.parametrize("seed", range(8))
def test_registry_upkeep(oracle, seed, path):
    w = synth.random_small(5000 + seed, n_keys=50, n_hist_txns=300, n_txns=120, n_range_cmds=10 + 4 * seed,
                           range_frac=0.3 * (seed % 2), with_slices=(seed % 3 == 1), start_inclusive=(seed % 4 == 2))
    _run(w, oracle, 3, 16, path=path, seed=seed)


@pytest.mark.parametrize("seed", range(3))
def test_registry_upkeep_device_entry(oracle, seed):
    w = synth.random_small(5100 + seed, n_keys=50, n_hist_txns=300, n_txns=120, n_range_cmds=20)
    _run(w, oracle, 2, 16, seed=seed, via="device")


def test_registry_upkeep_from_empty(oracle):
    # a store without range commands gains its first ones (the range part and stabbing index appear)
    w = synth.random_small(5200, n_keys=60, n_hist_txns=300, n_txns=150, n_range_cmds=0, range_frac=0.2)
    _run(w, oracle, 3, 24, seed=7)


def test_registry_upkeep_config4_scaled(oracle):
    # a config-4-shaped store (range commands over a large key line): batches of registrations and unions
    w = synth.config4(n_txns=3000, n_keys=6000, n_ranges=1500, n_hist_txns=6000)
    lo, hi = int(w.cfk.keys.min()), int(w.cfk.keys.max())
    import pyoracle
    import refmodel
    st = native.DeviceCommandStore(0, w.range_start_inclusive, 1, w.slices)
    orc = pyoracle.OracleStore(w.range_start_inclusive, 1, w.slices)
    try:
        st.load(w)
        orc.load(w)
        cmds = w.cmds
        for step in range(3):
            u = synth.range_cmd_updates(cmds, 77 + step, 200, lo=lo, hi=hi, hlc_hi=900, max_width=(hi - lo) // 400)
            st.range_cmds_update(u)
            orc.range_cmds_update(u)
            cmds = refmodel.range_cmds_update(cmds, u)
            got = st.calculate_partial_deps(w.queries, w.flags)
            ok, why = got.equals(orc.deps_batch(w.queries, w.flags), detail=True)
            assert ok, (step, why)
    finally:
        st.close()
        orc.close()


def test_registry_upkeep_then_sequential(oracle):
    # a SEQUENTIAL batch after upkeep: its Range-domain txns register on top of the updated registry
    w = synth.sequential_ranges(5300, n_keys=40, n_txns=80, n_range_cmds=12)
    import pyoracle
    st = native.DeviceCommandStore(0, w.range_start_inclusive, 1, w.slices)
    orc = pyoracle.OracleStore(w.range_start_inclusive, 1, w.slices)
    try:
        st.load(w)
        orc.load(w)
        u = synth.range_cmd_updates(w.cmds, 9, 10, epoch=1, hlc_hi=50)
        st.range_cmds_update(u)
        orc.range_cmds_update(u)
        got = st.calculate_partial_deps(w.queries, w.flags)
        ok, why = got.equals(orc.deps_batch(w.queries, w.flags), detail=True)
        assert ok, why
    finally:
        st.close()
        orc.close()


def test_registry_upkeep_errors():
    w = synth.random_small(5400, n_range_cmds=8)
    st = native.DeviceCommandStore(0, w.range_start_inclusive, 1, w.slices)
    try:
        st.load(w)
        t = w.cmds.txn.take(np.arange(1))
        key_dom = Tids(t.msb.copy(), t.lsb.copy() & ~np.uint64(1), t.node.copy())
        for bad in (RangeCommands(key_dom, np.array([0, 1], np.uint64), np.array([0], np.int64), np.array([5], np.int64)),
                    RangeCommands(t, np.array([0, 2], np.uint64), np.array([0, 3], np.int64), np.array([5, 9], np.int64)),
                    RangeCommands(t, np.array([0, 1], np.uint64), np.array([5], np.int64), np.array([5], np.int64))):
            with pytest.raises(native.AccordDepsError) as e:
                st.range_cmds_update(bad)
            assert e.value.code == A.AD_E_INVAL
        assert st.calculate_partial_deps(w.queries, w.flags).equals(native.resolve(w))
    finally:
        st.close()


def test_recovery_needs_facts_after_upkeep(oracle):
    # recovery facts describe the registry as loaded: after upkeep the range scans ask for them again
    w = synth.recovery_workload(5500, n_range_cmds=12, range_frac=0.3)
    st = native.DeviceCommandStore(0, w.range_start_inclusive, 1, w.slices)
    try:
        st.load(w)
        st.range_cmds_update(synth.range_cmd_updates(w.cmds, 3, 4))
        with pytest.raises(native.AccordDepsError) as e:
            st.recovery_scan(w.queries, A.RECOVER_SCANS[0])
        assert e.value.code == A.AD_E_STATE
    finally:
        st.close()
