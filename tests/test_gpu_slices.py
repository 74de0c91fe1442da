"""GPU parity of per-request slices (ad_query_soa.slice_set, ad_slice_sets_load): a batch of a store whose ownership
changed over epochs, each request scanning safeStore.ranges().allBetween(minUnsyncedEpoch, txnId | executeAt)
(PreAccept.java:100,130, Accept.java:115; CommandStores.java:233-242), some the store's own slices. Bit-exact against
the oracle (refcpu.c slice_select, pinned by the model in tests/test_slices.py) on every path that slices: the lean
kernels (KeyLines from k_prepare, and the range-command instantiation's own slice test), the general kernel, the
split kernels and their deferred sub-batch, Range-domain expansion, the device and host entry points, the
PCIe-facing ad_deps_batch_into and the recovery scans."""
import numpy as np
import pytest

from accord_deps import _abi as A
from accord_deps import native, synth

pytestmark = pytest.mark.gpu


def _check(w, oracle, paths=(0, 1), via="host"):
    exp = oracle.resolve(w)
    for path in paths:
        got = native.resolve(w, path=path, via=via)
        ok, why = got.equals(exp, detail=True)
        assert ok, "%s path %d via %s: %s; first mismatch %r" % (w.name, path, via, why, got.first_mismatch(exp))
    return exp


def _newer(w):
    """Every request newer than the store (epoch 4): the lean kernels take them."""
    q = w.queries
    for ts in (q.txn, q.exec):
        ts.msb[:] = (ts.msb & np.uint64(0x7FFF)) | np.uint64(4 << 15)
    return w


@pytest.mark.parametrize("rpw", ["2", "4", "8"])
@pytest.mark.parametrize("seed", range(6))
def test_lean_store(oracle, seed, rpw, monkeypatch):
    # no range commands / RedundantBefore: lean pass 1 reads the KeyLine k_prepare found under the request's slice
    monkeypatch.setenv("AD_LEAN_RPW", rpw)
    w = synth.random_small(1600 + seed, n_keys=60, n_range_cmds=0, n_redundant=0, max_keys=2 + seed % 7,
                           with_slices=(seed % 2 == 1), accept_frac=0.0)
    w = synth.with_epoch_slices(_newer(w), seed, n_epochs=4, store_every=(0 if seed % 3 == 0 else 4))
    _check(w, oracle, paths=(0,))


@pytest.mark.parametrize("seed", range(8))
def test_range_store(oracle, seed):
    # range commands with their stabbing index: the lean range instantiation tests the slice itself
    w = synth.random_small(1700 + seed, n_keys=60, n_range_cmds=20 + 5 * seed, n_redundant=0, max_keys=2 + seed % 7,
                           start_inclusive=(seed % 2 == 1), with_slices=(seed % 4 == 2))
    w = synth.with_epoch_slices(_newer(w) if seed % 2 else w, seed, n_epochs=4 if seed % 2 else 3,
                                store_every=(0 if seed % 3 == 0 else 3))
    _check(w, oracle)


@pytest.mark.parametrize("seed", range(10))
def test_mixed_stores_and_range_requests(oracle, seed):
    # RedundantBefore (general kernel), Range-domain requests (their expansion, the split kernels' sub-batch)
    w = synth.random_small(1800 + seed, n_keys=50 + seed, n_txns=120, range_frac=0.3, n_redundant=4 * (seed % 2),
                           n_range_cmds=(0 if seed % 5 == 4 else 16), with_slices=(seed % 3 == 1),
                           start_inclusive=(seed % 4 == 3))
    w = synth.with_epoch_slices(w, seed, store_every=(0 if seed % 2 else 4))
    _check(w, oracle)


@pytest.mark.parametrize("via", ["device", "regions"])
@pytest.mark.parametrize("seed", range(4))
def test_device_entry(oracle, seed, via):
    # slice_set as a device array (ad_deps_batch_device)
    w = synth.random_small(1900 + seed, n_keys=60, range_frac=0.2 * (seed % 2), n_range_cmds=(0 if seed < 2 else 20),
                           n_redundant=0)
    w = synth.with_epoch_slices(w, seed, store_every=3)
    _check(w, oracle, paths=(0,), via=via)


def test_host_api_into(oracle):
    # ad_deps_batch_into: a batch naming slice sets takes the staged path, sliced
    w = synth.with_epoch_slices(synth.random_small(2000, n_keys=80, n_txns=300, max_keys=6, n_range_cmds=30), 3)
    st = native.DeviceCommandStore(0, w.range_start_inclusive, 1, w.slices)
    try:
        st.load(w)
        for slices in (1, 3):
            got, stats, out = st.deps_batch_into(w.queries, slices=slices)
            ok, why = got.equals(oracle.resolve(w), detail=True)
            assert ok, why
            out.release()
    finally:
        st.close()


@pytest.mark.parametrize("scan", [0, 1, 2, 3])
def test_recovery_scans(oracle, scan):
    for seed in range(3):
        w = synth.with_epoch_slices(synth.recovery_workload(2100 + seed, n_known=30, range_frac=0.3 * (seed % 2)), seed + 11)
        exp = oracle.recover(w, scan)
        got = native.recover(w, scan)
        ok, why = got.equals(exp, detail=True)
        assert ok, (seed, scan, why)


def test_config2_scaled_two_epochs(oracle):
    # a config-2-shaped batch in the middle of a topology change: half the requests see the old epoch's slice
    w = synth.config2(n_txns=20000, n_keys=20000, n_hist_entries=200000)
    q = w.queries
    half = np.arange(len(q)) % 2 == 0               # half the requests in epoch 2 (still newer than the store)
    for ts in (q.txn, q.exec):
        ts.msb[half] = (ts.msb[half] & np.uint64(0x7FFF)) | np.uint64(2 << 15)
    w = synth.with_epoch_slices(w, 5, n_epochs=2)
    assert len(w.slice_sets) == 2                    # allBetween(1, 1): epoch 1 only; the rest: every key
    exp = oracle.resolve(w)
    got = native.resolve(w)
    assert got.equals(exp)
    assert got.stats["n_deferred_lean"] < len(w.queries)       # the lean kernels took them


def test_slice_set_beyond_the_sets(oracle):
    w = synth.with_epoch_slices(synth.random_small(2200, n_keys=40), 1)
    w.queries.slice_set[5] = len(w.slice_sets) + 2
    with pytest.raises(native.AccordDepsError) as e:
        native.resolve(w)
    assert e.value.code == A.AD_E_INVAL
    with pytest.raises(native.AccordDepsError) as e:
        native.resolve(w, via="device")
    assert e.value.code == A.AD_E_INVAL
