"""GPU parity of the PCIe-facing batch path a Java host binds (ad_deps_batch_into):
host query arrays in, caller-owned pinned host arrays out, the batch resolved in slices whose copy-out
overlaps the next slice. Results must equal the reference restatement (oracle) and ad_deps_batch's,
for every slicing, after growing too-small outputs (AD_E_SPACE), for SEQUENTIAL batches and for empty
batches."""
import numpy as np
import pytest

from accord_deps import _abi as A
from accord_deps import native, synth

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("slices", [1, 3])
def test_into_matches_oracle(oracle, seed, slices):
    w = synth.random_small(seed, n_keys=80, n_hist_txns=600, n_txns=300, max_keys=6, n_range_cmds=40)
    st = native.DeviceCommandStore(0, w.range_start_inclusive, 1, w.slices)
    try:
        st.load(w)
        got, stats, out = st.deps_batch_into(w.queries, slices=slices)
        ok, why = got.equals(oracle.resolve(w), detail=True)
        assert ok, why
        assert stats["n_txns"] == len(w.queries)
        out.release()
    finally:
        st.close()


@pytest.mark.parametrize("wire", ["1", "0"])
def test_into_config2_scaled_slicings_and_growth(wire, monkeypatch):
    # wire "0" (AD_INTO_WIRE=0): keyDeps cross PCIe full width (the path of slices whose segments do not fit
    # the u8 key / u16 keysToTxnIds wire form), on every slicing
    monkeypatch.setenv("AD_INTO_WIRE", wire)
    w = synth.config2(n_txns=60000, n_keys=40000, n_hist_entries=600000)
    st = native.DeviceCommandStore(0)
    try:
        st.load(w)
        ref = st.calculate_partial_deps(w.queries)
        out = None
        for slices in (1, 2, 4, 7):
            got, stats, out = st.deps_batch_into(w.queries, slices=slices, out=out)
            ok, why = got.equals(ref, detail=True)
            assert ok, (slices, why)
        out.release()
        # outputs far too small: AD_E_SPACE, then grown to the sizes the batch reported
        small = native.DeviceCommandStore.HostOut(st, len(w.queries), [1] * 9)
        got, _, out = st.deps_batch_into(w.queries, slices=3, out=small)
        ok, why = got.equals(ref, detail=True)
        assert ok, why
        assert out is not small
        out.release()
    finally:
        st.close()


def test_into_unpinned_outputs():
    w = synth.random_small(21, n_keys=60, n_hist_txns=400, n_txns=200)
    st = native.DeviceCommandStore(0, w.range_start_inclusive, 1, w.slices)
    try:
        st.load(w)
        got, _, _ = st.deps_batch_into(w.queries, slices=2, pin=False)
        ok, why = got.equals(st.calculate_partial_deps(w.queries), detail=True)
        assert ok, why
    finally:
        st.close()


def test_into_sequential_config1(oracle):
    w = synth.config1(n_txns=2000)
    st = native.DeviceCommandStore(0)
    try:
        st.load(w)
        got, _, out = st.deps_batch_into(w.queries, flags=A.AD_SEQUENTIAL, slices=4)
        ok, why = got.equals(oracle.resolve(w), detail=True)
        assert ok, why
        out.release()
    finally:
        st.close()


def test_into_empty_batch_and_bad_keys():
    w = synth.random_small(3)
    st = native.DeviceCommandStore(0, w.range_start_inclusive, 1, w.slices)
    try:
        st.load(w)
        got, stats, out = st.deps_batch_into(w.queries.take(np.zeros(0, np.int64)))
        assert got.n_txns == 0 and stats["n_txns"] == 0
        out.release()
        # keys of a request not ascending: AD_E_INVAL from the (threaded) host check, nothing resolved
        q = w.queries
        bad = q.take(np.arange(len(q)))
        i = int(np.nonzero(np.diff(bad.key_off.astype(np.int64)) >= 2)[0][0])
        a, b = int(bad.key_off[i]), int(bad.key_off[i] + 1)
        bad.keys[a], bad.keys[b] = bad.keys[b], bad.keys[a]
        with pytest.raises(native.AccordDepsError) as ei:
            st.deps_batch_into(bad, pin=False)
        assert ei.value.code == A.AD_E_INVAL and ("request %d" % i) in str(ei.value)
        # key_off not monotone (in the last slice of a sliced call): AD_E_INVAL naming the request
        bad = q.take(np.arange(len(q)))
        j = len(bad) - 2
        bad.key_off[j + 1] = bad.key_off[j] - 1 if bad.key_off[j] > 0 else bad.key_off[j + 2] + 1
        with pytest.raises(native.AccordDepsError) as ei:
            st.deps_batch_into(bad, slices=3)
        assert ei.value.code == A.AD_E_INVAL
    finally:
        st.close()


def test_into_registered_outputs():
    # the Panama binding's way: the caller's own pages pinned with ad_host_register (whole pages), reused
    # across batches and slicings, then unpinned; same results as the library-pinned outputs
    w = synth.config2(n_txns=30000, n_keys=20000, n_hist_entries=300000)
    st = native.DeviceCommandStore(0)
    try:
        st.load(w)
        ref = st.calculate_partial_deps(w.queries)
        out = None
        for slices in (1, 3):
            got, _, out = st.deps_batch_into(w.queries, slices=slices, out=out, pin="register")
            ok, why = got.equals(ref, detail=True)
            assert ok, (slices, why)
        out.release()
    finally:
        st.close()


def test_host_alloc_contract():
    import ctypes as C
    p = C.c_void_p()
    assert native.lib().ad_host_alloc(0, C.byref(p)) == A.AD_E_INVAL and not p.value
    assert native.lib().ad_host_alloc(1 << 20, C.byref(p)) == 0 and p.value and p.value % 4096 == 0
    assert native.lib().ad_host_free(p) == 0
    assert native.lib().ad_host_free(None) == 0


@pytest.mark.parametrize("pin", [True, "register"])
def test_views_outlive_their_hostout(pin):
    # an array taken from a HostOut stays valid after the HostOut is released and collected: each block of
    # output memory is its arrays' base, freed / unpinned by its own finalizer once no array is left
    import gc
    w = synth.random_small(5, n_keys=80, n_hist_txns=600, n_txns=300, max_keys=6, n_range_cmds=40)
    st = native.DeviceCommandStore(0, w.range_start_inclusive, 1, w.slices)
    try:
        st.load(w)
        _, _, out = st.deps_batch_into(w.queries, pin=pin, materialise=False)
        keep = out.txns[0][:int(out.off[1][-1])]                 # a view, not a copy
        off = out.off                                            # the offsets block
        exp_k, exp_o = keep.copy(), off.copy()
        out.release()
        del out
        gc.collect()
        # new pinned allocations that would reuse freed pages
        more = [native.DeviceCommandStore.HostOut(st, len(w.queries), [4096] * 9, pin) for _ in range(3)]
        assert np.array_equal(keep, exp_k) and np.array_equal(off, exp_o)
        del more, keep, off
        gc.collect()
        # a caller's HostOut reused across batches is not released by the call
        out2 = native.DeviceCommandStore.HostOut(st, len(w.queries), [1 << 16] * 9, pin)
        _, _, out3 = st.deps_batch_into(w.queries, out=out2, materialise=False)
        assert out3 is out2 and out2.off is not None
    finally:
        st.close()


def test_staged_upload_after_destroyed_context(oracle):
    # the hazard commit 7295a85 closed: a staged pageable upload on context A (columns larger than
    # one 8 MiB staging chunk, so both chunks of the pair carry events), A destroyed with its stream, then at once
    # a staged upload on a fresh context B drawing the same staging pair from the pool -- B's uploads must not wait
    # on events recorded on A's destroyed stream. Run once per suite; each round is checked bit-exact.
    w = synth.config2(n_txns=4000, n_keys=20000, n_hist_entries=400000)
    exp = oracle.resolve(w)
    for _ in range(3):
        a = native.DeviceCommandStore(0)
        a.load(w, prepare=False)               # staged H2D of the pageable columns on A's stream
        a.close()                              # ad_ctx_destroy: A's stream goes
        b = native.DeviceCommandStore(0)
        try:
            b.load(w)                          # staged again, same pool pair, fresh stream
            got = b.calculate_partial_deps(w.queries, w.flags)
        finally:
            b.close()
        ok, why = got.equals(exp, detail=True)
        assert ok, why
