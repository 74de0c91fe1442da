"""GPU parity: libaccord_deps (HIP, through the C ABI) vs the CPU restatement of the reference.

Bit-exact comparison of all three RelationMultiMaps of every request's PartialDeps
(keys, txnIds, keysToTxnIds), i.e. Deps.equals (Deps.java:294-303).
"""
import numpy as np
import pytest

from accord_deps import _abi as A
from accord_deps import native, synth

pytestmark = pytest.mark.gpu


def _compare(w, oracle, elide=1, paths=(0, 1)):
    """Both device paths: 0 = fused per-request kernel (+ split fallback), 1 = split kernels only."""
    exp = oracle.resolve(w, elide=elide)
    first = None
    for path in paths:
        got = native.resolve(w, elide=elide, path=path)
        ok, why = got.equals(exp, detail=True)
        if not ok:
            mm = got.first_mismatch(exp)
            raise AssertionError("%s path %d: %s; first mismatch %r" % (w.name, path, why, mm))
        first = first or got
    return first, exp


@pytest.mark.parametrize("seed", range(40))
def test_random_small(oracle, seed):
    w = synth.random_small(seed, with_slices=(seed % 4 == 3), start_inclusive=(seed % 5 == 4))
    _compare(w, oracle)


@pytest.mark.parametrize("via", ["device", "regions"])
@pytest.mark.parametrize("seed", range(12))
def test_random_small_device_outputs(oracle, seed, via):
    # the device entry point read back from the packed arrays and from the regions (AD_REGIONS): lean,
    # general, split and heavy-request paths all write the regions the result points at
    w = synth.random_small(200 + seed, with_slices=(seed % 4 == 3), n_range_cmds=(0 if seed % 3 == 0 else 30),
                           n_redundant=(0 if seed % 2 == 0 else 3), accept_frac=0.1 * (seed % 3), max_keys=2 + seed % 9)
    exp = oracle.resolve(w)
    got = native.resolve(w, via=via)
    ok, why = got.equals(exp, detail=True)
    assert ok, "%s via %s: %s; first mismatch %r" % (w.name, via, why, got.first_mismatch(exp))


@pytest.mark.parametrize("big", ["64", "100000"])
def test_big_requests_regions(oracle, big, monkeypatch):
    monkeypatch.setenv("AD_K2_BIG", big)       # heavy requests on the workgroup build (64) or one wave
    w = synth.random_small(77, n_keys=40, n_hist_txns=6000, n_txns=300, max_keys=8, n_range_cmds=50)
    got = native.resolve(w, via="regions")
    ok, why = got.equals(oracle.resolve(w), detail=True)
    assert ok, why


@pytest.mark.parametrize("even", ["0", "1"])
@pytest.mark.parametrize("case", ["heavy", "light", "mixed"])
def test_pack_copy_paths(oracle, even, case, monkeypatch):
    # the packed copy by k_pack_tiles (a wave per 64 requests) or k_pack_even (chunks of the output, the
    # chunk's requests in LDS windows of 1024: "light" has chunks spanning several windows, "heavy" requests
    # spanning several chunks)
    monkeypatch.setenv("AD_PACK_EVEN", even)
    if case == "heavy":
        w = synth.config2(n_txns=300, n_keys=40, n_hist_entries=60000, keys_per_txn=8, tail_unapplied=8000)
    elif case == "light":
        w = synth.random_small(3100, n_keys=900, n_hist_txns=300, n_txns=6000, max_keys=2)
    else:
        w = synth.random_small(3101, n_keys=300, n_hist_txns=4000, n_txns=3000, max_keys=6, n_range_cmds=40)
    _compare(w, oracle, paths=(0,))
    got = native.resolve(w, via="device")
    ok, why = got.equals(oracle.resolve(w), detail=True)
    assert ok, why


@pytest.mark.parametrize("n_hist", [7, 15, 16, 17, 120, 255, 256, 257, 511, 4097])
def test_dictionary_sample_windows(oracle, n_hist):
    # rank searches through the two-level dictionary sample (common.hpp dict_rank_sampled: every 256th
    # id, then every 16th inside that window, then 16 ids) around the windows' edges: half the requests
    # are Accepts (S = a proposed executeAt the store may hold, self = a txnId it holds), a fifth of the
    # executeAts lie below their txnIds
    w = synth.random_small(3000 + n_hist, n_keys=30, n_hist_txns=n_hist, n_txns=200, accept_frac=0.5,
                           exec_below_frac=0.2, n_range_cmds=0, n_redundant=0)
    _compare(w, oracle)


@pytest.mark.parametrize("seed", range(6))
def test_random_small_no_elision(oracle, seed):
    _compare(synth.random_small(100 + seed), oracle, elide=0)


@pytest.mark.parametrize("seed", range(4))
def test_random_larger(oracle, seed):
    w = synth.random_small(1000 + seed, n_keys=300, n_hist_txns=3000, n_txns=800, max_keys=8, n_range_cmds=200)
    _compare(w, oracle)


@pytest.mark.parametrize("rpw", ["2", "4", "8"])
@pytest.mark.parametrize("seed", range(16))
def test_random_small_lean_store(oracle, seed, rpw, monkeypatch):
    # lean pass 1 with two, four or eight requests per wave
    monkeypatch.setenv("AD_LEAN_RPW", rpw)
    # no range commands / redundant-before: the lean kernel runs first; older requests defer
    w = synth.random_small(500 + seed, n_range_cmds=0, n_redundant=0, accept_frac=0.2 * (seed % 4),
                           max_keys=2 + seed % 7)
    _compare(w, oracle, paths=(0,))


@pytest.mark.parametrize("rpw", ["2", "4", "8"])
@pytest.mark.parametrize("seed", range(16))
def test_random_small_lean_ranges(oracle, seed, rpw, monkeypatch):
    monkeypatch.setenv("AD_LEAN_RPW", rpw)
    # range commands with their stabbing index, no redundant-before: the lean kernel also builds
    # rangeDeps (multi-range commands, both range conventions, slices, erased ranges)
    w = synth.random_small(800 + seed, n_range_cmds=10 + 6 * seed, n_redundant=0, accept_frac=0.1 * (seed % 3),
                           max_keys=2 + seed % 7, start_inclusive=(seed % 2 == 1), with_slices=(seed % 4 == 2))
    # move (every other / every) request to epoch 3, newer than every id of the store, so it takes
    # the lean path; the rest defer to the general kernel
    q = w.queries
    sel = np.arange(len(q.txn.msb)) % (1 + seed % 2) == 0
    for ts in (q.txn, q.exec):
        ts.msb[sel] = (ts.msb[sel] & np.uint64(0x7FFF)) | np.uint64(3 << 15)
    got, _ = _compare(w, oracle, paths=(0,))
    assert got.stats["n_deferred_lean"] < len(w.queries)


@pytest.mark.parametrize("seed", range(4))
def test_range_build_64bit_words(oracle, seed, monkeypatch):
    # the lean kernels' rangeDeps build in 64-bit words (range id << 32 | rank; AD_RNG64): the path of stores
    # with 2^26 or more range ids or dictionary ranks, which the 32-bit build (rng32) cannot hold
    monkeypatch.setenv("AD_RNG64", "1")
    w = synth.random_small(820 + seed, n_range_cmds=40 + 10 * seed, n_redundant=0, max_keys=2 + seed % 7,
                           start_inclusive=(seed % 2 == 1))
    q = w.queries
    for ts in (q.txn, q.exec):                 # newer than the store: the lean kernels take them
        ts.msb[:] = (ts.msb & np.uint64(0x7FFF)) | np.uint64(3 << 15)
    _compare(w, oracle, paths=(0,))


@pytest.mark.parametrize("esp,sync,reads", [(0.0, 0.0, False), (0.3, 0.05, False), (0.0, 0.02, True)])
def test_config2_lean_classes(oracle, esp, sync, reads, monkeypatch):
    # every witness class on the lean path (Read -> Ws, Write -> RsOrWs, ExclusiveSyncPoint ->
    # AnyGloballyVisible incl. SyncPoints), with and without the lean kernel
    w = synth.config2(n_txns=4000, n_keys=20000, n_hist_entries=300000, esp_frac=esp, sync_frac=sync)
    if reads:
        w.queries.txn.lsb[:] = w.queries.txn.lsb & ~np.uint64(0xE)          # all Read
        w.queries.exec.lsb[:] = w.queries.txn.lsb
    got, exp = _compare(w, oracle, paths=(0,))
    assert got.stats["n_deferred_lean"] < len(w.queries)
    monkeypatch.setenv("AD_LEAN_RPW", "4")
    assert native.resolve(w).equals(exp)
    monkeypatch.delenv("AD_LEAN_RPW")
    monkeypatch.setenv("AD_NO_LEAN", "1")
    got2 = native.resolve(w)
    assert got2.equals(exp)


def test_lean_requests_below_newest_txn(oracle, monkeypatch):
    # late PreAccepts older than busy keys' newest txnIds (their uncommitted tail) but newer than
    # the keys' last committed Write: maxCommittedWriteBefore(S) is still the last committed Write,
    # so the lean kernel serves them with the rank < S filter (insertPos(S),
    # CommandsForKey.java:912-928) instead of deferring them to the tree descent
    from accord_deps.model import CfkSnapshot, Workload
    w = synth.config2(n_txns=4000, n_keys=2000, n_hist_entries=200000, tail_unapplied=6)
    c = w.cfk
    st = c.status.copy()
    st[(st == A.ST_COMMITTED) | (st == A.ST_STABLE)] = A.ST_ACCEPTED       # the tails stay uncommitted
    w = Workload(w.name, CfkSnapshot(c.keys, c.seg, c.txn, c.exec, st, c.pruned_before), w.cmds, w.redundant,
                 w.queries, w.flags, w.params, w.range_start_inclusive, w.slices)
    w = synth.with_request_mix(w, unordered_frac=1.0, unordered_window=6)
    q = w.queries
    seg = c.seg.astype(np.int64)
    last_hlc = (c.txn.lsb[seg[1:] - 1] >> np.uint64(16)).astype(np.int64)
    kidx = np.searchsorted(c.keys, q.keys)
    kidx_c = np.minimum(kidx, len(c.keys) - 1)
    held = c.keys[kidx_c] == q.keys
    req = np.repeat(np.arange(len(q.txn.msb)), np.diff(q.key_off.astype(np.int64)))
    older_key = held & (last_hlc[kidx_c] >= (q.txn.lsb[req] >> np.uint64(16)).astype(np.int64))
    n_older = len(np.unique(req[older_key]))
    got, exp = _compare(w, oracle, paths=(0,))
    assert n_older > 500
    assert got.stats["n_deferred_lean"] < n_older // 2
    monkeypatch.setenv("AD_NO_LEAN", "1")
    assert native.resolve(w).equals(exp)


def test_config1_sequential(oracle):
    got, exp = _compare(synth.config1(), oracle)
    assert got.pair_count(A.AD_MAP_KEY) > 0


def test_config2_scaled(oracle):
    w = synth.config2(n_txns=3000, n_keys=30000, n_hist_entries=400000, esp_frac=0.01)
    got, exp = _compare(w, oracle)
    assert got.pair_count(A.AD_MAP_DIRECT_KEY) > 0


def test_config3_scaled_sharded(oracle):
    w = synth.config3(n_txns=400_000, n_keys=50_000)
    lo, hi = synth.shard_bounds(4)
    for g in range(4):
        _compare(synth.slice_workload(w, lo[g], hi[g]), oracle)


def test_config4_scaled(oracle):
    w = synth.config4(n_txns=3000, n_keys=20000, n_ranges=5000, n_hist_txns=20000)
    got, exp = _compare(w, oracle)
    assert got.pair_count(A.AD_MAP_RANGE) > 0


@pytest.mark.parametrize("seed", range(6))
def test_range_tree_fallback(oracle, seed, monkeypatch):
    # no stabbing index (coverage budget 0): every range probe takes the max-end tree descent
    monkeypatch.setenv("AD_CELL_BUDGET", "0")
    _compare(synth.random_small(700 + seed, n_range_cmds=40, start_inclusive=(seed % 2 == 1)), oracle)
    _compare(synth.config4(n_txns=1000, n_keys=5000, n_ranges=800, n_hist_txns=4000, seed=seed), oracle, paths=(0,))


def test_big_requests(oracle):
    # a hot key with thousands of live entries -> per-probe outputs beyond the LDS staging
    w = synth.config2(n_txns=200, n_keys=50, n_hist_entries=40000, keys_per_txn=8, tail_unapplied=3000,
                      esp_frac=0.2)
    got, _ = _compare(w, oracle)
    assert got.stats["n_deferred"] > 0          # exercised the fused -> split hand-off


@pytest.mark.parametrize("sort", ["8192", "8192/rank", "0", "0/rank"])
@pytest.mark.parametrize("big", ["0", "64", "512"])
def test_big_requests_workgroup_build(oracle, big, sort, monkeypatch):
    # k_build_big (one 1024-thread workgroup per heavy request): every request (0), the medium ones
    # (64) or the default threshold, on hot keys with thousands of live entries, range commands and
    # RedundantBefore in the mix
    monkeypatch.setenv("AD_K2_BIG", big)
    # its maps merged in LDS (by the merge tree, or the rank merge) or in global scratch
    monkeypatch.setenv("AD_KB_SORT", sort.split("/")[0])
    monkeypatch.setenv("AD_KB_MERGE", "0" if sort.endswith("/rank") else "1")
    w = synth.config2(n_txns=200, n_keys=50, n_hist_entries=40000, keys_per_txn=8, tail_unapplied=3000,
                      esp_frac=0.2)
    _compare(w, oracle)
    _compare(synth.random_small(2100 + int(big), n_keys=40, n_hist_txns=2000, n_txns=200, max_keys=10,
                                n_range_cmds=60), oracle)


def test_many_keys_deferred(oracle):
    # requests with more than 8 keys take the split kernels from the fused kernel
    w = synth.random_small(2024, n_keys=200, n_hist_txns=2000, n_txns=300, max_keys=20, n_range_cmds=50)
    got, _ = _compare(w, oracle)
    assert got.stats["n_deferred"] > 0


def test_empty_batch_and_empty_snapshot(oracle):
    w = synth.random_small(3)
    w.queries = w.queries.window(0, 0)
    _compare(w, oracle)


@pytest.mark.parametrize("seed", range(4))
def test_ranges_without_cfk(oracle, seed, monkeypatch):
    # range commands (and redundant-before for odd seeds) on a store with no CommandsForKey: every
    # probe misses the key index but still reads its range cell / tree
    from accord_deps.model import CfkSnapshot
    w = synth.random_small(900 + seed, n_range_cmds=30, n_redundant=3 * (seed % 2), start_inclusive=(seed % 4 >= 2))
    w.cfk = CfkSnapshot.empty()
    _compare(w, oracle, paths=(0,))
    monkeypatch.setenv("AD_CELL_BUDGET", "0")
    _compare(w, oracle, paths=(0,))


def test_errors():
    w = synth.random_small(5)
    st = native.DeviceCommandStore()
    st.load(w)
    q = w.queries
    bad = q.window(0, len(q))
    i = int(np.argmax(np.diff(bad.key_off.astype(np.int64)) >= 2))
    k0 = int(bad.key_off[i])
    bad.keys[k0], bad.keys[k0 + 1] = bad.keys[k0 + 1], bad.keys[k0]
    with pytest.raises(native.AccordDepsError) as e:
        st.calculate_partial_deps(bad)
    assert e.value.code == A.AD_E_INVAL


@pytest.mark.parametrize("seed", range(6))
def test_ephemeral_reads_at_timestamp_max(oracle, seed):
    # GetEphemeralReadDeps (GetEphemeralReadDeps.java:76): executeAt = Timestamp.MAX -- a request above
    # every id of the store, on the lean path (no range commands) and the general one (with them)
    base = synth.random_small(700 + seed, n_keys=200, n_hist_txns=2000, n_txns=500, max_keys=8,
                              n_range_cmds=0 if seed % 2 else 100, n_redundant=0 if seed % 2 else 4)
    _compare(synth.with_ephemeral_reads(base, frac=0.5, seed=seed), oracle)


def test_ephemeral_reads_config2_scaled(oracle):
    w = synth.with_ephemeral_reads(synth.config2(n_txns=20000, n_keys=20000, n_hist_entries=200000), frac=0.3)
    _compare(w, oracle, paths=(0,))


@pytest.mark.parametrize("gap_bits", [40, 62])
def test_dictionary_bucket_index_clusters(oracle, gap_bits):
    # the rank searches' bucket index (common.hpp dict_bucket_of) spreads the dictionary's 128-bit span over
    # its buckets: ids in two clusters 2^gap_bits epochs apart leave nearly every bucket empty and each
    # cluster in one or two buckets, so the searches run over wide bucket ranges -- still exact. The ids of
    # the request mix (Accepts' executeAt and txnId, late PreAccepts) all need the search; the shift is
    # monotone, so the reference's answers keep their meaning
    import dataclasses
    from accord_deps.model import Tids
    w = synth.config2(n_txns=4000, n_keys=2000, n_hist_entries=200000)
    w = synth.with_request_mix(w, accept_frac=0.3, unordered_frac=0.3, unordered_window=3000)
    c, q = w.cfk, w.queries
    hlc_all = np.concatenate([(t.lsb >> np.uint64(16)) for t in (c.txn, c.exec, q.txn, q.exec)])
    pivot = np.uint64(np.median(hlc_all.astype(np.float64)))
    gap = np.uint64(1) << np.uint64(gap_bits)

    def shift(t):
        up = (t.lsb >> np.uint64(16)) >= pivot          # one epoch throughout: (msb, hlc) order is hlc order
        return Tids(np.where(up, t.msb + gap, t.msb).astype(np.uint64), t.lsb.copy(), t.node.copy())

    assert len(np.unique(c.txn.msb)) == 1 and len(np.unique(q.exec.msb)) == 1
    w = dataclasses.replace(w, cfk=dataclasses.replace(c, txn=shift(c.txn), exec=shift(c.exec)),
                            queries=dataclasses.replace(q, txn=shift(q.txn), exec=shift(q.exec)))
    got, exp = _compare(w, oracle, paths=(0,))
    assert got.stats["n_deferred_lean"] > 0
