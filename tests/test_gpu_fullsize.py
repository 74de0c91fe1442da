"""GPU parity at BASELINE.json's full sizes: the exact batches bench.py times, resolved on the
device through the C ABI (ad_deps_batch_device), and a sample of their requests compared bit-exactly
(Deps.equals, Deps.java:294-303: keys, txnIds, keysToTxnIds of all three maps) with the CPU
restatement of the reference (oracle/refcpu.c) over the same snapshot.

SNAPSHOT requests are independent (each reads the one immutable snapshot), so the sample -- the
first 2000 requests plus 2000 spread over the whole batch -- is resolved by the oracle as a batch
of its own and must equal those requests' slices of the device result. Size-independent checks
cover every request: CSR well-formedness (RelationMultiMap.checkValid, RelationMultiMap.java:1074-1097)
and the totals.

Configs: 2 (1M txns x 8 Zipf(0.99) keys, 16M-entry history: the headline batch), the same batch as a
replica's mix of fresh PreAccepts, Accepts of in-flight txns (S = executeAt, self excluded:
Accept.java:84-117, PreAccept.java:261) and out-of-order PreAccepts (general kernel), and 4 (1M txns
vs 100k range commands).
"""
import numpy as np
import pytest

from accord_deps import _abi as A
from accord_deps import native, synth

pytestmark = pytest.mark.gpu


def _sample(n, head=2000, spread=2000, seed=7):
    rng = np.random.default_rng(seed)
    idx = np.unique(np.concatenate([np.arange(min(n, head)), rng.choice(n, min(n, spread), replace=False)]))
    return idx


def _check_csr(store, res):
    """RelationMultiMap.checkValid over every request of the device result: heads ascending and
    absolute (nKeys + running count), each key's values strictly ascending indices below nIds, keys
    strictly ascending per request, ids strictly ascending per request."""
    n = res.n_txns
    for m in range(A.NMAPS):
        ko = store._d2h(res.keys_off[m], n + 1, np.uint64).astype(np.int64)
        to = store._d2h(res.txn_off[m], n + 1, np.uint64).astype(np.int64)
        oo = store._d2h(res.k2t_off[m], n + 1, np.uint64).astype(np.int64)
        nk = np.diff(ko)
        nt = np.diff(to)
        no = np.diff(oo)
        assert np.all(no >= nk) and np.all((no > nk) == (nk > 0)), A.MAP_NAMES[m]
        assert np.all((nt > 0) == (nk > 0)), A.MAP_NAMES[m]
        tx = store._d2h(res.txns[m], int(to[-1]), np.uint32).astype(np.int64)
        k2t = store._d2h(res.k2t[m], int(oo[-1]), np.int32).astype(np.int64)
        keys = store._d2h(res.keys[m], int(ko[-1]), np.int64)
        # ids ascending within a request
        req_t = np.repeat(np.arange(n), nt)
        same = req_t[1:] == req_t[:-1]
        assert np.all(tx[1:][same] > tx[:-1][same]), A.MAP_NAMES[m]
        req_k = np.repeat(np.arange(n), nk)
        samek = req_k[1:] == req_k[:-1]
        if m != A.AD_MAP_RANGE:
            assert np.all(keys[1:][samek] > keys[:-1][samek]), A.MAP_NAMES[m]
        # heads: k2t[o0 + j] for j < nk is nk + cumulative count, last one == no
        head_pos = np.repeat(oo[:-1], nk) + (np.arange(int(ko[-1])) - np.repeat(ko[:-1], nk))
        heads = k2t[head_pos]
        end_of_req = np.cumsum(nk) - 1
        assert np.all(heads[end_of_req[nk > 0]] == no[nk > 0]), A.MAP_NAMES[m]
        base = np.repeat(nk, nk)
        prev = np.concatenate([[0], heads[:-1]])
        first = np.ones(len(heads), bool)
        first[1:] = ~samek
        prev[first] = base[first]
        assert np.all(heads > prev), A.MAP_NAMES[m]
        # body values index the request's ids
        body = np.ones(int(oo[-1]), bool)
        body[head_pos] = False
        req_o = np.repeat(np.arange(n), no)
        assert np.all(k2t[body] >= 0) and np.all(k2t[body] < nt[req_o[body]]), A.MAP_NAMES[m]


def _run_full(w, oracle, expect_lean=None):
    import torch
    dev = torch.device("cuda", 0)
    st = native.DeviceCommandStore(device=0, slices=w.slices)
    try:
        st.load(w)
        qdev, keep = native.device_queries(w.queries, dev)
        res, stats = st.deps_batch_device(qdev)
        torch.cuda.synchronize(dev)
        idx = _sample(len(w.queries))
        got = st.device_result_to_host(res, idx)
        _check_csr(st, res)
        # the same invariants checked on the device (ad_check_result_device / ad_check_snapshot)
        assert st.check_result_device(res) == (0, None)
        assert st.check_snapshot() == (0, None)
        exp = oracle.OracleStore(w.range_start_inclusive, 1, w.slices).load(w).deps_batch(w.queries.take(idx), w.flags)
        ok, why = got.equals(exp, detail=True)
        if not ok:
            mm = got.first_mismatch(exp)
            raise AssertionError("%s: %s; first mismatch at sample %s (request %d): %r" %
                                 (w.name, why, mm[0] if mm else None, idx[mm[0]] if mm else -1, mm))
        # the packed arrays read back in full, then the same batch through its regions (AD_REGIONS, the
        # bench's default output): every request's three maps identical to the packed ones
        full = st.device_result_to_host(res)
        rres, rstats = st.deps_batch_device(qdev, regions=True)
        torch.cuda.synchronize(dev)
        assert not rres.keys[0] and rres.regions_bytes >= rres.region_bytes > 0
        assert rstats["n_pairs"] == stats["n_pairs"]
        viar = st.device_result_to_host(rres)
        ok, why = viar.equals(full, detail=True)
        assert ok, "%s: regions differ from the packed arrays: %s" % (w.name, why)
        return stats, got
    finally:
        st.close()


@pytest.fixture(scope="module")
def config2_full():
    return synth.config2()


def test_config2_full_headline_batch(oracle, config2_full):
    # the bench.py headline batch: 1M requests x 8 Zipf keys over a 16M-entry history (hottest key
    # ~1.04M entries)
    stats, got = _run_full(config2_full, oracle)
    assert stats["n_probes"] == 8_000_000
    assert sum(stats["n_pairs"]) > 20_000_000


def test_config2_full_request_mix(oracle, config2_full):
    # the same batch as 60 % fresh PreAccepts, 30 % Accepts of in-flight txns (S = executeAt,
    # self excluded), 10 % PreAccepts up to 2000 hlc ticks late (older than busy keys' newest
    # entries: the general kernel's tree descent over the hot segments)
    w = synth.with_request_mix(config2_full, accept_frac=0.3, unordered_frac=0.1, unordered_window=2000)
    stats, got = _run_full(w, oracle)
    assert w.params["n_accept"] > 200_000 and w.params["n_unordered"] > 50_000
    assert stats["n_deferred_lean"] > 0          # the general kernel ran on the late requests


def test_config4_full(oracle):
    w = synth.config4()
    stats, got = _run_full(w, oracle)
    assert stats["n_pairs"][A.AD_MAP_RANGE] > 0 and got.pair_count(A.AD_MAP_RANGE) > 0
    # the ~9 % of requests with 17..32 range emissions take lean pass 1's wide range round, not pass 2
    assert stats["n_lean_pass2"] < 10_000      # 95k before; what is left has more than 16 key emissions


def test_config4_dense_ranges_every_request(oracle):
    # config 4's range density (100k range commands, ~12 stabbing entries per 4-key request) over 4k requests,
    # every request checked: the wide range round (17..32 range emissions, two per lane) and the narrow one
    w = synth.config4(n_txns=4_000, n_hist_txns=20_000, seed=0xACC0D0B4)
    exp = oracle.resolve(w)
    got = native.resolve(w, via="regions")
    ok, why = got.equals(exp, detail=True)
    assert ok, "%s; first mismatch %r" % (why, got.first_mismatch(exp))


def test_config2_full_narrow_pass1(oracle, config2_full, monkeypatch):
    # lean pass 1's narrow kernel forced (AD_LEAN_WIDE1=0: <= 32 raw emissions per request, the requests
    # of 33..64 through lean pass 2) -- the same result as the wide kernel of the headline test
    monkeypatch.setenv("AD_LEAN_WIDE1", "0")
    stats, got = _run_full(config2_full, oracle)
    assert not stats["lean_wide1"] and stats["n_lean_pass2"] > 50_000


def test_lean_pass1_width_follows_the_batches(oracle, config2_full, monkeypatch):
    # abi.cpp lean_wide1: a store's first batch runs wide; config 2 (Zipf keys, ~13 % of requests above
    # 32 raw emissions) stays wide, config 3's store (uniform keys, almost none) turns narrow -- and the
    # narrow batch's result equals the wide one's
    import torch
    monkeypatch.delenv("AD_LEAN_WIDE1", raising=False)
    dev = torch.device("cuda", 0)
    w3 = synth.config3_shard(0, 1, txns_per_gpu=1_000_000, keys_per_gpu=160_000)[0]
    for w, second_wide in ((config2_full, True), (w3, False)):
        # the width choice is lean pass 1's at two requests per wave; config 3's 4-key requests would run four per
        # wave (abi.cpp lean_rpw1), so its store is held at two
        if w is w3:
            monkeypatch.setenv("AD_LEAN_RPW", "2")
        st = native.DeviceCommandStore(device=0, slices=w.slices)
        try:
            st.load(w)
            qdev, keep = native.device_queries(w.queries, dev)
            res1, s1 = st.deps_batch_device(qdev)
            torch.cuda.synchronize(dev)
            a = st.device_result_to_host(res1)
            res2, s2 = st.deps_batch_device(qdev)
            torch.cuda.synchronize(dev)
            assert s1["lean_wide1"] and s2["lean_wide1"] == second_wide, w.name
            ok, why = st.device_result_to_host(res2).equals(a, detail=True)
            assert ok, "%s: second batch differs: %s" % (w.name, why)
        finally:
            st.close()
