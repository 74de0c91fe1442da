"""CPU tests of bench.py's host-side legs: the multi-store CPU baseline (one refcpu CommandStore per
EvenSplit token slice on its own thread, reduced with PartialDeps.with) must reproduce the
single-store result exactly, and the request-mix generator must keep the workload's invariants."""
import numpy as np

import bench
from accord_deps import _abi as A
from accord_deps import synth


def test_cpu_baseline_stores_equals_single_store(oracle):
    w = synth.config2(n_txns=1500, n_keys=20000, n_hist_entries=150_000)
    exp = oracle.resolve(w)
    out = bench.cpu_baseline_stores(w, budget_s=1.0, threads=4, gpu_take=lambda idx: exp.take(idx))
    assert out["parity_sample"].endswith("bit-exact vs GPU"), out
    assert out["cores"] == 4 and out["value"] > 0


def test_request_mix_invariants(oracle):
    w = synth.config2(n_txns=3000, n_keys=20000, n_hist_entries=200_000)
    m = synth.with_request_mix(w, accept_frac=0.3, unordered_frac=0.2, unordered_window=300)
    assert m.params["n_accept"] > 500 and m.params["n_unordered"] > 300
    c = m.cfk
    seg = c.seg.astype(np.int64)
    # byId strictly ascending per key; committed executeAts unique per key (CommandsForKey.java:1438-1439)
    for k in np.random.default_rng(1).choice(len(c.keys), 300, replace=False):
        t = c.txn.take(slice(seg[k], seg[k + 1]))
        o = np.lexsort(t.order_key())
        assert np.all(o == np.arange(len(o)))
    q = m.queries
    # Accepts: executeAt above every id of the store; their txnId is in each of their keys' byId
    acc = np.nonzero((q.exec.msb != q.txn.msb) | (q.exec.lsb != q.txn.lsb) | (q.exec.node != q.txn.node))[0]
    assert len(acc) == m.params["n_accept"]
    r = oracle.resolve(m)
    # the accepted txn never depends on itself (PreAccept.java:261)
    for i in acc[:200]:
        ks, ke, t, k2t = r.maps[A.AD_MAP_KEY].request(i)
        me = (q.txn.msb[i], q.txn.lsb[i], q.txn.node[i])
        assert me not in t.tuples()
    # the reference model agrees on a sample
    import refmodel
    for i in list(acc[:20]) + list(range(20)):
        kd, rd, dd = refmodel.request_pairs(m, int(i))
        ks, ke, t, k2t = r.maps[A.AD_MAP_KEY].request(int(i))
        keys, vals, k2 = refmodel.csr(kd)
        assert ([int(x) for x in ks], t.tuples(), [int(x) for x in k2t]) == (keys, vals, k2)


def test_resolve_kernels_follow_the_library_stats():
    """bench.py names the roofline's kernels from what the library reports it launched (ad_stats.lean_rpw1 /
    lean_flags), never from the workload's shape (a 4-key batch was labelled with the 2-request
    kernels)."""
    split = [0.5, 0.0, 0.07, 0.1, 0.0, 0.03, 0.2]
    st = dict(lean_rpw1=4, lean_flags=A.AD_LEAN_RANGES | A.AD_LEAN_PASS2)
    assert bench.resolve_kernels(st, split) == ["k_prepare<true>", "k_resolve_lean<4u, true, false, 1>",
                                                "k_resolve_lean<2u, true, false, 2>", "k_resolve"]
    st = dict(lean_rpw1=2, lean_flags=A.AD_LEAN_WIDE1)
    assert bench.resolve_kernels(st, split) == ["k_prepare<true>", "k_resolve_lean<2u, false, true, 1>", "k_resolve"]
    st = dict(lean_rpw1=4, lean_flags=A.AD_LEAN_PASS2)
    assert bench.resolve_kernels(st, [0.5, 0, 0.07, 0.01, 0, 0.03, 0.0]) == ["k_prepare<true>",
                                                                              "k_resolve_lean<4u, false, false, 1>"]
    # no lean pass (a store with RedundantBefore entries): the general kernel alone
    assert bench.resolve_kernels(dict(lean_rpw1=0, lean_flags=0), [0.9, 0, 0.07, 0, 0, 0.03, 0]) == \
        ["k_prepare<false>", "k_resolve"]


def test_measured_traffic_never_falls_back_to_an_older_round():
    t, src = bench.measured_traffic(["k_no_such_kernel<1>"], "config2")
    assert t is None and src.startswith("missing")
