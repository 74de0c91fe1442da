"""Device invariant checks (SURVEY §5 debug aids; include/accord_deps.h ad_check_result_device /
ad_check_snapshot): valid device results and snapshots pass -- also after device-side
CommandsForKey updates -- and results broken in each way RelationMultiMap.checkValid
(RelationMultiMap.java:1074-1097) and the builder's layout (:147-260) forbid are flagged at the
right request and map."""
import ctypes as C

import numpy as np
import pytest

from accord_deps import _abi as A
from accord_deps import native, synth

pytestmark = pytest.mark.gpu


def _resolved(w):
    import torch
    st = native.DeviceCommandStore(device=0, slices=w.slices)
    st.load(w)
    qdev, keep = native.device_queries(w.queries, torch.device("cuda", 0))
    res, _ = st.deps_batch_device(qdev)
    torch.cuda.synchronize()
    return st, res, keep


def _host_arrays(st, res):
    n = res.n_txns
    out = []
    for m in range(A.NMAPS):
        ko = st._d2h(res.keys_off[m], n + 1, np.uint64)
        to = st._d2h(res.txn_off[m], n + 1, np.uint64)
        oo = st._d2h(res.k2t_off[m], n + 1, np.uint64)
        out.append([ko, st._d2h(res.keys[m], int(ko[-1]), np.int64), to, st._d2h(res.txns[m], int(to[-1]), np.uint32),
                    oo, st._d2h(res.k2t[m], int(oo[-1]), np.int32)])
    return out


def _device_result(arrs, n):
    """An AdDepsResult over torch copies of host arrays (each at least one element)."""
    import torch
    keep = []
    r = A.AdDepsResult()
    r.n_txns = n

    def dev(a):
        a = np.ascontiguousarray(a)
        if a.dtype == np.uint64:
            a = a.view(np.int64)
        elif a.dtype == np.uint32:
            a = a.view(np.int32)
        if len(a) == 0:
            a = np.zeros(1, a.dtype)
        t = torch.from_numpy(a.copy()).to("cuda:0")
        keep.append(t)
        return t.data_ptr()
    for m in range(A.NMAPS):
        ko, keys, to, tx, oo, k2t = arrs[m]
        r.keys_off[m], r.keys[m] = dev(ko), dev(keys)
        r.txn_off[m], r.txns[m] = dev(to), dev(tx)
        r.k2t_off[m], r.k2t[m] = dev(oo), dev(k2t)
    return r, keep


def _first_nonempty(arrs, m, min_keys=2, min_ids=2):
    ko, _, to, _, oo, _ = arrs[m]
    nk, nt = np.diff(ko.astype(np.int64)), np.diff(to.astype(np.int64))
    cand = np.nonzero((nk >= min_keys) & (nt >= min_ids))[0]
    assert len(cand), "workload has no request with %d keys / %d ids in map %d" % (min_keys, min_ids, m)
    return int(cand[0])


@pytest.fixture(scope="module")
def resolved():
    w = synth.random_small(5, n_keys=48, n_hist_txns=600, n_txns=400, max_keys=6, n_range_cmds=40)
    st, res, keep = _resolved(w)
    arrs = _host_arrays(st, res)
    yield st, res, arrs
    st.close()


def test_valid_results_and_snapshots_pass():
    for w in (synth.random_small(3, n_keys=64, n_hist_txns=400, n_txns=300, max_keys=6, n_range_cmds=30),
              synth.config2(n_txns=4000, n_keys=20000, n_hist_entries=300000),
              synth.config4(n_txns=3000, n_keys=20000, n_ranges=5000, n_hist_txns=20000)):
        st, res, keep = _resolved(w)
        try:
            assert st.check_result_device(res) == (0, None), w.name
            assert st.check_snapshot() == (0, None), w.name
        finally:
            st.close()


def test_copied_result_passes(resolved):
    st, res, arrs = resolved
    r, keep = _device_result(arrs, res.n_txns)
    assert st.check_result_device(r) == (0, None)


@pytest.mark.parametrize("fault", ["key_order", "txn_order", "txn_range", "end_offset", "last_end", "dup_value",
                                   "value_range", "unused_txn", "offsets"])
def test_broken_results_are_flagged(resolved, fault):
    st, res, arrs = resolved
    a = [[x.copy() for x in mp] for mp in arrs]
    m = A.AD_MAP_KEY
    t = _first_nonempty(a, m)
    ko, keys, to, tx, oo, k2t = a[m]
    k0, x0, p0 = int(ko[t]), int(to[t]), int(oo[t])
    nk, nt = int(ko[t + 1]) - k0, int(to[t + 1]) - x0
    if fault == "key_order":
        keys[k0], keys[k0 + 1] = keys[k0 + 1], keys[k0]
    elif fault == "txn_order":
        tx[x0], tx[x0 + 1] = tx[x0 + 1], tx[x0]
    elif fault == "txn_range":
        tx[x0 + nt - 1] = 2 ** 31            # beyond the dictionary
    elif fault == "end_offset":
        k2t[p0] = nk                          # first key without a value
    elif fault == "last_end":
        k2t[p0 + nk - 1] -= 1
    elif fault == "dup_value":
        # a key holding two values gets its first one twice
        ends = k2t[p0:p0 + nk].astype(np.int64)
        starts = np.concatenate([[nk], ends[:-1]])
        j = int(np.nonzero(ends - starts >= 2)[0][0]) if np.any(ends - starts >= 2) else None
        if j is None:
            pytest.skip("no key with two values")
        k2t[p0 + starts[j] + 1] = k2t[p0 + starts[j]]
    elif fault == "value_range":
        k2t[p0 + nk] = nt
    elif fault == "unused_txn":
        # every reference to the request's last id goes to id 0 instead (sortedness kept for keys
        # whose values would collide is not needed: the check must flag it either way)
        body = k2t[p0 + nk:int(oo[t + 1])]
        body[body == nt - 1] = 0
    elif fault == "offsets":
        ko[t + 1], ko[t] = ko[t], ko[t + 1]
    r, keep = _device_result(a, res.n_txns)
    n_bad, first = st.check_result_device(r)
    assert n_bad >= 1 and first == 3 * t + m, (fault, n_bad, first, t)


def test_snapshot_after_device_updates():
    import torch
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import cfk_update_gen as G
    w = synth.config2(n_txns=2000, n_keys=5000, n_hist_entries=60000)
    st = native.DeviceCommandStore(device=0, slices=w.slices)
    try:
        st.load(w)
        rng = np.random.default_rng(3)
        u = G.concat(G.transitions(w.cfk, rng, 5000)[0], G.fresh_preaccepts(w.cfk, rng, 500),
                     G.older_inserts(w.cfk, rng, 500, w=w))
        st.cfk_update(u)
        assert st.check_snapshot() == (0, None)
        qdev, keep = native.device_queries(w.queries, torch.device("cuda", 0))
        res, _ = st.deps_batch_device(qdev)
        torch.cuda.synchronize()
        assert st.check_result_device(res) == (0, None)
    finally:
        st.close()
