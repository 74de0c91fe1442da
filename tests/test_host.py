"""CPU tests: the C ABI library loads and exports every declared entry point, fails loudly without
a GPU, and the host-side data model / synthetic workloads honour the reference's invariants."""
import os
import re

import numpy as np
import pytest

from accord_deps import _abi as A
from accord_deps import native, synth
from accord_deps.model import Tids  # noqa: F401

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    hdr = open(os.path.join(ROOT, "include", "accord_deps.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    return sorted(set(re.findall(r"\b(ad_[a-z_]+)\s*\(", hdr)))


def test_header_and_library_exports():
    names = _declared()
    assert "ad_deps_batch" in names and "ad_cfk_load" in names
    L = native.lib()
    for n in names:
        assert hasattr(L, n), n
    assert set(names) == set(native.EXPORTS)
    assert L.ad_abi_version() == 6


def test_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    with pytest.raises(native.AccordDepsError) as e:
        native.DeviceCommandStore()
    assert e.value.code == A.AD_E_DEVICE


def test_struct_layouts_match_header():
    import ctypes as C
    # offsets the C side relies on (x86-64 SysV)
    assert C.sizeof(A.AdConfig) == 40
    assert A.AdQuerySoa.keys.offset == 8 * 9
    # n_txns, 6 x 3 pointers, stats, then regions, 3 region_off pointers, regions_bytes, region_bytes
    assert C.sizeof(A.AdDepsResult) == 8 + 6 * 3 * 8 + C.sizeof(A.AdStats) + 8 + 3 * 8 + 8 + 8
    assert A.AdDepsResult.regions.offset == 8 + 6 * 3 * 8 + C.sizeof(A.AdStats)


def _check_cfk_invariants(cfk):
    seg = cfk.seg.astype(np.int64)
    assert np.all(cfk.keys[1:] > cfk.keys[:-1]), "keys strictly ascending"
    assert seg[0] == 0 and seg[-1] == cfk.n_entries and np.all(np.diff(seg) >= 0)
    key_of = np.repeat(np.arange(len(cfk.keys)), np.diff(seg))
    tk = np.lexsort((cfk.txn.node.astype(np.int64), cfk.txn.lsb & np.uint64(0x1E), cfk.txn.lsb >> np.uint64(16),
                     cfk.txn.msb, key_of))
    assert np.array_equal(tk, np.arange(cfk.n_entries)), "byId sorted (CommandsForKey.java:1438)"
    committed = (cfk.status >= A.ST_COMMITTED) & (cfk.status <= A.ST_APPLIED)
    ex = cfk.exec.take(np.nonzero(committed)[0])
    keyc = key_of[committed]
    rows = set(zip(keyc.tolist(), ex.msb.tolist(), ex.lsb.tolist(), ex.node.tolist()))
    assert len(rows) == int(committed.sum()), "committed executeAt unique per key (:1439)"
    # an executeAt that differs from its txnId never equals another txnId: executeAt node ids are
    # disjoint from txnId node ids (CommandsForKeyTest.java:418-424,449-455 arranges the same)
    diff = ~((cfk.exec.msb == cfk.txn.msb) & (cfk.exec.lsb == cfk.txn.lsb) & (cfk.exec.node == cfk.txn.node))
    assert np.all(cfk.exec.node[diff] >= synth.EXEC_NODE_BASE)
    assert np.all(cfk.txn.node < synth.EXEC_NODE_BASE)


@pytest.mark.parametrize("gen", ["config2", "config3", "config4"])
def test_synthetic_configs_honour_invariants(gen):
    if gen == "config2":
        w = synth.config2(n_txns=2000, n_keys=20000, n_hist_entries=80000)
    elif gen == "config3":
        w = synth.config3(n_txns=40000, n_keys=5000)
    else:
        w = synth.config4(n_txns=2000, n_keys=5000, n_ranges=1000, n_hist_txns=5000)
    _check_cfk_invariants(w.cfk)
    q = w.queries
    for i in range(0, len(q), max(1, len(q) // 50)):
        ks = q.keys[int(q.key_off[i]):int(q.key_off[i + 1])]
        assert np.all(ks[1:] > ks[:-1])
    # every request is newer than every CommandsForKey txnId (SNAPSHOT of an older history)
    order_last = max(w.cfk.txn.tuples(), key=lambda t: (t[0], t[1] >> 16, t[1] & 0x1E, t[2]))
    first_q = min(q.txn.tuples(), key=lambda t: (t[0], t[1] >> 16, t[1] & 0x1E, t[2]))
    assert (first_q[0], first_q[1] >> 16) > (order_last[0], order_last[1] >> 16)


def test_config5_graph_is_consistent():
    g, p = synth.config5(n_txns=5000, n_keys=500)
    assert len(g.kind) == 5000
    ex = list(zip(g.exec.msb.tolist(), (g.exec.lsb >> np.uint64(16)).tolist(), g.exec.node.tolist()))
    assert len(set(ex)) == len(ex)
    assert g.dep_off[-1] == len(g.deps)


def test_random_small_invariants():
    for seed in range(20):
        w = synth.random_small(seed)
        _check_cfk_invariants(w.cfk)
        pb = w.cfk.pruned_before
        for i in np.nonzero(pb >= 0)[0]:
            e = int(w.cfk.seg[i]) + int(pb[i])
            assert w.cfk.status[e] == A.ST_APPLIED and w.cfk.txn.kind()[e] == A.KIND_WRITE


def test_slice_workload_partitions_keys():
    w = synth.config3(n_txns=20000, n_keys=3000)
    lo, hi = synth.shard_bounds(4)
    total_keys = 0
    total_probes = 0
    for g in range(4):
        s = synth.slice_workload(w, lo[g], hi[g])
        assert np.all((s.cfk.keys > lo[g]) & (s.cfk.keys <= hi[g]))
        assert np.all((s.queries.keys > lo[g]) & (s.queries.keys <= hi[g]))
        assert len(s.queries) == len(w.queries)
        total_keys += len(s.cfk.keys)
        total_probes += s.queries.n_probes
        _check_cfk_invariants(s.cfk)
    assert total_keys == len(w.cfk.keys)
    assert total_probes == w.queries.n_probes


def test_timestamp_packing_matches_reference_layout():
    # Timestamp(epoch, hlc, flags, node): msb = epoch<<15 | hlc>>>48, lsb = hlc<<16 | flags (Timestamp.java:81-89)
    from accord_deps.model import make_timestamps, make_txn_ids
    t = make_timestamps([3], [(1 << 50) + 5], [0x13], [7])
    assert int(t.msb[0]) == (3 << 15) | 4 and int(t.lsb[0]) == ((5 << 16) | 0x13)
    x = make_txn_ids([1], [9], [A.KIND_EXCLUSIVE_SYNC_POINT], [2], domain=1)
    assert int(x.kind()[0]) == A.KIND_EXCLUSIVE_SYNC_POINT and int(x.domain()[0]) == 1
    assert isinstance(x, Tids)
