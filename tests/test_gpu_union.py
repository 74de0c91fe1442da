"""GPU parity of the coordinator-side Deps.merge (ad_parts_union): replicas whose
key sets overlap (overlapping token slices) and whose answers differ (elision on / off) each
resolve the batch and export rank-format parts; the union on the GPU is compared bit-exactly with
the oracle's request-wise PartialDeps.with over the replicas' results (rc_result_merge, which
restates RelationMultiMap.linearUnion and handles repeated keys)."""
import numpy as np
import pytest
import torch

import pyoracle
from accord_deps import _abi as A
from accord_deps import exchange, native, synth

pytestmark = pytest.mark.gpu


def _union(w, bounds, elides, order=None):
    dev = torch.device("cuda", 0)
    n = len(w.queries)
    reps = []
    for (lo, hi), e in zip(bounds, elides):
        ws = synth.slice_workload(w, lo, hi)
        st = native.DeviceCommandStore(0, w.range_start_inclusive, e, ws.slices)
        st.load(ws)
        qdev, keep = native.device_queries(ws.queries, dev)
        reps.append((ws, e, exchange.GpuEngine(st, qdev, np.arange(n), dev), keep))
    g = exchange.build_global_dict([r[2].dictionary() for r in reps])
    for r in reps:
        r[2].set_global_dict(g)
    sends = []
    for ws, e, eng, keep in reps:
        eng.resolve()
        sends.append(eng.export(np.array([0, n], np.uint64)))
    torch.cuda.synchronize()
    order = order or list(range(len(reps)))
    recv, totals = {}, np.zeros(4, np.int64)
    for a, (name, mult) in enumerate((("hdr", 4), ("keys", 1), ("ids", 1), ("k2t", 1))):
        recv[name] = torch.cat([sends[i][0][name][:int(sends[i][1][0, a]) * mult] for i in order])
    for i in order:
        totals += sends[i][1][0]
    p = A.AdParts()
    p.hdr, p.keys, p.ids, p.k2t = (recv[k].data_ptr() for k in ("hdr", "keys", "ids", "k2t"))
    p.n_parts, p.n_key_words, p.n_ids, p.n_k2t = (int(x) for x in totals)
    p.id_format = A.AD_IDS_RANK
    owner = reps[0][2].store
    mg = owner.union_parts(p, [int(sends[i][1][0, 0]) for i in order], 0, n)
    got = owner.merged_to_host(mg)
    expect = pyoracle.merge_batches([pyoracle.resolve(ws, elide=e) for ws, e, _, _ in reps])
    for r in reps:
        r[2].store.close()
    return got, expect, mg


def _check(w, bounds, elides, order=None):
    got, expect, mg = _union(w, bounds, elides, order)
    ok, why = got.equals(expect, detail=True)
    assert ok, "%s; first mismatch %s" % (why, got.first_mismatch(expect))
    return mg


def _overlap(cuts):
    lo, hi = synth.cut_bounds(cuts)
    return list(zip(lo, hi))


@pytest.mark.parametrize("seed", range(10))
def test_random_small_overlapping_replicas(seed):
    w = synth.random_small(400 + seed)
    w.slices = None
    b = [(-(1 << 63), 150), (-200, (1 << 63) - 1), (-(1 << 63), (1 << 63) - 1)]
    _check(w, b, [1, 0, 1 - seed % 2], order=[2, 0, 1] if seed % 3 == 0 else None)


@pytest.mark.parametrize("n_rep", [2, 3, 5])
def test_config3_replicas(n_rep):
    w = synth.config3(n_txns=20000, n_keys=3000, seed=70 + n_rep)
    full = (-(1 << 63), (1 << 63) - 1)
    _check(w, [full] * n_rep, [i % 2 for i in range(n_rep)])


def test_config4_ranges_replicas():
    w = synth.config4(n_txns=2000, n_keys=3000, n_ranges=600, n_hist_txns=2000)
    _check(w, [(-(1 << 63), 1 << 30), (-(1 << 30), (1 << 63) - 1)], [1, 0])


def test_big_groups():
    # hot keys with hundreds of live entries: groups far beyond one wave
    w = synth.config2(n_txns=200, n_keys=40, n_hist_entries=40000, keys_per_txn=8, tail_unapplied=300)
    full = (-(1 << 63), (1 << 63) - 1)
    _check(w, [full, full, (-(1 << 62), 1 << 62)], [1, 0, 1])


def test_union_requires_rank_parts():
    dev = torch.device("cuda", 0)
    w = synth.config3(n_txns=2000, n_keys=300, seed=5)
    st = native.DeviceCommandStore(0)
    st.load(w)
    qdev, keep = native.device_queries(w.queries, dev)
    e = exchange.GpuEngine(st, qdev, np.arange(len(w.queries)), dev, parts_only=False)
    e.resolve()
    send, counts = e.export(np.array([0, len(w.queries)], np.uint64))
    torch.cuda.synchronize()
    p = A.AdParts()
    p.hdr, p.keys, p.ids, p.k2t = (send[k].data_ptr() for k in ("hdr", "keys", "ids", "k2t"))
    p.n_parts, p.n_key_words, p.n_ids, p.n_k2t = (int(x) for x in counts[0])
    with pytest.raises(native.AccordDepsError) as ei:
        st.union_parts(p, [int(counts[0, 0])], 0, len(w.queries))
    assert ei.value.code == A.AD_E_INVAL
    st.close()
