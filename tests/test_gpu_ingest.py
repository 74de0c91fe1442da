"""GPU parity of the device-side snapshot ingest (csrc/ingest.hip + the derivation of
cfk_update.hip): a store built on the device from the loaded columns (the default) against the same
store built by the host ingest (AD_INGEST_HOST), and both against the CPU restatement.

Compared: the id dictionary (ad_dict), every CommandsForKey as the store holds it (ad_cfk_byid,
ad_cfk_entries), the device invariants (ad_check_snapshot), and the PartialDeps of a batch over it
(bit-exact vs the oracle). Every load-time rejection the host ingest makes (CommandsForKey.java:1438,
:1439, Timestamp identity, status range, key-domain ids, key order, prunedBefore) is made by the
device route with the same code."""
import copy
import os
import sys

import numpy as np
import pytest

from accord_deps import _abi as A
from accord_deps import native, synth

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import cfk_update as U  # noqa: E402
import cfk_update_gen as G  # noqa: E402

pytestmark = pytest.mark.gpu


def _store(w, host, monkeypatch):
    if host:
        monkeypatch.setenv("AD_INGEST_HOST", "1")
    else:
        monkeypatch.delenv("AD_INGEST_HOST", raising=False)
    st = native.DeviceCommandStore(device=0, range_start_inclusive=w.range_start_inclusive, slices=w.slices)
    st.load(w)
    monkeypatch.delenv("AD_INGEST_HOST", raising=False)
    return st


def _same_tids(a, b):
    return np.array_equal(a.msb, b.msb) and np.array_equal(a.lsb, b.lsb) and np.array_equal(a.node, b.node)


def _compare_routes(w, oracle, monkeypatch):
    dev = _store(w, False, monkeypatch)
    host = _store(w, True, monkeypatch)
    try:
        assert dev.check_snapshot() == (0, None)
        assert _same_tids(dev.dictionary(), host.dictionary()), "dictionaries differ"
        kd, sd, td, pd = dev.cfk_byid()
        kh, sh, th, ph = host.cfk_byid()
        assert np.array_equal(kd, kh) and np.array_equal(sd, sh) and np.array_equal(pd, ph)
        assert _same_tids(td, th), "byId ids differ"
        std_, xd = dev.cfk_entries()
        sth, xh = host.cfk_entries()
        assert np.array_equal(std_, sth) and _same_tids(xd, xh), "entries differ"
        exp = oracle.resolve(w)
        got = dev.calculate_partial_deps(w.queries, w.flags)
        ok, why = got.equals(exp, detail=True)
        assert ok, "%s: %s; first mismatch %r" % (w.name, why, got.first_mismatch(exp))
    finally:
        dev.close()
        host.close()


@pytest.mark.parametrize("seed", range(12))
def test_random_stores(oracle, seed, monkeypatch):
    # every status, kind, prunedBefore, Accept-style executeAts, range commands, RedundantBefore, slices
    w = synth.random_small(900 + seed, with_slices=(seed % 4 == 3), start_inclusive=(seed % 5 == 4),
                           n_range_cmds=(0 if seed % 3 == 0 else 20), n_redundant=(0 if seed % 2 else 3))
    _compare_routes(w, oracle, monkeypatch)


def test_config2_scaled(oracle, monkeypatch):
    _compare_routes(synth.config2(n_txns=20_000, n_keys=20_000, n_hist_entries=300_000), oracle, monkeypatch)


def test_config4_scaled(oracle, monkeypatch):
    _compare_routes(synth.config4(n_txns=3000, n_keys=20000, n_ranges=5000, n_hist_txns=20000), oracle, monkeypatch)


@pytest.mark.parametrize("seed", range(3))
def test_device_ingest_then_updates(oracle, seed, monkeypatch):
    # a device-built store takes device updates (insertions with older ids: dictionary merges) and its
    # host views (entries, byId) follow; deps bit-exact vs the oracle over the updated CommandsForKey
    w = synth.random_small(77 + seed)
    w.flags = A.AD_SNAPSHOT
    rng = np.random.default_rng(seed)
    st = _store(w, False, monkeypatch)
    try:
        u1, _ = G.transitions(w.cfk, rng, 80)
        u2 = G.older_inserts(w.cfk, rng, 40, w=w)
        u = G.concat(u1, u2)
        new, _ = U.cfk_update(w.cfk, u)
        st.cfk_update(u)
        s, x = st.cfk_entries()
        assert s.tolist() == new.status.tolist() and _same_tids(x, new.exec)
        keys, seg, txn, _ = st.cfk_byid()
        assert np.array_equal(seg, new.seg) and _same_tids(txn, new.txn)
        old = w.cfk
        w.cfk = new
        try:
            exp = oracle.resolve(w)
            got = st.calculate_partial_deps(w.queries, w.flags)
            ok, why = got.equals(exp, detail=True)
            assert ok, why
        finally:
            w.cfk = old
    finally:
        st.close()


def _mutated(w, f):
    w2 = copy.deepcopy(w)
    f(w2.cfk)
    return w2


def _segments(cfk, min_len=2):
    seg = cfk.seg.astype(np.int64)
    return [k for k in range(len(cfk.keys)) if seg[k + 1] - seg[k] >= min_len]


def _swap_ids(cfk):
    k = _segments(cfk)[0]
    e = int(cfk.seg[k])
    for a in (cfk.txn, cfk.exec):
        for arr in (a.msb, a.lsb, a.node):
            arr[e], arr[e + 1] = arr[e + 1].copy(), arr[e].copy()


def _dup_exec(cfk):
    # two committed entries of one key executing at one timestamp
    com = (cfk.status >= A.ST_COMMITTED) & (cfk.status <= A.ST_APPLIED)
    seg = cfk.seg.astype(np.int64)
    for k in range(len(cfk.keys)):
        idx = np.nonzero(com[seg[k]:seg[k + 1]])[0] + seg[k]
        if len(idx) >= 2:
            a, b = int(idx[0]), int(idx[1])
            cfk.exec.msb[b], cfk.exec.lsb[b], cfk.exec.node[b] = cfk.exec.msb[a], cfk.exec.lsb[a], cfk.exec.node[a]
            return
    raise AssertionError("no key with two committed entries")


def _flag_bits(cfk):
    # an executeAt equal (Timestamp.equals) to another entry's txnId but with a non-identity flag bit
    # set: the library's id identity is the bits (AD_E_INCONSISTENT_ID)
    e = int(np.nonzero(cfk.status == A.ST_APPLIED)[0][-1])
    cfk.exec.msb[e], cfk.exec.lsb[e], cfk.exec.node[e] = cfk.txn.msb[0], cfk.txn.lsb[0] | np.uint64(0x20), cfk.txn.node[0]


def _bad_status(cfk):
    cfk.status[len(cfk.status) // 2] = 9


def _keys_order(cfk):
    cfk.keys[1], cfk.keys[2] = cfk.keys[2], cfk.keys[1]


def _pruned_outside(cfk):
    k = _segments(cfk, 1)[0]
    cfk.pruned_before[k] = int(cfk.seg[k + 1] - cfk.seg[k]) + 3


def _range_domain(cfk):
    # Routable.Domain.Range on a live CommandsForKey entry: the txn's id in every CommandsForKey that
    # holds it (and where it is its own executeAt), so that the bits stay one id's
    e = int(np.nonzero(cfk.status == A.ST_APPLIED)[0][0])
    m, l, n = cfk.txn.msb[e], cfk.txn.lsb[e], cfk.txn.node[e]
    for t in (cfk.txn, cfk.exec):
        hit = (t.msb == m) & (t.lsb == l) & (t.node == n)
        t.lsb[hit] |= np.uint64(1)


@pytest.mark.parametrize("mut,code", [(_swap_ids, A.AD_E_ORDER), (_dup_exec, A.AD_E_DUP_EXEC),
                                      (_flag_bits, A.AD_E_INCONSISTENT_ID), (_bad_status, A.AD_E_INVAL),
                                      (_keys_order, A.AD_E_INVAL), (_pruned_outside, A.AD_E_INVAL),
                                      (_range_domain, A.AD_E_INVAL)])
def test_load_rejections(mut, code, monkeypatch):
    w = synth.random_small(31, n_range_cmds=0, n_redundant=0, n_hist_txns=400)
    if w.cfk.pruned_before is None:
        w.cfk.pruned_before = np.full(len(w.cfk.keys), -1, np.int64)
    bad = _mutated(w, mut)
    for host in (False, True):
        with pytest.raises(native.AccordDepsError) as e:
            _store(bad, host, monkeypatch)
        assert e.value.code == code, "%s route: %s" % ("host" if host else "device", e.value)
