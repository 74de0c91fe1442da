"""Recovery scans: the oracle's CommandsForKey.mapReduceFull restatement
(rc_recovery_batch, oracle/refcpu.c) against an independent flat model of the four BeginRecovery
scans (refmodel.recovery_pairs; BeginRecovery.java:329-380, CommandsForKey.java:809-908), plus the
host-side checks of the C ABI's recovery entry points. CPU only."""
import numpy as np
import pytest

from accord_deps import _abi as A, native, synth
from accord_deps.model import Queries, Tids, make_txn_ids

import refmodel
from test_oracle import _request


@pytest.mark.parametrize("ranges", [False, True])
@pytest.mark.parametrize("seed", range(8))
@pytest.mark.parametrize("scan", A.RECOVER_SCANS)
def test_recovery_crosscheck(oracle, seed, scan, ranges):
    w = synth.recovery_workload(seed, with_slices=(seed % 3 == 2), start_inclusive=(seed % 4 == 1),
                                n_range_cmds=16 if ranges else 0)
    batch = oracle.recover(w, scan)
    hits = rhits = 0
    for i in range(len(w.queries)):
        kd, dd = refmodel.recovery_pairs(w, i, scan)
        rd = refmodel.recovery_range_pairs(w, i, scan)
        got = _request(batch, i)
        for m, pairs in ((0, kd), (1, rd), (2, dd)):
            assert got[m] == tuple(refmodel.csr(pairs)), (seed, scan, i, A.MAP_NAMES[m])
        hits += len(kd) + len(dd)
        rhits += len(rd)
    assert seed % 4 or hits > 0 or scan in (0, 2)          # the workloads reach the emitting branches



@pytest.mark.parametrize("seed", range(10))
@pytest.mark.parametrize("scan", A.RECOVER_SCANS)
def test_range_domain_recovery_crosscheck(oracle, seed, scan):
    # recovering Range-domain txns (sync points, range reads/writes: BeginRecovery hands their Ranges to
    # mapReduceFull, BeginRecovery.java:334,348,365,378): every CommandsForKey inside the sliced ranges
    # (InMemoryCommandStore.java:289-304) and the range commands intersecting them (:884-958)
    w = synth.recovery_workload(seed, with_slices=(seed % 3 == 2), start_inclusive=(seed % 4 == 1),
                                n_range_cmds=(0 if seed % 5 == 4 else 16), range_frac=0.6, n_txns=70)
    q = w.queries
    assert q.n_ranges > 0
    batch = oracle.recover(w, scan)
    for i in range(len(q)):
        kd, dd = refmodel.recovery_pairs(w, i, scan)
        rd = refmodel.recovery_range_pairs(w, i, scan)
        got = _request(batch, i)
        for m, pairs in ((0, kd), (1, rd), (2, dd)):
            assert got[m] == tuple(refmodel.csr(pairs)), (seed, scan, i, A.MAP_NAMES[m], q.ranges_of(i))


def test_range_domain_recovery_reaches_every_scan(oracle):
    # over a few seeds the Range-domain requests emit keyDeps and rangeDeps in every scan
    tot = {s: [0, 0] for s in A.RECOVER_SCANS}
    for seed in range(8):
        w = synth.recovery_workload(seed, n_range_cmds=16, range_frac=0.6, n_txns=70, n_hist_txns=200)
        q = w.queries
        isr = [i for i in range(len(q)) if q.ranges_of(i)]
        for s in A.RECOVER_SCANS:
            b = oracle.recover(w, s)
            for i in isr:
                got = _request(b, i)
                tot[s][0] += len(got[0][1]) + len(got[2][1])
                tot[s][1] += len(got[1][1])
    # scan 1 (WITH) finds no key entries: a Range-domain txnId is never in a CommandsForKey's byId, and an
    # unknown testTxnId has no witnesses there (CommandsForKey.java:826-836, hasAsDep false)
    assert all(v[1] > 0 and (v[0] > 0) == (s != 1) for s, v in tot.items()), tot


def test_recovery_ranges_reach_every_scan(oracle):
    # the range-command half emits in every scan over a few seeds
    tot = {s: 0 for s in A.RECOVER_SCANS}
    for seed in range(8):
        w = synth.recovery_workload(seed, n_range_cmds=16)
        for s in A.RECOVER_SCANS:
            b = oracle.recover(w, s)
            tot[s] += b.pair_count(1)
    assert all(v > 0 for v in tot.values()), tot


def test_recovery_branches_covered(oracle):
    # over a few seeds every scan emits, and WITH/WITHOUT both see known and unknown txnIds
    tot = {s: 0 for s in A.RECOVER_SCANS}
    for seed in range(6):
        w = synth.recovery_workload(seed, n_hist_txns=200, accept_frac=0.5)
        for s in A.RECOVER_SCANS:
            tot[s] += sum(oracle.recover(w, s).pair_count(m) for m in range(3))
    assert all(v > 0 for v in tot.values()), tot


def test_missing_list_decides_witness(oracle):
    # one key: T (Write) known; E (Write, STABLE, executeAt > T) with and without T in missing()
    T = make_txn_ids(1, np.array([100], np.uint64), A.KIND_WRITE, np.array([1]))
    E = make_txn_ids(1, np.array([50], np.uint64), A.KIND_WRITE, np.array([2]))
    Ex = make_txn_ids(1, np.array([200], np.uint64), A.KIND_WRITE, np.array([1 << 24]))
    from accord_deps.model import CfkSnapshot, RangeCommands, Redundant, Workload
    txn = Tids.concat([E, T])
    ex = Tids.concat([Ex, T])
    q = Queries(T, T, np.array([0, 1], np.uint64), np.array([7], np.int64))
    for with_t, exp1, exp3 in ((False, 1, 0), (True, 0, 1)):
        miss = T if with_t else T.take(np.zeros(0, np.int64))
        cfk = CfkSnapshot(np.array([7]), np.array([0, 2], np.uint64), txn, ex,
                          np.array([A.ST_STABLE, A.ST_PREACCEPTED], np.uint8), None,
                          np.array([0, len(miss), len(miss)], np.uint64), miss)
        w = Workload("kat", cfk, RangeCommands.empty(), Redundant.empty(), q)
        # scan 1 (STARTED_BEFORE, WITH, IS_STABLE): E witnessed T unless T is missing
        assert oracle.recover(w, 1).pair_count(0) == exp1
        # scan 3 (ANY, WITHOUT, IS_STABLE): E executes after T without witnessing it
        assert oracle.recover(w, 3).pair_count(0) == exp3


def test_recovery_rejects_range_commands(oracle):
    w = synth.random_small(3)                            # has live range commands
    with pytest.raises(oracle.OracleError) as e:
        oracle.recover(w, 0)
    assert e.value.code == A.AD_E_STATE


def test_abi_exports_recovery():
    L = native.lib()
    for sym in ("ad_cfk_missing_load", "ad_recovery_batch", "ad_recovery_batch_device"):
        assert sym in native.EXPORTS
        getattr(L, sym)
