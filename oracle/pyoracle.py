"""ctypes wrapper of the CPU restatement (oracle/librefcpu.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, as the checker -- never by the product path.
"""
import ctypes as C
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "cassandra-accord_amd"))

from accord_deps import _abi as A  # noqa: E402
from accord_deps.model import DepsMap, PartialDepsBatch, Tids  # noqa: E402

LIB_PATH = os.path.join(HERE, "librefcpu.so")


class RcResult(C.Structure):
    _fields_ = [("n_txns", C.c_uint64),
                ("keys_off", A.P * 3), ("keys", A.P * 3), ("keys_end", A.P * 3),
                ("txn_off", A.P * 3), ("txn_msb", A.P * 3), ("txn_lsb", A.P * 3), ("txn_node", A.P * 3),
                ("k2t_off", A.P * 3), ("k2t", A.P * 3), ("scan_entries", C.c_uint64)]


def build(target=None):
    """make in oracle/, serialised across processes (pytest-xdist workers build concurrently)."""
    import fcntl
    os.makedirs(os.path.join(HERE, "build"), exist_ok=True)
    with open(os.path.join(HERE, "build", ".lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        subprocess.check_call(["make", "-s", "-C", HERE] + ([target] if target else []))


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.rc_store_create.argtypes = [C.POINTER(A.AdConfig), C.POINTER(C.c_void_p)]
        L.rc_store_destroy.argtypes = [C.c_void_p]
        L.rc_last_error.argtypes = [C.c_void_p]
        L.rc_last_error.restype = C.c_char_p
        L.rc_cfk_load.argtypes = [C.c_void_p, C.POINTER(A.AdCfkSoa)]
        L.rc_range_cmds_load.argtypes = [C.c_void_p, C.POINTER(A.AdRangeCmdsSoa)]
        L.rc_redundant_load.argtypes = [C.c_void_p, C.POINTER(A.AdRedundantSoa)]
        L.rc_range_cmds_update.argtypes = [C.c_void_p, C.POINTER(A.AdRangeCmdsSoa)]
        L.rc_redundant_advance.argtypes = [C.c_void_p, C.POINTER(A.AdRedundantSoa)]
        L.rc_slice_sets_load.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p]
        L.rc_deps_batch.argtypes = [C.c_void_p, C.POINTER(A.AdQuerySoa), C.c_uint32, C.c_uint64, C.c_uint64,
                                    C.POINTER(C.POINTER(RcResult))]
        L.rc_result_free.argtypes = [C.POINTER(RcResult)]
        L.rc_result_merge.argtypes = [C.POINTER(C.POINTER(RcResult)), C.c_int, C.POINTER(C.POINTER(RcResult))]
        L.rc_levels.argtypes = [C.POINTER(A.AdGraphSoa), C.c_void_p]
        L.rc_preaccept.argtypes = [C.POINTER(A.AdRangeMapSoa), C.POINTER(A.AdRangeMapSoa), C.POINTER(A.AdQuerySoa),
                                   C.c_uint32, C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        L.rc_cfk_missing_load.argtypes = [C.c_void_p, C.POINTER(A.AdCfkMissingSoa)]
        L.rc_range_cmds_recovery_load.argtypes = [C.c_void_p, C.POINTER(A.AdRangeCmdsRecoverySoa)]
        L.rc_recovery_batch.argtypes = [C.c_void_p, C.POINTER(A.AdQuerySoa), C.c_uint32, C.c_uint64, C.c_uint64,
                                        C.POINTER(C.POINTER(RcResult))]
        L.rc_tid_cmp.argtypes = [C.c_uint64, C.c_uint64, C.c_int32, C.c_uint64, C.c_uint64, C.c_int32]
        _lib = L
    return _lib


class OracleError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("refcpu error %d: %s" % (code, msg))
        self.code = code


def _arr(p, n, dtype):
    if n == 0:
        return np.zeros(0, dtype)
    return np.ctypeslib.as_array(C.cast(p, C.POINTER(np.ctypeslib.as_ctypes_type(dtype))), shape=(n,)).copy()


def make_config(range_start_inclusive=0, elide=1, slices=None):
    cfg = A.AdConfig()
    cfg.device = 0
    cfg.range_start_inclusive = range_start_inclusive
    cfg.elide = elide
    keep = []
    if slices is not None and len(slices):
        s = np.ascontiguousarray(np.asarray(slices, np.int64)[:, 0])
        e = np.ascontiguousarray(np.asarray(slices, np.int64)[:, 1])
        keep = [s, e]
        cfg.n_slices = len(s)
        cfg.slice_start, cfg.slice_end = A.ptr(s), A.ptr(e)
    return cfg, keep


class OracleStore:
    """One reference CommandStore (InMemoryCommandStore semantics), CPU restatement."""

    def __init__(self, range_start_inclusive=0, elide=1, slices=None):
        L = lib()
        cfg, keep = make_config(range_start_inclusive, elide, slices)
        h = C.c_void_p()
        rc = L.rc_store_create(C.byref(cfg), C.byref(h))
        if rc:
            raise OracleError(rc, "create")
        self.h = h
        self._keep = keep

    def close(self):
        if self.h:
            lib().rc_store_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def _check(self, rc):
        if rc:
            raise OracleError(rc, lib().rc_last_error(self.h).decode())

    def load(self, workload):
        L = lib()
        self._check(L.rc_cfk_load(self.h, C.byref(workload.cfk.soa())))
        self._check(L.rc_range_cmds_load(self.h, C.byref(workload.cmds.soa())))
        self._check(L.rc_redundant_load(self.h, C.byref(workload.redundant.soa())))
        ss = getattr(workload, "slice_sets_csr", lambda: None)()
        if ss is not None:
            off, st, en = ss
            self._keep_ss = ss
            self._check(L.rc_slice_sets_load(self.h, len(off) - 1, A.ptr(off), A.ptr(st), A.ptr(en)))
        ms = workload.cfk.missing_soa()
        if ms is not None:
            self._check(L.rc_cfk_missing_load(self.h, C.byref(ms)))
        rs = workload.cmds.recovery_soa()
        if rs is not None:
            self._check(L.rc_range_cmds_recovery_load(self.h, C.byref(rs)))
        return self

    def range_cmds_update(self, cmds):
        """rc_range_cmds_update: registry upkeep rows (a RangeCommands: historical / erased / update per row)."""
        self._check(lib().rc_range_cmds_update(self.h, C.byref(cmds.soa())))

    def redundant_advance(self, redundant):
        """rc_redundant_advance: the same entries with watermarks moved forward (truncation on the next read)."""
        self._check(lib().rc_redundant_advance(self.h, C.byref(redundant.soa())))

    def recovery_batch(self, queries, scan, first=0, count=0):
        """rc_recovery_batch: BeginRecovery scan `scan` (AD_RECOVER_*) per request."""
        L = lib()
        out = C.POINTER(RcResult)()
        self._check(L.rc_recovery_batch(self.h, C.byref(queries.soa()), scan, first, count, C.byref(out)))
        try:
            return result_to_batch(out.contents)
        finally:
            L.rc_result_free(out)

    def deps_batch(self, queries, flags=A.AD_SNAPSHOT, first=0, count=0):
        L = lib()
        out = C.POINTER(RcResult)()
        self._check(L.rc_deps_batch(self.h, C.byref(queries.soa()), flags, first, count, C.byref(out)))
        try:
            return result_to_batch(out.contents)
        finally:
            L.rc_result_free(out)


def result_to_batch(r):
    n = r.n_txns
    maps = []
    for m in range(3):
        ko = _arr(r.keys_off[m], n + 1, np.uint64)
        to = _arr(r.txn_off[m], n + 1, np.uint64)
        oo = _arr(r.k2t_off[m], n + 1, np.uint64)
        nk, nt, no = int(ko[-1]), int(to[-1]), int(oo[-1])
        maps.append(DepsMap(ko, _arr(r.keys[m], nk, np.int64),
                            _arr(r.keys_end[m], nk, np.int64) if m == A.AD_MAP_RANGE else None,
                            to, Tids(_arr(r.txn_msb[m], nt, np.uint64), _arr(r.txn_lsb[m], nt, np.uint64),
                                     _arr(r.txn_node[m], nt, np.int32)),
                            oo, _arr(r.k2t[m], no, np.int32)))
    return PartialDepsBatch(maps, scan_entries=int(r.scan_entries))


def resolve(workload, elide=1, first=0, count=0):
    """Run a whole workload through a fresh oracle store."""
    st = OracleStore(workload.range_start_inclusive, elide, workload.slices)
    try:
        st.load(workload)
        return st.deps_batch(workload.queries, workload.flags, first, count)
    finally:
        st.close()


def recover(workload, scan, first=0, count=0):
    """One BeginRecovery scan over a workload through a fresh oracle store."""
    st = OracleStore(workload.range_start_inclusive, 1, workload.slices)
    try:
        st.load(workload)
        return st.recovery_batch(workload.queries, scan, first, count)
    finally:
        st.close()


def resolve_sharded(workload, n_shards, elide=1, bounds=None):
    """Oracle of the multi-GPU path: one CommandStore per EvenSplit token slice (synth.shard_bounds),
    each resolving every request restricted to its slice, then the per-store results combined
    request-wise with PartialDeps.with (rc_result_merge; CommandStores.java:576-593)."""
    from accord_deps import synth
    L = lib()
    lo, hi = synth.shard_bounds(n_shards) if bounds is None else bounds
    parts = []
    try:
        for g in range(n_shards):
            w = synth.slice_workload(workload, lo[g], hi[g])
            st = OracleStore(w.range_start_inclusive, elide, w.slices)
            try:
                st.load(w)
                out = C.POINTER(RcResult)()
                st._check(L.rc_deps_batch(st.h, C.byref(w.queries.soa()), w.flags, 0, 0, C.byref(out)))
                parts.append(out)
            finally:
                st.close()
        arr = (C.POINTER(RcResult) * len(parts))(*parts)
        merged = C.POINTER(RcResult)()
        rc = L.rc_result_merge(arr, len(parts), C.byref(merged))
        if rc:
            raise OracleError(rc, "merge")
        try:
            return result_to_batch(merged.contents)
        finally:
            L.rc_result_free(merged)
    finally:
        for p in parts:
            L.rc_result_free(p)


def _batch_to_rc(b, keep):
    """An RcResult viewing the arrays of a PartialDepsBatch (kept alive in `keep`)."""
    r = RcResult()
    r.n_txns = b.n_txns
    for m in range(3):
        mm = b.maps[m]
        arrs = dict(keys_off=A.as_u64(mm.keys_off), keys=A.as_i64(mm.keys),
                    keys_end=A.as_i64(mm.keys_end) if mm.keys_end is not None else
                    (A.as_i64(mm.keys) if m == A.AD_MAP_RANGE else None),
                    txn_off=A.as_u64(mm.txn_off), txn_msb=A.as_u64(mm.txn.msb), txn_lsb=A.as_u64(mm.txn.lsb),
                    txn_node=A.as_i32(mm.txn.node), k2t_off=A.as_u64(mm.k2t_off), k2t=A.as_i32(mm.k2t))
        keep.append(arrs)
        for name, a in arrs.items():
            getattr(r, name)[m] = A.ptr(a) if a is not None else None
    return r


def merge_batches(batches):
    """Request-wise PartialDeps.with over several PartialDepsBatch of equal length (rc_result_merge)."""
    L = lib()
    keep = []
    rcs = [_batch_to_rc(b, keep) for b in batches]
    arr = (C.POINTER(RcResult) * len(rcs))(*[C.pointer(r) for r in rcs])
    merged = C.POINTER(RcResult)()
    rc = L.rc_result_merge(arr, len(rcs), C.byref(merged))
    if rc:
        raise OracleError(rc, "merge")
    try:
        return result_to_batch(merged.contents)
    finally:
        L.rc_result_free(merged)


def levels(graph):
    out = np.zeros(len(graph.kind), np.uint32)
    rc = lib().rc_levels(C.byref(graph.soa()), A.ptr(out))
    if rc:
        raise OracleError(rc, "levels")
    return out


def preaccept(max_conflicts, reject_before, queries, permit_fast_path=1, node_epoch=0):
    """rc_preaccept: (minNonConflicting Tids, AD_PA_* flags) per request."""
    n = len(queries)
    om, ol = np.zeros(n, np.uint64), np.zeros(n, np.uint64)
    on, of = np.zeros(n, np.int32), np.zeros(n, np.uint8)
    mc = max_conflicts.soa() if max_conflicts is not None else None
    rb = reject_before.soa() if reject_before is not None else None
    rc = lib().rc_preaccept(C.byref(mc) if mc else None, C.byref(rb) if rb else None, C.byref(queries.soa()),
                            permit_fast_path, node_epoch, A.ptr(om), A.ptr(ol), A.ptr(on), A.ptr(of))
    if rc:
        raise OracleError(rc, "preaccept")
    return Tids(om, ol, on), of


def tid_cmp(a, b):
    return lib().rc_tid_cmp(a[0], a[1], a[2], b[0], b[1], b[2])
