"""ctypes binding of libaccord_deps.so (the HIP product path).

`DeviceCommandStore` mirrors the reference's per-store entry point for this path:
  SafeCommandStore.mapReduceActive / PreAccept.calculatePartialDeps (PreAccept.java:245-267),
batched: `calculate_partial_deps(queries)` answers every request of a batch, returning the
three RelationMultiMaps of each PartialDeps. Errors surface as `AccordDepsError` carrying the
AD_E_* code (the Java wrapper maps these to IllegalStateException).

There is no CPU fallback: if the library or a GPU is missing, this module raises.
"""
import ctypes as C
import weakref
import os

import numpy as np

from . import _abi as A
from .model import DepsMap, PartialDepsBatch, Tids

LIB_PATH = os.environ.get("ACCORD_DEPS_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libaccord_deps.so")

EXPORTS = ("ad_abi_version", "ad_ctx_create", "ad_ctx_destroy", "ad_last_error", "ad_cfk_load",
           "ad_range_cmds_load", "ad_redundant_load", "ad_prepare", "ad_deps_batch", "ad_result_free",
           "ad_deps_batch_device", "ad_dict", "ad_range_table", "ad_parts_export", "ad_parts_merge",
           "ad_copy_to_host", "ad_levels", "ad_levels_device", "ad_set_global_dict", "ad_preaccept_maps_load",
           "ad_preaccept_device", "ad_parts_union", "ad_cfk_missing_load", "ad_range_cmds_recovery_load", "ad_recovery_batch",
           "ad_recovery_batch_device", "ad_cfk_update", "ad_cfk_update_device", "ad_cfk_entries",
           "ad_cfk_ballots_load", "ad_cfk_ballots",
           "ad_exchange_local", "ad_comm_unique_id", "ad_comm_init", "ad_exchange", "ad_exchange_plan",
           "ad_check_result_device", "ad_check_snapshot", "ad_cfk_prune", "ad_cfk_byid", "ad_cfk_missing",
           "ad_cfk_load_pruned", "ad_host_register", "ad_host_unregister", "ad_deps_batch_into",
           "ad_debug_guard_check", "ad_host_alloc", "ad_host_free", "ad_cfk_update_status",
           "ad_slice_sets_load", "ad_redundant_advance", "ad_range_cmds_update")


class AccordDepsError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("libaccord_deps error %d: %s" % (code, msg))
        self.code = code


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise AccordDepsError(A.AD_E_DEVICE, "libaccord_deps.so not built (run __graft_entry__.build())")
        # One HIP runtime per process: if PyTorch is present it must load its libamdhip64.so.7
        # first, so that this library binds to the same runtime by soname (two runtimes in one
        # process cannot share the device: hipErrorNoDevice).
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = C.CDLL(LIB_PATH)
        L.ad_abi_version.restype = C.c_int
        L.ad_ctx_create.argtypes = [C.POINTER(A.AdConfig), C.POINTER(C.c_void_p)]
        L.ad_ctx_destroy.argtypes = [C.c_void_p]
        L.ad_last_error.argtypes = [C.c_void_p]
        L.ad_last_error.restype = C.c_char_p
        L.ad_cfk_load.argtypes = [C.c_void_p, C.POINTER(A.AdCfkSoa)]
        L.ad_range_cmds_load.argtypes = [C.c_void_p, C.POINTER(A.AdRangeCmdsSoa)]
        L.ad_redundant_load.argtypes = [C.c_void_p, C.POINTER(A.AdRedundantSoa)]
        L.ad_prepare.argtypes = [C.c_void_p]
        L.ad_slice_sets_load.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p]
        L.ad_deps_batch.argtypes = [C.c_void_p, C.POINTER(A.AdQuerySoa), C.c_uint32, C.POINTER(C.POINTER(A.AdDepsResult))]
        L.ad_result_free.argtypes = [C.POINTER(A.AdDepsResult)]
        L.ad_deps_batch_device.argtypes = [C.c_void_p, C.POINTER(A.AdQuerySoa), C.c_uint32, C.c_void_p,
                                           C.POINTER(A.AdDepsResult)]
        L.ad_dict.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_void_p), C.POINTER(C.c_void_p),
                              C.POINTER(C.c_void_p)]
        L.ad_range_table.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_void_p), C.POINTER(C.c_void_p)]
        L.ad_parts_export.argtypes = [C.c_void_p, C.POINTER(A.AdDepsResult), C.c_void_p, C.c_uint32, C.c_void_p,
                                      C.c_void_p, C.POINTER(A.AdParts), C.c_void_p]
        L.ad_parts_merge.argtypes = [C.c_void_p, C.POINTER(A.AdParts), C.c_uint32, C.c_void_p, C.c_uint64, C.c_uint64,
                                     C.c_void_p, C.POINTER(A.AdMerged)]
        L.ad_copy_to_host.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64]
        L.ad_parts_union.argtypes = [C.c_void_p, C.POINTER(A.AdParts), C.c_uint32, C.c_void_p, C.c_uint64, C.c_uint64,
                                     C.c_void_p, C.POINTER(A.AdMerged)]
        L.ad_set_global_dict.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p]
        L.ad_preaccept_maps_load.argtypes = [C.c_void_p, C.POINTER(A.AdRangeMapSoa), C.POINTER(A.AdRangeMapSoa)]
        L.ad_preaccept_device.argtypes = [C.c_void_p, C.POINTER(A.AdQuerySoa), C.c_uint32, C.c_uint64, C.c_void_p,
                                          C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.POINTER(A.AdStats)]
        L.ad_levels.argtypes = [C.c_void_p, C.POINTER(A.AdGraphSoa), C.c_void_p, C.POINTER(A.AdStats)]
        L.ad_levels_device.argtypes = [C.c_void_p, C.POINTER(A.AdGraphSoa), C.c_void_p, C.c_void_p,
                                       C.POINTER(A.AdStats)]
        L.ad_cfk_missing_load.argtypes = [C.c_void_p, C.POINTER(A.AdCfkMissingSoa)]
        L.ad_range_cmds_recovery_load.argtypes = [C.c_void_p, C.POINTER(A.AdRangeCmdsRecoverySoa)]
        L.ad_recovery_batch.argtypes = [C.c_void_p, C.POINTER(A.AdQuerySoa), C.c_uint32,
                                        C.POINTER(C.POINTER(A.AdDepsResult))]
        L.ad_recovery_batch_device.argtypes = [C.c_void_p, C.POINTER(A.AdQuerySoa), C.c_uint32, C.c_void_p,
                                               C.POINTER(A.AdDepsResult)]
        L.ad_cfk_update.argtypes = [C.c_void_p, C.POINTER(A.AdCfkUpdateSoa), C.POINTER(C.c_uint64), C.POINTER(A.AdStats)]
        L.ad_cfk_update_status.argtypes = [C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_int64)]
        L.ad_cfk_update_device.argtypes = [C.c_void_p, C.POINTER(A.AdCfkUpdateSoa), C.c_void_p, C.POINTER(C.c_uint64),
                                           C.POINTER(A.AdStats)]
        L.ad_cfk_ballots_load.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p]
        L.ad_cfk_ballots.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_void_p), C.POINTER(C.c_void_p),
                                     C.POINTER(C.c_void_p)]
        L.ad_cfk_entries.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_void_p), C.POINTER(C.c_void_p),
                                     C.POINTER(C.c_void_p), C.POINTER(C.c_void_p)]
        L.ad_exchange_local.argtypes = [C.POINTER(C.c_void_p), C.c_uint32, C.POINTER(C.POINTER(A.AdDepsResult)),
                                        C.POINTER(C.c_void_p), C.POINTER(C.c_void_p), C.c_void_p, C.c_void_p,
                                        C.POINTER(A.AdMerged), C.POINTER(A.AdExchangeStats)]
        L.ad_comm_unique_id.argtypes = [C.c_void_p]
        L.ad_comm_init.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int]
        L.ad_exchange.argtypes = [C.c_void_p, C.POINTER(A.AdDepsResult), C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint64,
                                  C.c_void_p, C.POINTER(A.AdMerged), C.POINTER(A.AdExchangeStats)]
        L.ad_exchange_plan.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.POINTER(A.AdXfer), C.c_void_p,
                                       C.c_void_p, C.POINTER(C.c_uint32)]
        L.ad_check_result_device.argtypes = [C.c_void_p, C.POINTER(A.AdDepsResult), C.c_void_p, C.POINTER(C.c_uint64),
                                             C.POINTER(C.c_uint64)]
        L.ad_redundant_advance.argtypes = [C.c_void_p, C.POINTER(A.AdRedundantSoa), C.POINTER(A.AdStats)]
        L.ad_range_cmds_update.argtypes = [C.c_void_p, C.POINTER(A.AdRangeCmdsSoa), C.POINTER(A.AdStats)]
        L.ad_cfk_prune.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_int32, C.c_int64, C.POINTER(C.c_uint64),
                                   C.POINTER(A.AdStats)]
        L.ad_cfk_byid.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_void_p), C.POINTER(C.c_void_p),
                                  C.POINTER(C.c_uint64), C.POINTER(C.c_void_p), C.POINTER(C.c_void_p),
                                  C.POINTER(C.c_void_p), C.POINTER(C.c_void_p)]
        L.ad_cfk_missing.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_void_p), C.POINTER(C.c_void_p),
                                     C.POINTER(C.c_void_p), C.POINTER(C.c_void_p)]
        L.ad_host_register.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64]
        L.ad_host_unregister.argtypes = [C.c_void_p, C.c_void_p]
        L.ad_debug_guard_check.argtypes = [C.c_char_p, C.c_uint64]
        L.ad_host_alloc.argtypes = [C.c_uint64, C.POINTER(C.c_void_p)]
        L.ad_host_free.argtypes = [C.c_void_p]
        L.ad_deps_batch_into.argtypes = [C.c_void_p, C.POINTER(A.AdQuerySoa), C.c_uint32, C.POINTER(A.AdDepsResult),
                                         C.c_void_p, C.c_void_p, C.c_uint32]
        L.ad_cfk_load_pruned.argtypes = [C.c_void_p, C.POINTER(C.c_uint64)] + [C.POINTER(C.c_void_p)] * 5
        L.ad_check_snapshot.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        _lib = L
    return _lib


def exchange_stats(s):
    return dict(bytes_moved=int(s.bytes_moved), ms_export=s.ms_export, ms_move=s.ms_move, ms_merge=s.ms_merge,
                ms_total=s.ms_total)


def comm_unique_id():
    """ad_comm_unique_id: the RCCL id rank 0 shares with the other ranks (bytes)."""
    b = (C.c_uint8 * A.AD_COMM_ID_BYTES)()
    rc = lib().ad_comm_unique_id(C.cast(b, C.c_void_p))
    if rc:
        raise AccordDepsError(rc, "ad_comm_unique_id")
    return bytes(b)


def exchange_row(counts, id_format, status=0, send_cap=None, recv_cap=None):
    """One rank's row of the exchange table (accord_deps.h, ad_exchange_plan): counts[world, 4] units
    per destination and array, then the header (format, status as -code, capacities in units)."""
    counts = np.asarray(counts, np.uint64).reshape(-1, 4)
    big = np.full(4, np.iinfo(np.uint64).max, np.uint64)
    hdr = np.zeros(A.AD_XROW_HDR, np.uint64)
    hdr[0] = A.AD_XROW_MAGIC
    hdr[1] = id_format
    hdr[2] = np.uint64(-int(status)) if status else 0
    hdr[4:8] = big if send_cap is None else np.asarray(send_cap, np.uint64)
    hdr[8:12] = big if recv_cap is None else np.asarray(recv_cap, np.uint64)
    return np.concatenate([counts.reshape(-1), hdr])


def exchange_plan(table, world, rank):
    """ad_exchange_plan (pure host code, no device): the transfers of `rank` from the gathered
    exchange table [world, AD_XROW_WORDS]. Returns (rc, xfers[4, world, 4] = (send_off, send_bytes,
    recv_off, recv_bytes) in bytes, recv_units[4], src_parts[world], flags)."""
    t = np.ascontiguousarray(table, np.uint64).reshape(-1)
    if len(t) != world * A.xrow_words(world):
        raise ValueError("exchange table of %d words for world %d" % (len(t), world))
    xf = (A.AdXfer * (4 * world))()
    ru = np.zeros(4, np.uint64)
    sp = np.zeros(world, np.uint64)
    fl = C.c_uint32(0)
    rc = lib().ad_exchange_plan(A.ptr(t), world, rank, xf, A.ptr(ru), A.ptr(sp), C.byref(fl))
    x = np.array([(f.send_off, f.send_bytes, f.recv_off, f.recv_bytes) for f in xf], np.uint64).reshape(4, world, 4)
    return rc, x, ru, sp, int(fl.value)


def exchange_local(stores, results, txn_index_ptrs, dest_firsts, txn_bases, n_owned):
    """ad_exchange_local over DeviceCommandStores of one process (slice order): every store's parts
    moved to the owners and merged there. Returns ([AdMerged] per store, stats dict)."""
    n = len(stores)
    ctxs = (C.c_void_p * n)(*[st.h.value for st in stores])
    res = (C.POINTER(A.AdDepsResult) * n)(*[C.pointer(r) for r in results])
    ti = (C.c_void_p * n)(*txn_index_ptrs)
    dfs = [np.ascontiguousarray(d, np.uint64) for d in dest_firsts]
    df = (C.c_void_p * n)(*[A.ptr(d) for d in dfs])
    tb = np.ascontiguousarray(txn_bases, np.uint64)
    no = np.ascontiguousarray(n_owned, np.uint64)
    out = (A.AdMerged * n)()
    s = A.AdExchangeStats()
    rc = lib().ad_exchange_local(ctxs, n, res, ti, df, A.ptr(tb), A.ptr(no), out, C.byref(s))
    if rc:
        msgs = [lib().ad_last_error(st.h).decode() for st in stores]
        raise AccordDepsError(rc, "; ".join(m for m in msgs if m))
    return list(out), exchange_stats(s)


def _view(p, n, dtype):
    if n == 0:
        return np.zeros(0, dtype)
    return np.ctypeslib.as_array(C.cast(p, C.POINTER(np.ctypeslib.as_ctypes_type(dtype))), shape=(n,))


def stats_dict(s):
    return dict(n_txns=s.n_txns, n_probes=s.n_probes, n_pairs=list(s.n_pairs), n_unique=list(s.n_unique),
                n_keys=list(s.n_keys), n_deferred=s.n_deferred, n_deferred_lean=s.n_deferred_lean, n_lean_pass2=s.n_lean_pass2,
                lean_wide1=bool(s.n_launches), lean_rpw1=int(s.lean_rpw1), lean_flags=int(s.lean_flags),
                ms_device=s.ms_device, ms_ingest=s.ms_ingest, ms_stage=list(s.ms_stage)[:7],
                bytes_stage=list(s.bytes_stage)[:7])


class DeviceCommandStore:
    """One CommandStore's snapshot resident on one MI355X (an `ad_ctx`)."""

    def __init__(self, device=0, range_start_inclusive=0, elide=1, slices=None, path=0):
        L = lib()
        cfg = A.AdConfig()
        cfg.device = device
        cfg.range_start_inclusive = range_start_inclusive
        cfg.elide = elide
        cfg.path = path
        self._keep = []
        self.global_dict = None          # Tids installed with set_global_dict
        if slices is not None and len(slices):
            s = np.ascontiguousarray(np.asarray(slices, np.int64)[:, 0])
            e = np.ascontiguousarray(np.asarray(slices, np.int64)[:, 1])
            self._keep = [s, e]
            cfg.n_slices = len(s)
            cfg.slice_start, cfg.slice_end = A.ptr(s), A.ptr(e)
        h = C.c_void_p()
        rc = L.ad_ctx_create(C.byref(cfg), C.byref(h))
        if rc:
            raise AccordDepsError(rc, L.ad_last_error(None).decode())
        self.h = h
        self.device = device

    def close(self):
        if getattr(self, "h", None):
            lib().ad_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def _check(self, rc):
        if rc:
            raise AccordDepsError(rc, lib().ad_last_error(self.h).decode())

    def load(self, workload, prepare=True):
        L = lib()
        self._check(L.ad_cfk_load(self.h, C.byref(workload.cfk.soa())))
        self._check(L.ad_range_cmds_load(self.h, C.byref(workload.cmds.soa())))
        self._check(L.ad_redundant_load(self.h, C.byref(workload.redundant.soa())))
        ba = workload.cfk.ballot_arrays()
        if ba is not None:
            self._check(L.ad_cfk_ballots_load(self.h, len(ba[0]), A.ptr(ba[0]), A.ptr(ba[1]), A.ptr(ba[2])))
        ms = workload.cfk.missing_soa()
        if ms is not None:
            self._check(L.ad_cfk_missing_load(self.h, C.byref(ms)))
        rs = workload.cmds.recovery_soa()
        if rs is not None:
            self._check(L.ad_range_cmds_recovery_load(self.h, C.byref(rs)))
        ss = getattr(workload, "slice_sets_csr", lambda: None)()
        if ss is not None:
            self.load_slice_sets(*ss)
        if prepare:
            self._check(L.ad_prepare(self.h))
        return self

    def load_slice_sets(self, set_off, start, end):
        """ad_slice_sets_load: the store's slice sets (CSR of normalised ranges) that Queries.slice_set names."""
        off, s, e = A.as_u64(set_off), A.as_i64(start), A.as_i64(end)
        self._check(lib().ad_slice_sets_load(self.h, len(off) - 1 if len(off) else 0, A.ptr(off), A.ptr(s), A.ptr(e)))

    def cfk_update(self, updates):
        """CommandsForKey.update for a batch (host arrays): returns (n_applied, stats)."""
        n, st = C.c_uint64(), A.AdStats()
        self._check(lib().ad_cfk_update(self.h, C.byref(updates.soa()), C.byref(n), C.byref(st)))
        return n.value, stats_dict(st)

    def cfk_update_status(self):
        """ad_cfk_update_status: (explicit updates of the last batch stand, index of the update a failure
        names or -1)."""
        ap, fi = C.c_int(), C.c_int64()
        self._check(lib().ad_cfk_update_status(self.h, C.byref(ap), C.byref(fi)))
        return bool(ap.value), int(fi.value)

    def cfk_update_device(self, udev, stream=None):
        """As cfk_update over device arrays (an AdCfkUpdateSoa of device pointers)."""
        n, st = C.c_uint64(), A.AdStats()
        self._check(lib().ad_cfk_update_device(self.h, C.byref(udev), stream, C.byref(n), C.byref(st)))
        return n.value, stats_dict(st)

    def range_cmds_update(self, cmds):
        """ad_range_cmds_update: registry upkeep rows (a RangeCommands: historical / erased / update per row);
        the range part of the snapshot follows without a rebuild. Returns stats."""
        st = A.AdStats()
        self._check(lib().ad_range_cmds_update(self.h, C.byref(cmds.soa()), C.byref(st)))
        return stats_dict(st)

    def redundant_advance(self, redundant):
        """ad_redundant_advance: the loaded RedundantBefore's entries with epochs / watermarks moved forward; the
        CommandsForKeys are truncated on the device. Returns stats (n_keys[0] entries removed, [1] keys changed)."""
        st = A.AdStats()
        self._check(lib().ad_redundant_advance(self.h, C.byref(redundant.soa()), C.byref(st)))
        return stats_dict(st)

    def cfk_prune(self, keys=None, prune_interval=1, min_hlc_delta=0):
        """Pruning.maybePrune for the CommandsForKey of `keys` (None: every key): returns
        (entries removed, stats)."""
        n, st = C.c_uint64(), A.AdStats()
        ka = None if keys is None else np.ascontiguousarray(np.asarray(keys, np.int64))
        self._check(lib().ad_cfk_prune(self.h, None if ka is None else A.ptr(ka), 0 if ka is None else len(ka),
                                       int(prune_interval), int(min_hlc_delta), C.byref(n), C.byref(st)))
        return n.value, stats_dict(st)

    def cfk_missing(self):
        """(off, Tids) of every entry's TxnInfo.missing() as it stands."""
        ne = C.c_uint64()
        po, pm, pl, pn = (C.c_void_p() for _ in range(4))
        self._check(lib().ad_cfk_missing(self.h, C.byref(ne), C.byref(po), C.byref(pm), C.byref(pl), C.byref(pn)))
        off = _view(po, ne.value + 1, np.uint64).copy()
        nm = int(off[-1]) if len(off) else 0
        return off, Tids(_view(pm, nm, np.uint64).copy(), _view(pl, nm, np.uint64).copy(), _view(pn, nm, np.int32).copy())

    def cfk_load_pruned(self):
        """LoadPruned requests of the last update batch (ad_cfk_load_pruned): [(update index, key,
        (msb, lsb, node))] in batch order."""
        n = C.c_uint64()
        pu, pk, pm, pl, pn = (C.c_void_p() for _ in range(5))
        self._check(lib().ad_cfk_load_pruned(self.h, C.byref(n), C.byref(pu), C.byref(pk), C.byref(pm), C.byref(pl),
                                             C.byref(pn)))
        m = n.value
        u, k = _view(pu, m, np.uint64), _view(pk, m, np.int64)
        ms, ls, ns = _view(pm, m, np.uint64), _view(pl, m, np.uint64), _view(pn, m, np.int32)
        return [(int(u[j]), int(k[j]), (int(ms[j]), int(ls[j]), int(ns[j]))) for j in range(m)]

    def cfk_byid(self):
        """(keys, seg, txnIds (Tids), prunedBefore indices) of the store's CommandsForKeys as they stand."""
        nk, ne = C.c_uint64(), C.c_uint64()
        pk, ps, pm, pl, pn, pp = (C.c_void_p() for _ in range(6))
        self._check(lib().ad_cfk_byid(self.h, C.byref(nk), C.byref(pk), C.byref(ps), C.byref(ne), C.byref(pm), C.byref(pl),
                                      C.byref(pn), C.byref(pp)))
        k, e = nk.value, ne.value
        return (_view(pk, k, np.int64).copy(), _view(ps, k + 1, np.uint64).copy(),
                Tids(_view(pm, e, np.uint64).copy(), _view(pl, e, np.uint64).copy(), _view(pn, e, np.int32).copy()),
                _view(pp, k, np.int64).copy())

    def cfk_entries(self):
        """(status, executeAt Tids) of every entry as the store now holds them (load order)."""
        n = C.c_uint64()
        ps, pm, pl, pn = C.c_void_p(), C.c_void_p(), C.c_void_p(), C.c_void_p()
        self._check(lib().ad_cfk_entries(self.h, C.byref(n), C.byref(ps), C.byref(pm), C.byref(pl), C.byref(pn)))
        k = n.value
        return _view(ps, k, np.uint8).copy(), Tids(_view(pm, k, np.uint64).copy(), _view(pl, k, np.uint64).copy(),
                                                   _view(pn, k, np.int32).copy())

    def cfk_ballots(self):
        """TxnInfo.ballot() of every entry as the store now holds them (Tids, load order)."""
        n = C.c_uint64()
        pm, pl, pn = C.c_void_p(), C.c_void_p(), C.c_void_p()
        self._check(lib().ad_cfk_ballots(self.h, C.byref(n), C.byref(pm), C.byref(pl), C.byref(pn)))
        k = n.value
        return Tids(_view(pm, k, np.uint64).copy(), _view(pl, k, np.uint64).copy(), _view(pn, k, np.int32).copy())

    def dictionary(self):
        n = C.c_uint64()
        pm, pl, pn = C.c_void_p(), C.c_void_p(), C.c_void_p()
        self._check(lib().ad_dict(self.h, C.byref(n), C.byref(pm), C.byref(pl), C.byref(pn)))
        k = n.value
        return Tids(_view(pm, k, np.uint64).copy(), _view(pl, k, np.uint64).copy(), _view(pn, k, np.int32).copy())

    def set_global_dict(self, g):
        """Install the global TxnId dictionary (Tids, ascending and unique; exchange.build_global_dict):
        parts are then exported as uint32 global ranks (accord_deps.h ad_set_global_dict)."""
        m = np.ascontiguousarray(g.msb, np.uint64)
        ls = np.ascontiguousarray(g.lsb, np.uint64)
        nd = np.ascontiguousarray(g.node, np.int32)
        self._check(lib().ad_set_global_dict(self.h, len(m), A.ptr(m), A.ptr(ls), A.ptr(nd)))
        self.global_dict = Tids(m, ls, nd)

    def load_preaccept_maps(self, max_conflicts=None, reject_before=None):
        """Install the store's maxConflicts / rejectBefore (model.RangeMap, None = empty)."""
        mc = max_conflicts.soa() if max_conflicts is not None else None
        rb = reject_before.soa() if reject_before is not None else None
        self._check(lib().ad_preaccept_maps_load(self.h, C.byref(mc) if mc else None, C.byref(rb) if rb else None))

    def preaccept_device(self, qdev, out, permit_fast_path=1, node_epoch=0, stream=None):
        """ad_preaccept_device: `qdev` device queries, `out` dict of device tensors msb/lsb/node/flags.
        Returns the stats dict."""
        s = A.AdStats()
        self._check(lib().ad_preaccept_device(self.h, C.byref(qdev), permit_fast_path, node_epoch, stream,
                                              out["msb"].data_ptr(), out["lsb"].data_ptr(), out["node"].data_ptr(),
                                              out["flags"].data_ptr(), C.byref(s)))
        return stats_dict(s)

    def preaccept(self, queries, permit_fast_path=1, node_epoch=0):
        """Host convenience: (minNonConflicting Tids, AD_PA_* flags) per request."""
        import torch
        dev = torch.device("cuda", self.device)
        qdev, keep = device_queries(queries, dev)
        n = len(queries)
        out = dict(msb=torch.zeros(max(n, 1), dtype=torch.int64, device=dev),
                   lsb=torch.zeros(max(n, 1), dtype=torch.int64, device=dev),
                   node=torch.zeros(max(n, 1), dtype=torch.int32, device=dev),
                   flags=torch.zeros(max(n, 1), dtype=torch.uint8, device=dev))
        torch.cuda.synchronize(dev)
        st = self.preaccept_device(qdev, out, permit_fast_path, node_epoch)
        o = {k: v.cpu().numpy()[:n] for k, v in out.items()}
        return Tids(o["msb"].view(np.uint64), o["lsb"].view(np.uint64), o["node"]), o["flags"], st

    def range_table(self):
        n = C.c_uint64()
        ps, pe = C.c_void_p(), C.c_void_p()
        self._check(lib().ad_range_table(self.h, C.byref(n), C.byref(ps), C.byref(pe)))
        return _view(ps, n.value, np.int64).copy(), _view(pe, n.value, np.int64).copy()

    def calculate_partial_deps(self, queries, flags=A.AD_SNAPSHOT):
        """Batched PreAccept.calculatePartialDeps; host arrays in, materialised PartialDeps out."""
        L = lib()
        out = C.POINTER(A.AdDepsResult)()
        self._check(L.ad_deps_batch(self.h, C.byref(queries.soa()), flags, C.byref(out)))
        return self._host_result(out)

    def recovery_scan(self, queries, scan):
        """Batched BeginRecovery scan `scan` (A.AD_RECOVER_*; ad_recovery_batch): host arrays in,
        materialised Deps out (keyDeps / directKeyDeps of the visited (key, txnId) pairs)."""
        out = C.POINTER(A.AdDepsResult)()
        self._check(lib().ad_recovery_batch(self.h, C.byref(queries.soa()), scan, C.byref(out)))
        return self._host_result(out)

    def recovery_scan_device(self, qdev, scan, stream=None):
        """Device-resident recovery scan (ad_recovery_batch_device): (AdDepsResult of device pointers, stats)."""
        out = A.AdDepsResult()
        self._check(lib().ad_recovery_batch_device(self.h, C.byref(qdev), scan, stream, C.byref(out)))
        return out, stats_dict(out.stats)

    def _host_result(self, out):
        L = lib()
        try:
            r = out.contents
            n = r.n_txns
            raw = []
            for m in range(A.NMAPS):
                ko = _view(r.keys_off[m], n + 1, np.uint64).copy()
                to = _view(r.txn_off[m], n + 1, np.uint64).copy()
                oo = _view(r.k2t_off[m], n + 1, np.uint64).copy()
                raw.append((ko, _view(r.keys[m], int(ko[-1]), np.int64).copy(), to,
                            _view(r.txns[m], int(to[-1]), np.uint32).copy(), oo,
                            _view(r.k2t[m], int(oo[-1]), np.int32).copy()))
            stats = stats_dict(r.stats)
        finally:
            L.ad_result_free(out)
        return self.materialise(raw, stats)

    def deps_batch_stats(self, queries, flags=A.AD_SNAPSHOT):
        """ad_deps_batch as a host caller uses it (host arrays in, host CSR arrays out; snapshot
        ingest, PCIe and device work included), without building Python objects from the result.
        Returns the stats dict."""
        L = lib()
        out = C.POINTER(A.AdDepsResult)()
        self._check(L.ad_deps_batch(self.h, C.byref(queries.soa()), flags, C.byref(out)))
        try:
            return stats_dict(out.contents.stats)
        finally:
            L.ad_result_free(out)

    class _Block:
        """One block of output memory that owns its pinning: library-pinned (ad_host_alloc) or numpy pages
        registered with ad_host_register. Exposes the memory through __array_interface__, so every numpy
        view of it keeps it alive (the block is its base); the memory is freed / unpinned by a finalizer
        when the last view and the block are gone -- a view that outlives its HostOut stays valid."""
        PAGE = 4096

        def __init__(self, store, nbytes, pin):
            nbytes = max(int(nbytes), 1)
            if pin is True:
                p = C.c_void_p()
                rc = lib().ad_host_alloc(nbytes, C.byref(p))
                if rc or not p.value:
                    raise AccordDepsError(rc or A.AD_E_NOMEM, "ad_host_alloc(%d) failed" % nbytes)
                addr = p.value
                self._fin = weakref.finalize(self, DeviceCommandStore._Block._host_free, addr)
            else:
                # zeroed numpy memory on whole pages of its own: a registration covers exactly its pages,
                # so pinning (page-granular) never shares a page with another array or the Python heap
                P = DeviceCommandStore._Block.PAGE
                span = -(-nbytes // P) * P
                raw = np.zeros(span + P, np.uint8)
                at = (-raw.ctypes.data) % P
                addr = raw.ctypes.data + at
                if pin == "register":
                    store._check(lib().ad_host_register(store.h, C.c_void_p(addr), span))
                    # the finalizer holds the numpy memory until it has been unpinned
                    self._fin = weakref.finalize(self, DeviceCommandStore._Block._unregister, addr, raw)
                else:
                    self._fin = weakref.finalize(self, lambda r: None, raw)
            self.__array_interface__ = {"data": (addr, False), "shape": (nbytes,), "typestr": "|u1", "version": 3}

        @staticmethod
        def _host_free(addr):
            if lib().ad_host_free(C.c_void_p(addr)) != 0:
                raise AccordDepsError(A.AD_E_DEVICE, "ad_host_free failed")

        @staticmethod
        def _unregister(addr, raw):
            if lib().ad_host_unregister(None, C.c_void_p(addr)) != 0:
                raise AccordDepsError(A.AD_E_DEVICE, "ad_host_unregister failed")

        def array(self, shape, dtype):
            dtype = np.dtype(dtype)
            count = int(np.prod(shape))
            a = np.asarray(self)[:count * dtype.itemsize].view(dtype).reshape(shape)
            a[...] = 0
            return a

    class HostOut:
        """Caller-owned host output arrays of ad_deps_batch_into (numpy). pin=True: views of pinned memory
        from ad_host_alloc (the default: copy-outs are DMAs straight into them); pin="register": numpy
        pages of their own pinned with ad_host_register (the Panama binding's way);
        pin=False: plain pageable numpy (filled through the library's staging). Grown (re-made) when a
        batch needs more. Every array keeps its memory (a _Block) alive: release() only drops this
        object's references, and the memory is freed / unpinned once no array of it is left."""

        def __init__(self, store, n, cap, pin=True):
            self.store, self.pin, self.n = store, pin, n
            self.cap = [int(x) for x in cap]
            shapes = [((9, n + 1), np.uint64)] + [(max(1, self.cap[3 * m]), np.int64) for m in range(3)] + \
                     [(max(1, self.cap[3 * m + 1]), np.uint32) for m in range(3)] + \
                     [(max(1, self.cap[3 * m + 2]), np.int32) for m in range(3)]
            arrs = []
            for shape, dt in shapes:
                nbytes = int(np.prod(shape)) * np.dtype(dt).itemsize
                arrs.append(DeviceCommandStore._Block(store, nbytes, pin).array(shape, dt))
            self.off = arrs[0]
            self.keys, self.txns, self.k2t = arrs[1:4], arrs[4:7], arrs[7:10]

        def release(self):
            # the store's copy stream is drained by every ad_deps_batch_into return; the memory goes with
            # the last array of it
            self.off = self.keys = self.txns = self.k2t = None

        def soa(self):
            r = A.AdDepsResult()
            r.n_txns = self.n
            for m in range(3):
                r.keys_off[m] = A.ptr(self.off[3 * m])
                r.txn_off[m] = A.ptr(self.off[3 * m + 1])
                r.k2t_off[m] = A.ptr(self.off[3 * m + 2])
                r.keys[m] = A.ptr(self.keys[m])
                r.txns[m] = A.ptr(self.txns[m])
                r.k2t[m] = A.ptr(self.k2t[m])
            return r

    def deps_batch_into(self, queries, flags=A.AD_SNAPSHOT, slices=0, out=None, pin=True, materialise=True):
        """ad_deps_batch_into: host arrays in, caller-owned (pinned) host arrays out, the batch resolved in
        slices whose copy-out overlaps the next slice. `out`: a HostOut to reuse (grown on AD_E_SPACE).
        Returns (PartialDepsBatch or None, stats dict, the HostOut)."""
        n = len(queries)
        mine = False                        # this call made `out` (a caller's HostOut is never released here)
        if out is None or out.n != n:
            np_ = queries.n_probes
            out = DeviceCommandStore.HostOut(self, n, [np_, 2 * np_, 4 * np_] * 3, pin)
            mine = True
        need = np.zeros(9, np.uint64)
        soa = queries.soa()
        try:
            while True:
                r = out.soa()
                cap = np.asarray(out.cap, np.uint64)
                rc = lib().ad_deps_batch_into(self.h, C.byref(soa), flags, C.byref(r), A.ptr(cap), A.ptr(need), slices)
                if rc != A.AD_E_SPACE:
                    break
                if mine:
                    out.release()
                out = DeviceCommandStore.HostOut(self, n, [int(x) + int(x) // 4 + 16 for x in need], pin)
                mine = True
            self._check(rc)
        except BaseException:
            if mine:
                out.release()
            raise
        stats = stats_dict(r.stats)
        if not materialise:
            return None, stats, out
        raw = []
        for m in range(3):
            ko, to, oo = out.off[3 * m].copy(), out.off[3 * m + 1].copy(), out.off[3 * m + 2].copy()
            raw.append((ko, out.keys[m][:int(ko[-1])].copy(), to, out.txns[m][:int(to[-1])].copy(), oo,
                        out.k2t[m][:int(oo[-1])].copy()))
        return self.materialise(raw, stats), stats, out

    def materialise(self, raw, stats=None):
        d = self.dictionary()
        rs, re = self.range_table()
        maps = []
        for m, (ko, keys, to, tx, oo, k2t) in enumerate(raw):
            txn = d.take(tx.astype(np.int64))
            if m == A.AD_MAP_RANGE:
                rid = keys.astype(np.int64)
                maps.append(DepsMap(ko, rs[rid], re[rid], to, txn, oo, k2t))
            else:
                maps.append(DepsMap(ko, keys, None, to, txn, oo, k2t))
        return PartialDepsBatch(maps, stats=stats or {})

    def deps_batch_device(self, qdev, stream=None, parts_only=False, regions=False):
        """Device-resident batch. `qdev` is an AdQuerySoa of device pointers. Returns
        (AdDepsResult with device pointers owned by the store, stats dict). `parts_only`: the result
        is only exported as parts (AD_PARTS_ONLY: no packed arrays); `regions`: the result is read
        through its regions (AD_REGIONS: no packed arrays)."""
        out = A.AdDepsResult()
        flags = (A.AD_SNAPSHOT | A.AD_N_KEYS | (A.AD_PARTS_ONLY if parts_only else 0) |
                 (A.AD_REGIONS if regions else 0))
        self._check(lib().ad_deps_batch_device(self.h, C.byref(qdev), flags, stream, C.byref(out)))
        return out, stats_dict(out.stats)

    # ---- debug invariant checks (accord_deps.h) -------------------------------------
    def check_result_device(self, res, stream=None):
        """(violations, first failing request * 3 + map or None) of a device result."""
        n, first = C.c_uint64(0), C.c_uint64(0)
        self._check(lib().ad_check_result_device(self.h, C.byref(res), stream, C.byref(n), C.byref(first)))
        return n.value, (None if first.value == 2 ** 64 - 1 else first.value)

    def check_snapshot(self):
        """(violations, first failing key index or None) of the prepared snapshot."""
        n, first = C.c_uint64(0), C.c_uint64(0)
        self._check(lib().ad_check_snapshot(self.h, C.byref(n), C.byref(first)))
        return n.value, (None if first.value == 2 ** 64 - 1 else first.value)

    # ---- multi-GPU exchange (accord_deps.h "multi-GPU exchange") ----------------
    def export_parts(self, res, txn_index_ptr, dest_first, parts, stream=None):
        """Export the device result `res` as parts into the device arrays of `parts` (AdParts with
        capacities). Returns (rc, dest_counts[n_dest, 4]); rc is AD_OK or AD_E_SPACE (sizes set in
        `parts`, caller grows its buffers and calls again)."""
        df = np.ascontiguousarray(dest_first, dtype=np.uint64)
        n_dest = len(df) - 1
        counts = np.zeros((n_dest, 4), np.uint64)
        rc = lib().ad_parts_export(self.h, C.byref(res), txn_index_ptr, n_dest, A.ptr(df), stream,
                                   C.byref(parts), A.ptr(counts))
        if rc not in (A.AD_OK, A.AD_E_SPACE):
            self._check(rc)
        return rc, counts

    def merge_parts(self, parts, src_parts, txn_base, n_owned, stream=None):
        """K3: merge received parts (device AdParts, sources concatenated in slice order) into the
        PartialDeps of requests [txn_base, txn_base + n_owned). Returns an AdMerged (device)."""
        sp = np.ascontiguousarray(src_parts, dtype=np.uint64)
        out = A.AdMerged()
        self._check(lib().ad_parts_merge(self.h, C.byref(parts), len(sp), A.ptr(sp), txn_base, n_owned, stream,
                                         C.byref(out)))
        return out

    def union_parts(self, parts, src_parts, txn_base, n_owned, stream=None):
        """ad_parts_union: Deps.merge of rank-format parts whose keys may overlap across sources
        (replica replies). Returns an AdMerged (device)."""
        sp = np.ascontiguousarray(src_parts, dtype=np.uint64)
        out = A.AdMerged()
        self._check(lib().ad_parts_union(self.h, C.byref(parts), len(sp), A.ptr(sp), txn_base, n_owned, stream,
                                         C.byref(out)))
        return out

    def comm_init(self, uid, rank, world):
        """ad_comm_init: join the node's RCCL communicator (uid from comm_unique_id on rank 0)."""
        b = (C.c_uint8 * A.AD_COMM_ID_BYTES).from_buffer_copy(uid)
        self._check(lib().ad_comm_init(self.h, C.cast(b, C.c_void_p), rank, world))

    def exchange(self, res, txn_index_ptr, dest_first, txn_base, n_owned, stream=None):
        """ad_exchange (RCCL): this rank's export, exchange and K3 merge. Returns (AdMerged, stats)."""
        df = np.ascontiguousarray(dest_first, np.uint64)
        out = A.AdMerged()
        s = A.AdExchangeStats()
        self._check(lib().ad_exchange(self.h, C.byref(res), txn_index_ptr, A.ptr(df), txn_base, n_owned, stream,
                                      C.byref(out), C.byref(s)))
        return out, exchange_stats(s)

    def levels_device(self, gdev, out_ptr, stream=None):
        """ad_levels_device: graph and output already in HBM. Returns the stats dict."""
        s = A.AdStats()
        self._check(lib().ad_levels_device(self.h, C.byref(gdev), out_ptr, stream, C.byref(s)))
        return levels_stats(s)

    def device_result_to_host(self, res, idx=None, via_regions=None):
        """Materialise the device result `res` of the last deps_batch_device as a PartialDepsBatch, for
        every request or only the requests `idx`: from the packed arrays, or (`via_regions`, default
        when the packed arrays are absent: AD_REGIONS) from each request's region."""
        if via_regions is None:
            via_regions = not res.keys[0]
        if via_regions:
            return self.materialise(self._regions_raw(res, idx))
        n = res.n_txns
        raw = []
        for m in range(A.NMAPS):
            ko = self._d2h(res.keys_off[m], n + 1, np.uint64)
            to = self._d2h(res.txn_off[m], n + 1, np.uint64)
            oo = self._d2h(res.k2t_off[m], n + 1, np.uint64)
            raw.append((ko, self._d2h(res.keys[m], int(ko[-1]), np.int64), to,
                        self._d2h(res.txns[m], int(to[-1]), np.uint32), oo, self._d2h(res.k2t[m], int(oo[-1]), np.int32)))
        if idx is not None:
            idx = np.asarray(idx, np.int64)
            sub = []
            for ko, keys, to, tx, oo, k2t in raw:
                parts = []
                for off, arr in ((ko, keys), (to, tx), (oo, k2t)):
                    o = off.astype(np.int64)
                    cnt = o[idx + 1] - o[idx]
                    no = np.zeros(len(idx) + 1, np.uint64)
                    no[1:] = np.cumsum(cnt)
                    src = np.repeat(o[idx] - no[:-1].astype(np.int64), cnt) + np.arange(int(no[-1]))
                    parts += [no, arr[src]]
                sub.append(tuple(parts))
            raw = sub
        return self.materialise(raw)

    def _regions_raw(self, res, idx=None):
        """The (offsets, keys, offsets, txnIds, offsets, keysToTxnIds) columns of every map, read from
        the regions of a device result (accord_deps.h ad_deps_result.regions) for the requests idx."""
        n = res.n_txns
        arena = self._d2h(res.regions, int(res.regions_bytes), np.uint8)
        sel = np.arange(n, dtype=np.int64) if idx is None else np.asarray(idx, np.int64)

        words = {8: arena[:len(arena) // 8 * 8].view(np.int64), 4: arena[:len(arena) // 4 * 4].view(np.int32)}

        def gather(base, cnt, width, dtype):
            # cnt[i] elements of `width` bytes from byte base[i] on (a multiple of width), concatenated
            tot = int(cnt.sum())
            if tot == 0:
                return np.zeros(0, dtype)
            w = words[width]
            pos = np.repeat(base // width, cnt) + (np.arange(tot) - np.repeat(np.cumsum(cnt) - cnt, cnt))
            if pos.max() >= len(w):
                raise AssertionError("a region reaches beyond regions_bytes")
            return w[pos].view(dtype)

        raw = []
        for m in range(A.NMAPS):
            ko = self._d2h(res.keys_off[m], n + 1, np.uint64).astype(np.int64)
            to = self._d2h(res.txn_off[m], n + 1, np.uint64).astype(np.int64)
            oo = self._d2h(res.k2t_off[m], n + 1, np.uint64).astype(np.int64)
            ro = self._d2h(res.region_off[m], n, np.uint64).astype(np.int64)
            nk, nt, no = ko[sel + 1] - ko[sel], to[sel + 1] - to[sel], oo[sel + 1] - oo[sel]
            base = np.where(nk > 0, ro[sel], 0)
            if np.any(base % 8):
                raise AssertionError("a region is not 8-byte aligned")
            cols = []
            for cnt, off, width, dt in ((nk, base, 8, np.int64), (nt, base + 8 * nk, 4, np.uint32),
                                        (no, base + 8 * nk + 4 * nt, 4, np.int32)):
                o = np.zeros(len(sel) + 1, np.uint64)
                o[1:] = np.cumsum(cnt)
                cols += [o, gather(off, cnt, width, dt)]
            raw.append(tuple(cols))
        return raw

    def _d2h(self, p, n, dtype):
        a = np.zeros(max(n, 0), dtype)
        if n:
            self._check(lib().ad_copy_to_host(self.h, A.ptr(a), p, a.nbytes))
        return a

    def merged_to_host(self, mg, idx=None):
        """Materialise an AdMerged into a PartialDepsBatch (ids as TxnIds, ranges as (start, end)), for
        every owned request or only the owned requests `idx` (indices from 0 = txn_base)."""
        n = mg.n_txns
        maps = []
        for m in range(A.NMAPS):
            w = 2 if m == A.AD_MAP_RANGE else 1
            ko = self._d2h(mg.keys_off[m], n + 1, np.uint64)
            to = self._d2h(mg.txn_off[m], n + 1, np.uint64)
            oo = self._d2h(mg.k2t_off[m], n + 1, np.uint64)
            kw = self._d2h(mg.keys[m], w * int(mg.n_keys[m]), np.int64).reshape(-1, w)
            k2t = self._d2h(mg.k2t[m], int(mg.n_k2t[m]), np.int32)
            rank_ids = mg.id_format == A.AD_IDS_RANK
            if rank_ids:
                if self.global_dict is None:
                    raise ValueError("rank-format merge result without the global dictionary")
                ids = self._d2h(mg.txns[m], int(mg.n_ids[m]), np.uint32)
            else:
                ids = self._d2h(mg.txns[m], 3 * int(mg.n_ids[m]), np.int64).reshape(-1, 3)
            if idx is not None:
                ix = np.asarray(idx, np.int64)
                cols = []
                for off, arr in ((ko, kw), (to, ids), (oo, k2t)):
                    o = off.astype(np.int64)
                    cnt = o[ix + 1] - o[ix]
                    no = np.zeros(len(ix) + 1, np.uint64)
                    no[1:] = np.cumsum(cnt)
                    src = np.repeat(o[ix] - no[:-1].astype(np.int64), cnt) + np.arange(int(no[-1]))
                    cols += [no, arr[src]]
                ko, kw, to, ids, oo, k2t = cols
            if rank_ids:
                txn = self.global_dict.take(ids.astype(np.int64))
            else:
                txn = Tids(ids[:, 0].view(np.uint64).copy(), ids[:, 1].view(np.uint64).copy(), ids[:, 2].astype(np.int32))
            if m == A.AD_MAP_RANGE:
                maps.append(DepsMap(ko, kw[:, 0].copy(), kw[:, 1].copy(), to, txn, oo, k2t))
            else:
                maps.append(DepsMap(ko, kw[:, 0].copy(), None, to, txn, oo, k2t))
        return PartialDepsBatch(maps)


def device_queries(q, dev):
    """Stage a Queries batch in HBM (torch tensors as allocator). Returns (AdQuerySoa of device
    pointers, dict of the tensors that must stay alive)."""
    import torch

    def to_dev(a):
        a = np.ascontiguousarray(a)
        if a.dtype == np.uint64:
            a = a.view(np.int64)
        return torch.from_numpy(a).to(dev)
    keep = {k: to_dev(v) for k, v in [
        ("tm", q.txn.msb), ("tl", q.txn.lsb), ("tn", q.txn.node),
        ("em", q.exec.msb), ("el", q.exec.lsb), ("en", q.exec.node),
        ("ko", q.key_off), ("k", q.keys)]}
    if q.min_epoch is not None:
        keep["me"] = to_dev(np.asarray(q.min_epoch, np.int64))
    if q.range_off is not None:
        keep["ro"], keep["rs"], keep["re"] = to_dev(q.range_off), to_dev(q.range_start), to_dev(q.range_end)
    if q.slice_set is not None:
        keep["ss"] = to_dev(np.asarray(q.slice_set, np.uint32).view(np.int32))
    s = A.AdQuerySoa()
    s.n_txns = len(q)
    s.txn_msb, s.txn_lsb, s.txn_node = keep["tm"].data_ptr(), keep["tl"].data_ptr(), keep["tn"].data_ptr()
    s.exec_msb, s.exec_lsb, s.exec_node = keep["em"].data_ptr(), keep["el"].data_ptr(), keep["en"].data_ptr()
    s.min_epoch = keep["me"].data_ptr() if "me" in keep else None
    s.key_off, s.keys = keep["ko"].data_ptr(), keep["k"].data_ptr()
    s.n_keys = int(q.key_off[-1]) if len(q.key_off) else 0
    if q.range_off is not None:
        s.range_off, s.range_start, s.range_end = keep["ro"].data_ptr(), keep["rs"].data_ptr(), keep["re"].data_ptr()
        s.n_ranges = q.n_ranges
    s.slice_set = keep["ss"].data_ptr() if "ss" in keep else None
    return s, keep


def resolve(workload, device=0, elide=1, path=0, via="host"):
    """PartialDeps of a workload's batch: through ad_deps_batch (via "host"), or with the queries in HBM
    through ad_deps_batch_device read back from the packed arrays ("device") or from the regions
    (AD_REGIONS, "regions"; SNAPSHOT batches only)."""
    st = DeviceCommandStore(device, workload.range_start_inclusive, elide, workload.slices, path)
    try:
        st.load(workload)
        if via == "host":
            return st.calculate_partial_deps(workload.queries, workload.flags)
        import torch
        dev = torch.device("cuda", device)
        qdev, keep = device_queries(workload.queries, dev)
        res, stats = st.deps_batch_device(qdev, regions=(via == "regions"))
        torch.cuda.synchronize(dev)
        return st.device_result_to_host(res)
    finally:
        st.close()


def recover(workload, scan, device=0):
    """One BeginRecovery scan over every request of the workload (fresh store)."""
    st = DeviceCommandStore(device, workload.range_start_inclusive, 1, workload.slices)
    try:
        st.load(workload)
        return st.recovery_scan(workload.queries, scan)
    finally:
        st.close()


def levels_stats(s):
    d = stats_dict(s)
    d.update(n_levels=int(s.n_levels), n_edges=int(s.n_edges), n_launches=int(s.n_launches),
             packed=bool(s.n_deferred))
    return d


def levels(graph, device=0):
    """Apply levels of a waitingOn graph (model.Graph) on the GPU through ad_levels (K5).
    Returns (u32 levels per txn, stats dict)."""
    st = DeviceCommandStore(device)
    try:
        out = np.zeros(len(graph.kind), np.uint32)
        s = A.AdStats()
        soa = graph.soa()
        st._check(lib().ad_levels(st.h, C.byref(soa), out.ctypes.data, C.byref(s)))
        return out, levels_stats(s)
    finally:
        st.close()


def device_updates(u, dev):
    """Copy a CfkUpdates batch to device `dev`; returns (AdCfkUpdateSoa of device pointers, keepalive)."""
    import torch

    def to_dev(a):
        return torch.from_numpy(np.ascontiguousarray(a).view(np.int64 if a.dtype.itemsize == 8 else
                                                              np.int32 if a.dtype.itemsize == 4 else np.uint8)).to(dev)
    arrs = [u.keys, u.txn.msb, u.txn.lsb, u.txn.node, u.exec.msb, u.exec.lsb, u.exec.node, u.status]
    if u.ballot is not None:
        arrs += [u.ballot.msb, u.ballot.lsb, u.ballot.node]
    t = [to_dev(a) for a in arrs]
    s = A.AdCfkUpdateSoa()
    s.n = len(u)
    (s.keys, s.txn_msb, s.txn_lsb, s.txn_node, s.exec_msb, s.exec_lsb, s.exec_node, s.status) = [x.data_ptr() for x in t[:8]]
    if u.ballot is not None:
        s.ballot_msb, s.ballot_lsb, s.ballot_node = [x.data_ptr() for x in t[8:11]]
    if u.dep_off is not None:
        dt = [to_dev(a) for a in (u.dep_off, u.deps.msb, u.deps.lsb, u.deps.node)]
        t += dt
        s.dep_off, s.dep_msb, s.dep_lsb, s.dep_node = [x.data_ptr() for x in dt]
    return s, t


def device_graph(graph, dev):
    """Stage a Graph in HBM (torch tensors as allocator). Returns (AdGraphSoa of device pointers,
    dict of the tensors that must stay alive)."""
    import torch

    def to_dev(a):
        a = np.ascontiguousarray(a)
        if a.dtype == np.uint64:
            a = a.view(np.int64)
        if a.dtype == np.uint32:
            a = a.view(np.int32)
        return torch.from_numpy(a).to(dev)
    keep = {k: to_dev(v) for k, v in [("em", graph.exec.msb), ("el", graph.exec.lsb), ("en", graph.exec.node),
                                      ("kind", graph.kind), ("ko", graph.key_off), ("k", graph.keys)]}
    if graph.dep_off is not None:
        keep["do"] = to_dev(graph.dep_off)
        keep["d"] = to_dev(graph.deps)
    s = A.AdGraphSoa()
    s.n_txns = len(graph.kind)
    s.exec_msb, s.exec_lsb, s.exec_node = keep["em"].data_ptr(), keep["el"].data_ptr(), keep["en"].data_ptr()
    s.kind, s.key_off, s.keys = keep["kind"].data_ptr(), keep["ko"].data_ptr(), keep["k"].data_ptr()
    s.dep_off = keep["do"].data_ptr() if "do" in keep else None
    s.deps = keep["d"].data_ptr() if "d" in keep else None
    return s, keep


def guard_check():
    """AD_GUARD debug mode: (number of damaged device guard bands, report); (0, "") when the mode is off."""
    buf = C.create_string_buffer(1 << 16)
    bad = lib().ad_debug_guard_check(buf, len(buf))
    return bad, buf.value.decode(errors="replace")
