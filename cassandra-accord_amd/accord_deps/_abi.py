"""ctypes mirror of include/accord_deps.h (the C ABI of libaccord_deps.so).

Struct layouts only; loading the product library lives in ``native.py``. The oracle
wrapper (``oracle/pyoracle.py``) reuses these layouts because the oracle consumes the same
SoA formats.
"""
import ctypes as C

import numpy as np

AD_OK = 0
AD_E_INVAL = -1
AD_E_NOMEM = -2
AD_E_DEVICE = -3
AD_E_ORDER = -4
AD_E_DUP_EXEC = -5
AD_E_INCONSISTENT_ID = -6
AD_E_NOT_LOADED = -7
AD_E_STATE = -8
AD_E_CAPACITY = -9
AD_E_SPACE = -10
AD_E_PEER = -11
AD_E_PARTIAL = -12

AD_MAP_KEY, AD_MAP_RANGE, AD_MAP_DIRECT_KEY = 0, 1, 2
NMAPS = 3
MAP_NAMES = ("keyDeps", "rangeDeps", "directKeyDeps")
AD_SNAPSHOT, AD_SEQUENTIAL = 0, 1
AD_PARTS_ONLY = 2        # ad_deps_batch_device: result only exported as parts (no packed arrays)
AD_N_KEYS = 4            # ad_deps_batch_device: AdQuerySoa.n_keys = key_off[n_txns]
AD_REGIONS = 8           # ad_deps_batch_device: the result is read through its regions (no packed copy)

# InternalStatus ordinals (CommandsForKey.java:493-501)
ST_TRANSITIVELY_KNOWN = 0
ST_HISTORICAL = 1
ST_PREACCEPTED = 2
ST_ACCEPTED = 3
ST_COMMITTED = 4
ST_STABLE = 5
ST_APPLIED = 6
ST_INVALID = 7

# Txn.Kind ordinals (Txn.java:53-112)
KIND_READ, KIND_WRITE, KIND_EPHEMERAL_READ, KIND_SYNC_POINT, KIND_EXCLUSIVE_SYNC_POINT, KIND_LOCAL_ONLY = range(6)

P = C.c_void_p


class AdConfig(C.Structure):
    _fields_ = [("device", C.c_int32), ("range_start_inclusive", C.c_int32), ("elide", C.c_int32),
                ("path", C.c_int32), ("n_slices", C.c_uint64), ("slice_start", P), ("slice_end", P)]


class AdCfkSoa(C.Structure):
    _fields_ = [("n_keys", C.c_uint64), ("keys", P), ("seg", P), ("n_entries", C.c_uint64),
                ("txn_msb", P), ("txn_lsb", P), ("txn_node", P),
                ("exec_msb", P), ("exec_lsb", P), ("exec_node", P),
                ("status", P), ("pruned_before", P)]


class AdCfkUpdateSoa(C.Structure):
    _fields_ = [("n", C.c_uint64), ("keys", P), ("txn_msb", P), ("txn_lsb", P), ("txn_node", P),
                ("exec_msb", P), ("exec_lsb", P), ("exec_node", P), ("status", P),
                ("ballot_msb", P), ("ballot_lsb", P), ("ballot_node", P),
                ("dep_off", P), ("dep_msb", P), ("dep_lsb", P), ("dep_node", P)]


class AdCfkMissingSoa(C.Structure):
    _fields_ = [("n_entries", C.c_uint64), ("off", P), ("msb", P), ("lsb", P), ("node", P)]


# recovery scans (accord_deps.h ad_recovery_batch; BeginRecovery.java:329-380)
AD_RECOVER_STARTED_BEFORE_ACCEPTED_NO_WITNESS = 0
AD_RECOVER_STARTED_BEFORE_STABLE_WITNESS = 1
AD_RECOVER_STARTED_AFTER_ACCEPTED_NO_WITNESS = 2
AD_RECOVER_EXECUTES_AFTER_STABLE_NO_WITNESS = 3
RECOVER_SCANS = (0, 1, 2, 3)


class AdRangeCmdsSoa(C.Structure):
    _fields_ = [("n_cmds", C.c_uint64), ("txn_msb", P), ("txn_lsb", P), ("txn_node", P),
                ("erased", P), ("historical", P), ("range_off", P), ("range_start", P), ("range_end", P)]


AD_RS_PROPOSED, AD_RS_STABLE = 1, 2


class AdRangeCmdsRecoverySoa(C.Structure):
    _fields_ = [("n_cmds", C.c_uint64), ("status", P), ("has_deps", P), ("exec_msb", P), ("exec_lsb", P),
                ("exec_node", P), ("dep_off", P), ("dep_msb", P), ("dep_lsb", P), ("dep_node", P)]


class AdRedundantSoa(C.Structure):
    _fields_ = [("n", C.c_uint64), ("range_start", P), ("range_end", P), ("start_epoch", P), ("end_epoch", P),
                ("wm_msb", P), ("wm_lsb", P), ("wm_node", P)]


class AdQuerySoa(C.Structure):
    _fields_ = [("n_txns", C.c_uint64), ("txn_msb", P), ("txn_lsb", P), ("txn_node", P),
                ("exec_msb", P), ("exec_lsb", P), ("exec_node", P), ("min_epoch", P),
                ("key_off", P), ("keys", P), ("n_keys", C.c_uint64),
                ("range_off", P), ("range_start", P), ("range_end", P), ("n_ranges", C.c_uint64),
                ("slice_set", P)]


AD_SLICE_STORE = 0xFFFFFFFF


class AdStats(C.Structure):
    _fields_ = [("n_txns", C.c_uint64), ("n_probes", C.c_uint64), ("n_pairs", C.c_uint64 * NMAPS),
                ("n_unique", C.c_uint64 * NMAPS), ("n_keys", C.c_uint64 * NMAPS), ("scan_entries", C.c_uint64),
                ("ms_device", C.c_double), ("ms_ingest", C.c_double),
                ("ms_stage", C.c_double * 8), ("n_deferred", C.c_uint64), ("bytes_stage", C.c_uint64 * 8),
                ("n_levels", C.c_uint64), ("n_edges", C.c_uint64), ("n_launches", C.c_uint64),
                ("n_deferred_lean", C.c_uint64), ("n_lean_pass2", C.c_uint64),
                ("lean_rpw1", C.c_uint32), ("lean_flags", C.c_uint32)]


AD_LEAN_WIDE1, AD_LEAN_RANGES, AD_LEAN_PASS2 = 1, 2, 4


class AdDepsResult(C.Structure):
    _fields_ = [("n_txns", C.c_uint64),
                ("keys_off", P * NMAPS), ("keys", P * NMAPS),
                ("txn_off", P * NMAPS), ("txns", P * NMAPS),
                ("k2t_off", P * NMAPS), ("k2t", P * NMAPS),
                ("stats", AdStats),
                ("regions", P), ("region_off", P * NMAPS), ("regions_bytes", C.c_uint64), ("region_bytes", C.c_uint64)]


class AdGraphSoa(C.Structure):
    _fields_ = [("n_txns", C.c_uint64), ("exec_msb", P), ("exec_lsb", P), ("exec_node", P), ("kind", P),
                ("key_off", P), ("keys", P), ("dep_off", P), ("deps", P)]


class AdRangeMapSoa(C.Structure):
    _fields_ = [("n_values", C.c_uint64), ("starts", P), ("msb", P), ("lsb", P), ("node", P), ("present", P),
                ("inclusive_ends", C.c_uint32)]


AD_PA_FAST, AD_PA_REJECTED, AD_PA_ESP = 1, 2, 4


class AdParts(C.Structure):
    _fields_ = [("n_parts", C.c_uint64), ("n_key_words", C.c_uint64), ("n_ids", C.c_uint64), ("n_k2t", C.c_uint64),
                ("hdr", P), ("keys", P), ("ids", P), ("k2t", P),
                ("cap_parts", C.c_uint64), ("cap_key_words", C.c_uint64), ("cap_ids", C.c_uint64),
                ("cap_k2t", C.c_uint64), ("id_format", C.c_uint32)]


AD_IDS_TRIPLET = 0
AD_IDS_RANK = 1

# exchange table / plan (accord_deps.h, ad_exchange_plan)
AD_XROW_HDR = 12
AD_XROW_MAGIC = 0x41445852
AD_XPLAN_GROW = 1


def xrow_words(world):
    return 4 * world + AD_XROW_HDR


class AdXfer(C.Structure):
    _fields_ = [("send_off", C.c_uint64), ("send_bytes", C.c_uint64), ("recv_off", C.c_uint64),
                ("recv_bytes", C.c_uint64)]


class AdMerged(C.Structure):
    _fields_ = [("n_txns", C.c_uint64), ("txn_base", C.c_uint64),
                ("keys_off", P * NMAPS), ("keys", P * NMAPS),
                ("txn_off", P * NMAPS), ("txns", P * NMAPS),
                ("k2t_off", P * NMAPS), ("k2t", P * NMAPS),
                ("n_keys", C.c_uint64 * NMAPS), ("n_ids", C.c_uint64 * NMAPS), ("n_k2t", C.c_uint64 * NMAPS),
                ("ms_device", C.c_double), ("id_format", C.c_uint32)]


class AdExchangeStats(C.Structure):
    _fields_ = [("bytes_moved", C.c_uint64), ("ms_export", C.c_double), ("ms_move", C.c_double),
                ("ms_merge", C.c_double), ("ms_total", C.c_double)]


AD_COMM_ID_BYTES = 128


def ptr(a):
    """Pointer to a numpy array's data (None for None). Caller keeps the array alive."""
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"], "arrays handed to the ABI must be C-contiguous"
    return a.ctypes.data  # numpy allocates >= 1 byte, so empty arrays still get a valid pointer


def as_u64(a):
    return np.ascontiguousarray(a, dtype=np.uint64)


def as_i64(a):
    return np.ascontiguousarray(a, dtype=np.int64)


def as_i32(a):
    return np.ascontiguousarray(a, dtype=np.int32)


def as_u8(a):
    return np.ascontiguousarray(a, dtype=np.uint8)


def as_u32(a):
    return np.ascontiguousarray(a, dtype=np.uint32)
