/*
 * accord_deps.h — C ABI of the MI355X-native batched dependency-resolution engine
 * for Accord's PreAccept/Accept path (libaccord_deps.so).
 *
 * The library replaces, for one CommandStore (one GPU = one token-range slice):
 *
 *   SafeCommandStore.mapReduceActive(keys, slice, startedBefore, kinds, map, p1, acc)
 *       accord-core/src/main/java/accord/local/SafeCommandStore.java:292
 *     as implemented by InMemorySafeStore.mapReduceActive
 *       accord-core/src/main/java/accord/impl/InMemoryCommandStore.java:863-871
 *     -> CommandsForKey.mapReduceActive   (local/cfk/CommandsForKey.java:910-968)
 *     -> mapReduceRangesInternal           (impl/InMemoryCommandStore.java:884-1017)
 *   composed by PreAccept.calculatePartialDeps (messages/PreAccept.java:245-267)
 *     (also reached from Accept.calculatePartialDeps, messages/Accept.java:113-117)
 *     -> Deps.AbstractBuilder.add         (primitives/Deps.java:80-106)
 *     -> RelationMultiMap.AbstractBuilder (utils/RelationMultiMap.java:88-260)
 *     -> RedundantBefore.collectDeps      (local/RedundantBefore.java:183-192,420-423)
 *     -> PartialDeps.with / linearUnion   (primitives/PartialDeps.java:73-81,
 *                                          utils/RelationMultiMap.java:561-816)
 *
 * Instead of one callback per (key, txnId), a whole batch of calculatePartialDeps
 * requests is resolved per call, and the results come back already in the CSR form
 * that KeyDeps.SerializerSupport.create(Keys, TxnId[], int[]) (primitives/KeyDeps.java:69-72)
 * and RangeDeps.SerializerSupport.create(Range[], TxnId[], int[]) (primitives/RangeDeps.java:100-103)
 * wrap without a rebuild.
 *
 * Conventions
 *  - TxnId / Timestamp travel as structure-of-arrays {msb u64, lsb u64, node i32}, the exact
 *    fields of accord.primitives.Timestamp (Timestamp.java:77-79) and Node.Id.id (Node.java:104-137).
 *    Order is Timestamp.compareTo (Timestamp.java:208-217); identity is Timestamp.equals
 *    (Timestamp.java:244-249, mask 0xFFFFFFFFFFFF001E). Two ids equal under that identity
 *    must be bit-identical (checked; AD_E_INCONSISTENT_ID).
 *  - Keys and range bounds travel as order-preserving int64 ordinals (Key.compareTo ==
 *    signed int64 compare). Ranges are EndInclusive (s,e] unless ad_config.range_start_inclusive.
 *  - Inputs are caller-owned and only read during the call. Results are library-owned
 *    until ad_result_free (host variant) or the next batch call (device variant).
 *  - One ad_ctx per CommandStore / per GPU; a ctx is not thread-safe (the reference's
 *    SafeCommandStore is single-threaded, SafeCommandStore.java:52-57).
 *  - Every entry point returns AD_OK (0) or a negative AD_E_* code; ad_last_error(ctx)
 *    gives the message (the Java wrapper maps it to IllegalStateException).
 */
#ifndef ACCORD_DEPS_H
#define ACCORD_DEPS_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AD_ABI_VERSION 6

/* ---- status codes ---------------------------------------------------------------- */
#define AD_OK                  0
#define AD_E_INVAL            -1  /* malformed input (unsorted keys, bad kind, ...)        */
#define AD_E_NOMEM            -2  /* host or device allocation failed                      */
#define AD_E_DEVICE           -3  /* HIP runtime error                                      */
#define AD_E_ORDER            -4  /* byId not strictly increasing (CommandsForKey.java:1438)*/
#define AD_E_DUP_EXEC         -5  /* duplicate executeAt among committed (CommandsForKey.java:1439) */
#define AD_E_INCONSISTENT_ID  -6  /* equal ids with different bits                          */
#define AD_E_NOT_LOADED       -7  /* batch before ad_cfk_load                               */
#define AD_E_STATE            -8  /* reference would throw (e.g. prunedBefore walk off end) */
#define AD_E_CAPACITY         -9  /* id dictionary exceeds 2^28 entries                     */
#define AD_E_SPACE           -10  /* a caller-provided output buffer is too small (sizes set) */
#define AD_E_PEER            -11  /* another rank of an exchange step reported a failure     */
#define AD_E_PARTIAL         -12  /* ad_cfk_update: the explicit updates were applied, what follows
                                   * them (deps-derived additions, missing() lists) was not -- see
                                   * ad_cfk_update_status                                      */

/* ---- InternalStatus ordinals (CommandsForKey.java:493-501) -------------------------- */
#define AD_ST_TRANSITIVELY_KNOWN                          0
#define AD_ST_HISTORICAL                                  1
#define AD_ST_PREACCEPTED_OR_ACCEPTED_INVALIDATE          2
#define AD_ST_ACCEPTED                                    3
#define AD_ST_COMMITTED                                   4
#define AD_ST_STABLE                                      5
#define AD_ST_APPLIED                                     6
#define AD_ST_INVALID_OR_TRUNCATED_OR_UNMANAGED_COMMITTED 7

/* ---- Txn.Kind ordinals (Txn.java:53-112); kind = (lsb >> 1) & 7, domain = lsb & 1 --- */
#define AD_KIND_READ                 0
#define AD_KIND_WRITE                1
#define AD_KIND_EPHEMERAL_READ       2
#define AD_KIND_SYNC_POINT           3
#define AD_KIND_EXCLUSIVE_SYNC_POINT 4
#define AD_KIND_LOCAL_ONLY           5

/* ---- result maps (Deps.java:59-119: keyDeps, rangeDeps, directKeyDeps) --------------- */
#define AD_MAP_KEY        0
#define AD_MAP_RANGE      1
#define AD_MAP_DIRECT_KEY 2
#define AD_NMAPS          3

/* ---- batch flags ------------------------------------------------------------------- */
/* SNAPSHOT: every request reads the same immutable snapshot (GetDeps / non-participating
 *           Accept, Accept.java:87-94).
 * SEQUENTIAL: requests are applied in the given order; before request i's deps are computed
 *           its txnId is inserted into each of its keys' CommandsForKey as
 *           PREACCEPTED_OR_ACCEPTED_INVALIDATE (PreAccept.apply: Commands.preaccept precedes
 *           calculatePartialDeps, PreAccept.java:116-132; CommandsForKey.update :972-1042).
 *           The inserted entries stay in the ctx snapshot afterwards, as they do in the CFK. */
#define AD_SNAPSHOT   0u
#define AD_SEQUENTIAL 1u
/* ad_deps_batch_device only: the caller exports the result as parts (ad_parts_export) and does
 * not read the packed arrays; they are not produced (keys/txns/k2t NULL, offsets valid) and the
 * export reads the per-request regions of the batch directly. */
#define AD_PARTS_ONLY 2u
/* ad_deps_batch_device only: ad_query_soa.n_keys holds key_off[n_txns] */
#define AD_N_KEYS     4u
/* ad_deps_batch_device only: the result is read through its regions (ad_deps_result.regions,
 * region_off): each request's three RelationMultiMaps stay where the kernels wrote them, once, and
 * the packed arrays are not produced (keys/txns/k2t NULL; the *_off arrays still give every
 * request's sizes and its position in a packed layout). This is the device path's primary output: a
 * Java host builds each request's KeyDeps / RangeDeps from its own region. */
#define AD_REGIONS    8u

typedef struct ad_config {
    int32_t device;                 /* HIP device ordinal                                   */
    int32_t range_start_inclusive;  /* 0: Range.EndInclusive (s,e]; 1: StartInclusive [s,e) */
    int32_t elide;                  /* CommandsForKey.ELIDE_TRANSITIVE_DEPENDENCIES (:173), 1 */
    int32_t path;                   /* 0: fused per-request kernel, split kernels for the rest
                                     * (default); 1: split kernels only (testing)            */
    /* the store's owned ranges (SafeCommandStore.ranges(); slice in mapReduceForKey,
     * InMemoryCommandStore.java:280). n_slices == 0 means "owns every key". */
    uint64_t n_slices;
    const int64_t* slice_start;
    const int64_t* slice_end;
} ad_config;

/* CommandsForKey snapshots of the store, in the shape of
 * CommandsForKey.SerializerSupport.create(Key, TxnInfo[] byId, Unmanaged[], TxnId prunedBefore)
 * (CommandsForKey.java:226-232). Entries of key k are [seg[k], seg[k+1]) in byId order. */
typedef struct ad_cfk_soa {
    uint64_t n_keys;
    const int64_t*  keys;            /* [n_keys] strictly ascending                         */
    const uint64_t* seg;             /* [n_keys+1]                                          */
    uint64_t n_entries;
    const uint64_t* txn_msb;         /* TxnInfo (a TxnId)                                   */
    const uint64_t* txn_lsb;
    const int32_t*  txn_node;
    const uint64_t* exec_msb;        /* TxnInfo.executeAt (== txnId unless hasExecuteAt)    */
    const uint64_t* exec_lsb;
    const int32_t*  exec_node;
    const uint8_t*  status;          /* AD_ST_*                                             */
    const int64_t*  pruned_before;   /* [n_keys] index within the key's byId of prunedBefore, -1 = NONE; NULL = none */
} ad_cfk_soa;

/* Range-domain commands registered with the store (InMemoryCommandStore.rangeCommands and
 * historicalRangeCommands, :103-104,740-763,797-830); their ranges are already sliced to
 * the store as in InMemoryCommandStore.java:758-761. */
typedef struct ad_range_cmds_soa {
    uint64_t n_cmds;
    const uint64_t* txn_msb;
    const uint64_t* txn_lsb;
    const int32_t*  txn_node;
    const uint8_t*  erased;          /* 1: saveStatus >= Erased (skipped, :897); NULL = none  */
    const uint8_t*  historical;      /* 1: historicalRangeCommands entry; NULL = none        */
    const uint64_t* range_off;       /* [n_cmds+1]                                          */
    const int64_t*  range_start;
    const int64_t*  range_end;
} ad_range_cmds_soa;

/* RedundantBefore entries (RedundantBefore.java:59-120); disjoint ranges. */
typedef struct ad_redundant_soa {
    uint64_t n;
    const int64_t*  range_start;
    const int64_t*  range_end;
    const int64_t*  start_epoch;     /* inclusive */
    const int64_t*  end_epoch;       /* exclusive */
    const uint64_t* wm_msb;          /* shardAppliedOrInvalidatedBefore */
    const uint64_t* wm_lsb;
    const int32_t*  wm_node;
} ad_redundant_soa;

/* A batch of calculatePartialDeps(safeStore, txnId, keys, ..., minEpoch, executeAt, ranges)
 * requests (PreAccept.java:245). Keys of request i: keys[key_off[i] .. key_off[i+1]),
 * strictly ascending (accord.primitives.Keys). */
typedef struct ad_query_soa {
    uint64_t n_txns;
    const uint64_t* txn_msb;
    const uint64_t* txn_lsb;
    const int32_t*  txn_node;
    const uint64_t* exec_msb;        /* executeAt: == txnId for PreAccept, proposed for Accept */
    const uint64_t* exec_lsb;
    const int32_t*  exec_node;
    const int64_t*  min_epoch;       /* minUnsyncedEpoch (RedundantBefore bounds); NULL = 0  */
    const uint64_t* key_off;         /* [n_txns+1] */
    const int64_t*  keys;
    uint64_t        n_keys;          /* key_off[n_txns], read only under AD_N_KEYS (a device batch
                                      * then needs no device-to-host read before its first kernel) */
    /* Range-domain requests (a txn whose Seekables are Ranges: sync points, range reads and writes;
     * SafeCommandStore.mapReduceActive takes Seekables, SafeCommandStore.java:292). NULL range_off:
     * every request is key-domain. Otherwise request i has the ranges
     * [range_start[j], range_end[j]) j in [range_off[i], range_off[i+1]) -- Ranges normalised as
     * accord.primitives.Ranges is: start < end, ascending, disjoint (end[j] <= start[j+1]), with the
     * store's inclusivity (ad_config.range_start_inclusive) -- and then no keys (a request has keys or
     * ranges, never both). For such a request the store visits every CommandsForKey whose key lies in
     * the ranges sliced to the store's slices (InMemoryCommandStore.mapReduceForKey, case Range,
     * :289-304), every range command with a range intersecting those sliced ranges
     * (mapReduceRangesInternal, :884-1017) and the RedundantBefore entries intersecting the request's
     * (unsliced) ranges (RedundantBefore.collectDeps, RedundantBefore.java:420-423). In an AD_SEQUENTIAL
     * batch such a request first registers as a range command (PreAccept.apply, PreAccept.java:116-132;
     * InMemoryCommandStore.java:740-763): its ranges sliced to the store, less those of the
     * RedundantBefore entries that make it shard-redundant (RedundantBefore.java:216-225), seen by every
     * later request of the batch and kept by the store (a txnId already among the range commands:
     * AD_E_INVAL). ad_recovery_batch takes them too (a recovering sync point or range txn). */
    const uint64_t* range_off;       /* [n_txns+1] or NULL */
    const int64_t*  range_start;
    const int64_t*  range_end;
    uint64_t        n_ranges;        /* range_off[n_txns], read only under AD_N_KEYS */
    /* The slice of each request's scan (SafeCommandStore.mapReduceActive's `slice`, SafeCommandStore.java:292) when
     * it is not the store's own: PreAccept (PreAccept.java:100,130), Accept (Accept.java:115), GetDeps and
     * GetEphemeralReadDeps (GetDeps.java:75, GetEphemeralReadDeps.java:75) slice to
     * safeStore.ranges().allBetween(minUnsyncedEpoch, txnId | executeAt) (RangesForEpoch.allBetween,
     * CommandStores.java:233-242), which differs between the requests of one batch during a topology change.
     * slice_set[i] is an index into the store's slice sets (ad_slice_sets_load), or AD_SLICE_STORE for the
     * store's own slices (ad_config.slice_*). NULL: every request reads the store's slices. It slices the keys a
     * request scans (mapReduceForKey, InMemoryCommandStore.java:280), a Range-domain request's ranges (:289-304) and
     * the range commands' fold (:887,951-961); RedundantBefore stays unsliced (RedundantBefore.java:420-423), and the
     * registration of a SEQUENTIAL batch's insertions keeps the store's slices. An index beyond the loaded sets:
     * AD_E_INVAL. ad_deps_batch_device / ad_recovery_batch_device: a device array. */
    const uint32_t* slice_set;
} ad_query_soa;
#define AD_SLICE_STORE 0xFFFFFFFFu

typedef struct ad_stats {
    uint64_t n_txns, n_probes;
    uint64_t n_pairs[AD_NMAPS];      /* txn-key (or txn-range) pairs emitted per map         */
    uint64_t n_unique[AD_NMAPS];     /* sum over txns of unique txnIds per map               */
    uint64_t n_keys[AD_NMAPS];       /* sum over txns of keys (ranges) with >= 1 dep per map  */
    uint64_t scan_entries;           /* CFK entries a reference scan would visit (sum of end) */
    double   ms_device;              /* device time of the resolve pipeline                  */
    double   ms_ingest;
    /* per-stage device time (HIP events): 0 encode (K0), 1 conflict scan (K1), 2 range probe
     * (K4), 3 build sizing (K2 pass 1), 4 offsets scan, 5 build emit (K2 pass 2) */
    double   ms_stage[8];            /* path 0: 0 fused resolve, 1 deferred requests (split),
                                      * 5 offsets + pack; with AD_STAGE_EVENTS=1 in the environment
                                      * the resolve is split further: 2 k_prepare, 0 lean pass 1,
                                      * 3 lean pass 2, 6 general kernel (three more event records,
                                      * ~4 us of idle GPU each, so off by default) */
    uint64_t n_deferred;             /* requests resolved by the split kernels (path 0);
                                      * ad_levels: 1 when the packed path ran (keys-only sorts,
                                      * predecessor records), 0 for the CSR path               */
    uint64_t bytes_stage[8];         /* algorithmic bytes per stage            */
    /* ad_levels: n_txns, n_probes = txn-key occurrences, ms_stage[0] build (exec ranking, key
     * chains, successor CSR), ms_stage[1] frontier loop, and: */
    uint64_t n_levels;               /* 1 + max level                                         */
    uint64_t n_edges;                /* edges of the sparsified waitingOn DAG                  */
    uint64_t n_launches;             /* frontier-step launches; ad_deps_batch*: 1 when lean pass 1
                                      * ran its wide kernel (up to 64 raw emissions per request) */
    uint64_t n_deferred_lean;        /* ad_deps_batch*: requests the lean passes handed to the general kernel */
    uint64_t n_lean_pass2;           /* ad_deps_batch*: requests lean pass 1 handed to lean pass 2     */
    /* ad_deps_batch*: which lean kernels ran (so a profile can be matched to the batch exactly):
     * requests per wave of lean pass 1 (0: the lean passes did not run) and AD_LEAN_* flags */
    uint32_t lean_rpw1;
    uint32_t lean_flags;
} ad_stats;
#define AD_LEAN_WIDE1  1u   /* lean pass 1 ran its wide kernel (up to 64 raw emissions per request)     */
#define AD_LEAN_RANGES 2u   /* the lean kernels' range-command instantiation (store with range commands) */
#define AD_LEAN_PASS2  4u   /* lean pass 2 was launched                                                 */

/* Results, one CSR triple per map and request, packed in request order.
 * For request i and map m:
 *   keys      [keys_off[m][i]  .. keys_off[m][i+1])   key ordinals (m = KEY/DIRECT_KEY) or
 *                                                       range ids into ad_range_table (m = RANGE)
 *   txnIds    [txn_off[m][i]   .. txn_off[m][i+1])    indices into ad_dict (ascending == sorted TxnIds)
 *   k2t       [k2t_off[m][i]   .. k2t_off[m][i+1])    the exact int[] keysToTxnIds of
 *             RelationMultiMap (RelationMultiMap.java:245-257): nKeys absolute end offsets
 *             starting at nKeys, then the value indices of each key in ascending order. */
typedef struct ad_deps_result {
    uint64_t  n_txns;
    uint64_t* keys_off[AD_NMAPS];
    int64_t*  keys[AD_NMAPS];
    uint64_t* txn_off[AD_NMAPS];
    uint32_t* txns[AD_NMAPS];
    uint64_t* k2t_off[AD_NMAPS];
    int32_t*  k2t[AD_NMAPS];
    ad_stats  stats;
    /* Regions (ad_deps_batch_device; every result, AD_REGIONS or not): request i's map m, when it has
     * nK = keys_off[m][i+1] - keys_off[m][i] > 0 keys, is the 8-byte aligned block at byte offset
     * region_off[m][i] of `regions`:
     *     int64 keys[nK] | uint32 txnIds[nT] | int32 keysToTxnIds[nKT]
     * with nT, nKT the differences of txn_off / k2t_off -- the three arrays of that map as above.
     * region_off of an empty map is unspecified. regions_bytes: bytes of `regions` in use (the regions
     * plus the unused tails of the kernels' allocation chunks); region_bytes: the payload of the regions
     * (their three arrays, alignment padding excluded). */
    const uint8_t*  regions;
    const uint64_t* region_off[AD_NMAPS];
    uint64_t        regions_bytes;
    uint64_t        region_bytes;
} ad_deps_result;

typedef struct ad_ctx ad_ctx;

/* ---- lifecycle ---------------------------------------------------------------------- */
int  ad_abi_version(void);
int  ad_ctx_create(const ad_config* cfg, ad_ctx** out);
void ad_ctx_destroy(ad_ctx* ctx);
const char* ad_last_error(const ad_ctx* ctx);

/* ---- snapshot upload (ingest; builds the id dictionary, ranks and device indexes) ---- */
int ad_cfk_load(ad_ctx* ctx, const ad_cfk_soa* cfk);
int ad_range_cmds_load(ad_ctx* ctx, const ad_range_cmds_soa* cmds);
/* The registry's upkeep as the store applies it, command by command, without a snapshot rebuild: each row of
 * `upd`, in order (the same SoA as the load; its flags say what the row is):
 *   historical[i] = 1: registerHistoricalTransactions -- historicalRangeCommands.merge(txnId, ranges, Ranges::with)
 *                      (InMemoryCommandStore.java:814-828); nothing when txnId is a live range command;
 *   erased[i] = 1:     the live command's status became Erased (InMemorySafeStore.update returns early, the scan
 *                      skips it, :748-749,892); nothing when the txnId is not registered;
 *   otherwise:         InMemorySafeStore.update (:740-763): rangeCommands.computeIfAbsent(txnId).update(ranges) --
 *                      registered when absent, else its Ranges united with these (RangeCommand.update :547-551,
 *                      Ranges.with = AbstractRanges.union(MERGE_OVERLAPPING), AbstractRanges.java:486-574).
 * Ranges are the host's `keysOrRanges.slice(allBetween(txnId, executeAtOrTxnId))` less the shard-redundant ones
 * (:758-761), normalised. New commands take the next load indices (ad_range_cmds_recovery_load then describes
 * the registry in that order; its facts are dropped by every update). New txnIds join the id dictionary on the
 * device; the range part of the snapshot (range entries, stabbing cells, range trees, KeyLines) is rebuilt from
 * the registry while the CommandsForKeys stay. stats (may be NULL): ms_stage[0] registry upkeep (host),
 * ms_stage[1] range part refresh, n_keys[0] commands registered, n_keys[1] range entries, n_keys[2] ids added. */
int ad_range_cmds_update(ad_ctx* ctx, const ad_range_cmds_soa* upd, ad_stats* stats);
int ad_redundant_load(ad_ctx* ctx, const ad_redundant_soa* rb);
/* Every read of the store sees its CommandsForKeys truncated to the RedundantBefore: the snapshot is
 * truncated on the device when it is built (SafeCommandStore.maybeTruncate, SafeCommandStore.java:165-171
 * -> CommandsForKey.withRedundantBeforeAtLeast, CommandsForKey.java:1317-1341): byId below the key's
 * shardRedundantBefore leaves, the missing() lists of the rest lose the ids below it, a prunedBefore at or
 * below it becomes NO_INFO. SEQUENTIAL PreAccepts below it register nothing (CommandsForKey.java:997);
 * ad_cfk_update leaves that filter to the caller.
 *
 * ad_redundant_advance: the store's RedundantBefore moves forward in place, without a snapshot rebuild
 * (RedundantBefore.merge as the store's GC advances it, CommandStore.upsertRedundantBefore). rb names the
 * same entries (ranges) as the loaded RedundantBefore, in the same order, with epochs and watermarks that
 * may change: each watermark at or above the loaded one (AD_E_INVAL otherwise, as
 * CommandsForKey.java:1319's Invariants.checkArgument). New watermarks join the id dictionary on the
 * device and every CommandsForKey whose watermark moved is truncated on the device (its missing() lists
 * too, wherever they are held). A change of ranges is an ad_redundant_load. stats (may be NULL):
 * ms_device = device time of the truncation, ms_stage[0] = the watermarks' dictionary growth (host-timed), n_keys[0]
 * = entries removed, n_keys[1] = CommandsForKeys changed, n_keys[2] = ids added to the dictionary. */
int ad_redundant_advance(ad_ctx* ctx, const ad_redundant_soa* rb, ad_stats* stats);
/* Build the id dictionary and device indexes of the loaded snapshot now (otherwise the first
 * batch does it). Ingest time is reported in ad_stats.ms_ingest, never in ms_device. */
int ad_prepare(ad_ctx* ctx);

/* The store's slice sets (ad_query_soa.slice_set): set k is the Ranges [start[j], end[j]) for j in
 * [set_off[k], set_off[k+1]) -- normalised as accord.primitives.Ranges (start < end, ascending, disjoint), in the
 * store's inclusivity; an empty set owns no key. A host binding loads the distinct RangesForEpoch.allBetween results
 * its batch needs (CommandStores.java:233-242). Host arrays, copied; replaces the previous sets
 * (no rebuild of the snapshot). n_sets == 0 removes them. */
int ad_slice_sets_load(ad_ctx* ctx, uint32_t n_sets, const uint64_t* set_off, const int64_t* start, const int64_t* end);

/* ---- batch resolve, host buffers in / host result out ------------------------------ */
int  ad_deps_batch(ad_ctx* ctx, const ad_query_soa* q, uint32_t flags, ad_deps_result** out);
void ad_result_free(ad_deps_result* r);

/* Pin caller-owned host memory for DMA (hipHostRegister): a Panama Arena segment a Java host reuses
 * batch after batch for queries and results. Unregister before freeing it. Pinning is page-granular:
 * register whole pages the caller owns (page-aligned p, bytes a multiple of the page size, e.g. an Arena
 * allocation with 4096-byte alignment); a sub-page range shares its pages with unrelated memory, which
 * its unregistration would unpin under any transfer still using them. ad_host_unregister accepts a
 * NULL ctx (a registration is process-wide): a finalizer can unpin memory whose ctx is already gone. */
int ad_host_register(ad_ctx* ctx, void* p, uint64_t bytes);
int ad_host_unregister(ad_ctx* ctx, void* p);
/* Pinned host memory allocated by the library (hipHostMalloc, portable, page-aligned): the preferred home
 * of a caller's reusable query / result arrays -- no registration of the caller's own pages. *p is set
 * (NULL on failure: AD_E_NOMEM). ad_host_free waits for the device before releasing the pages. Whatever
 * the caller passes that is neither (pageable memory) is bounced through the library's own pinned
 * staging, never handed to a pageable HIP copy. */
int ad_host_alloc(uint64_t bytes, void** p);
int ad_host_free(void* p);

/* Debug (AD_GUARD=1 or 2 in the environment): device allocations carry guard bands; returns the number
 * of damaged bands found among live allocations and those freed since the last call (0: none, or the
 * mode is off) and writes a description into buf (up to n bytes, NUL-terminated). */
int ad_debug_guard_check(char* buf, uint64_t n);

/* ad_deps_batch into caller-owned host arrays (the PCIe-facing path a Java host binds): `out`'s array
 * pointers are the caller's -- per map keys_off / txn_off / k2t_off with n_txns + 1 entries each, and
 * keys / txns / k2t with capacities cap[3 m + {0, 1, 2}] (elements); ideally pinned
 * (ad_host_alloc, or ad_host_register), so that every copy is a DMA straight into them (pageable arrays
 * are filled through the library's staging, synchronously). Same results as ad_deps_batch. The batch is resolved
 * in `slices` slices of requests (0: one per 128k requests, at most 8 for key-only SNAPSHOT batches and
 * 4 otherwise; SEQUENTIAL batches run whole): slice j's result is copied out while slice j + 1 is staged
 * and resolved into a second result bank. Key-only SNAPSHOT batches: the library's host threads pack
 * each slice's inputs into pinned staging (checking the keys in the same pass) while the previous slice
 * resolves, and a kernel writes the results straight into pinned output arrays over PCIe, beside the
 * next slice's host-to-device copy. need[9] receives the sizes the batch needed; when a capacity was too
 * small the call returns AD_E_SPACE and can be repeated with larger arrays. On any error return the
 * output arrays' contents are unspecified (slices before the failing one may have been written).
 * out->stats sums the slices' device stats. */
int ad_deps_batch_into(ad_ctx* ctx, const ad_query_soa* q, uint32_t flags, ad_deps_result* out, const uint64_t* cap /*[9]*/,
                       uint64_t* need /*[9]*/, uint32_t slices);

/* ---- batch resolve, device-resident (HBM) buffers in and out ----------------------- *
 * q's arrays are device pointers. *out receives device pointers owned by ctx, valid until
 * the next batch call on ctx; out->stats is filled after the call returns. All work is
 * enqueued on `stream` (a hipStream_t; NULL = the ctx stream) and completes before return.
 * Only AD_SNAPSHOT is supported here. */
int ad_deps_batch_device(ad_ctx* ctx, const ad_query_soa* q_dev, uint32_t flags, void* stream,
                         ad_deps_result* out);

/* ---- id dictionary / range table views (host copies owned by ctx) ------------------- */
int ad_dict(const ad_ctx* ctx, uint64_t* n, const uint64_t** msb, const uint64_t** lsb,
            const int32_t** node);
int ad_range_table(const ad_ctx* ctx, uint64_t* n, const int64_t** start, const int64_t** end);

/* ---- multi-GPU exchange ------------------------------------------------
 * One ctx per GPU = one CommandStore owning a token slice (ad_config.slice_*). A request that
 * touches several stores is resolved by each of them (CommandStores.mapReduce,
 * CommandStores.java:576-593); the per-store PartialDeps are combined with PartialDeps.with
 * (PartialDeps.java:73-81; PreAccept.reduce, PreAccept.java:140-156) on the GPU that owns the
 * request. The partials travel between GPUs (RCCL all-to-all) in this flat format.
 *
 * Parts: the non-empty maps of one store's batch result, in request order, maps ascending.
 *   hdr  [n_parts * 4] int64: {global request index << 2 | map, n_keys, n_ids, n_k2t}
 *   keys [n_key_words] int64: key ordinals; AD_MAP_RANGE: {start, end} per range (2 words)
 *   ids  [n_ids * 3]   int64: {msb, lsb, node} of each TxnId (ascending within a part)
 *   k2t  [n_k2t]       int32: the part's keysToTxnIds (indices into its own ids)
 * All arrays are device memory. */
typedef struct ad_parts {
    uint64_t n_parts, n_key_words, n_ids, n_k2t;          /* sizes                             */
    int64_t* hdr;
    int64_t* keys;
    int64_t* ids;
    int32_t* k2t;
    uint64_t cap_parts, cap_key_words, cap_ids, cap_k2t;  /* capacities of the arrays (export) */
    uint32_t id_format;   /* AD_IDS_TRIPLET: ids as above; AD_IDS_RANK: ids holds n_ids uint32 ranks
                           * into the global dictionary (ad_set_global_dict). Chosen by the caller of
                           * ad_parts_export (the format its ids buffer was sized for; RANK without an
                           * installed global dictionary covering the store: AD_E_STATE), read by
                           * ad_parts_merge. cap_ids counts ids in that format. */
} ad_parts;

#define AD_IDS_TRIPLET 0
#define AD_IDS_RANK    1

/* Global TxnId dictionary of a multi-store node: the ascending, duplicate-free union (Timestamp
 * order) of the dictionaries (ad_dict) of every store taking part in the exchange, built once per
 * snapshot (ingest time, not batch time). Host arrays. The store's snapshot is (re)built over this
 * dictionary: ad_dict then returns it and the txnIds of every result index into it, so the ids the
 * kernels emit are node-wide ranks. Every id of the snapshot must occur in it (AD_E_INVAL otherwise,
 * and the dictionary is not installed). Call it after the ad_*_load calls, before ad_prepare, to
 * build the snapshot once. While installed, ad_parts_export writes ids as those uint32 ranks
 * (AD_IDS_RANK: 4 bytes on the wire instead of 24, no translation) and ad_parts_merge merges
 * integer ranks. Loading a new snapshot, or an ad_cfk_update that adds ids, uninstalls it. */
int ad_set_global_dict(ad_ctx* ctx, uint64_t n, const uint64_t* msb, const uint64_t* lsb, const int32_t* node);

/* Export the device result `res_dev` of the last ad_deps_batch_device on ctx as parts, into
 * the caller's device arrays of `out` (capacities cap_*). txn_index_dev[i] is request i's
 * global index (ascending). Requests [dest_first[d], dest_first[d+1]) go to destination d
 * (host array, n_dest + 1 entries, dest_first[n_dest] == batch size); dest_counts (host,
 * n_dest * 4) receives per destination {parts, key words, ids, k2t}. If a capacity is too
 * small, the sizes are set in `out` and AD_E_SPACE is returned with nothing written. */
int ad_parts_export(ad_ctx* ctx, const ad_deps_result* res_dev, const int64_t* txn_index_dev, uint32_t n_dest,
                    const uint64_t* dest_first, void* stream, ad_parts* out, uint64_t* dest_counts);

/* Merged PartialDeps of the requests a GPU owns (ids as {msb,lsb,node}, or as global ranks, id_format).
 * For owned request r (global index txn_base + r) and map m: keys [keys_off[m][r], keys_off[m][r+1])
 * (AD_MAP_RANGE: ranges, 2 words each in keys[m]), txns [txn_off[m][r], ..) as triplets,
 * k2t [k2t_off[m][r], ..) the keysToTxnIds of the merged RelationMultiMap. Device memory owned
 * by ctx, valid until the next ad_parts_merge on ctx. */
typedef struct ad_merged {
    uint64_t  n_txns;
    uint64_t  txn_base;
    uint64_t* keys_off[AD_NMAPS];
    int64_t*  keys[AD_NMAPS];
    uint64_t* txn_off[AD_NMAPS];
    int64_t*  txns[AD_NMAPS];
    uint64_t* k2t_off[AD_NMAPS];
    int32_t*  k2t[AD_NMAPS];
    uint64_t  n_keys[AD_NMAPS], n_ids[AD_NMAPS], n_k2t[AD_NMAPS];   /* totals per map           */
    double    ms_device;
    uint32_t  id_format;   /* AD_IDS_TRIPLET: txns as {msb,lsb,node} int64 triplets; AD_IDS_RANK (merges of
                            * rank-format parts): txns[m] holds n_ids[m] uint32 ranks into the global
                            * dictionary the caller installed (ad_set_global_dict), ascending per request */
} ad_merged;

/* Merge the parts received from n_src stores (concatenated in source = slice order; source s
 * sent src_parts[s] parts) for the requests [txn_base, txn_base + n_owned). Keys of different
 * stores must be disjoint and ascending in source order (AD_E_INVAL otherwise). */
int ad_parts_merge(ad_ctx* ctx, const ad_parts* in_dev, uint32_t n_src, const uint64_t* src_parts,
                   uint64_t txn_base, uint64_t n_owned, void* stream, ad_merged* out);

/* Deps.merge of replies whose key sets may overlap -- the coordinator's union of the PartialDeps
 * its replicas return for one transaction (CoordinateTransaction.java:70-101,
 * Deps.merge Deps.java:281-286, RelationMultiMap.linearUnion RelationMultiMap.java:561-816): as
 * ad_parts_merge, but keys (ranges) of different sources may repeat and their TxnId sets are
 * unioned. Parts must carry global ranks (AD_IDS_RANK). Sources in any order. */
int ad_parts_union(ad_ctx* ctx, const ad_parts* in_dev, uint32_t n_src, const uint64_t* src_parts,
                   uint64_t txn_base, uint64_t n_owned, void* stream, ad_merged* out);

/* ---- node exchange (SURVEY §8 e): combine the stores' PartialDeps on the owning store --------
 * After every store of a node resolved its share of a node batch (ad_deps_batch_device, AD_PARTS_ONLY
 * is enough), each store's parts are exported grouped by owner, moved to the owner and merged there
 * (K3, ad_parts_merge) -- CommandStores.mapReduce's reduce with PartialDeps.with
 * (CommandStores.java:576-593, PreAccept.reduce PreAccept.java:140-156). Store s (slice order) owns the
 * requests [txn_base[s], txn_base[s] + n_owned[s]) of the node batch; dest_first[s] (host, n + 1 entries)
 * cuts store s's local batch (ascending global indices txn_index[s], device) by owner. Ids move as
 * global ranks when every store has the node's global dictionary installed (ad_set_global_dict),
 * else as {msb, lsb, node} triplets. Results: one ad_merged per store, device memory owned by it. */
typedef struct ad_exchange_stats {
    uint64_t bytes_moved;          /* bytes sent to other stores (xGMI payload) */
    double ms_export, ms_move, ms_merge, ms_total;
} ad_exchange_stats;

/* One process driving every store of the node (the Java host: one process, a CommandStore per thread,
 * one GPU each -- or several stores on one GPU): device copies, hipMemcpyPeerAsync over xGMI between
 * GPUs. ctxs[s], res[s], txn_index[s], dest_first[s] per store; out[n]. On an error every store's stream is
 * synchronised before the call returns (nothing it queued is left running) and every out[] is zeroed. */
int ad_exchange_local(ad_ctx* const* ctxs, uint32_t n, const ad_deps_result* const* res, const int64_t* const* txn_index,
                      const uint64_t* const* dest_first, const uint64_t* txn_base, const uint64_t* n_owned,
                      ad_merged* out, ad_exchange_stats* stats);

/* One process per GPU: an RCCL communicator over the node's stores (rank = slice order). Rank 0 makes
 * the id (ad_comm_unique_id) and the host shares it out of band; every rank then calls ad_comm_init. */
#define AD_COMM_ID_BYTES 128
int ad_comm_unique_id(uint8_t* id /* [AD_COMM_ID_BYTES] */);
int ad_comm_init(ad_ctx* ctx, const uint8_t* id, int rank, int world);
/* This rank's step: export sizes, RCCL all-gather of the exchange table (below), grouped send/recv of
 * the parts over xGMI, K3 merge of the requests [txn_base, txn_base + n_owned) this rank owns.
 * dest_first: host, world + 1 entries. Enqueued on `stream` (NULL: the ctx stream), complete on return.
 * One host synchronisation plans the move (the table read back), one completes the merge; a step that
 * grows some rank's buffers adds a one-word status all-gather. Failure is collective: a rank whose
 * export fails still joins the table all-gather with its status, and every rank then returns (its own
 * code, or AD_E_PEER). An error after the table is agreed aborts the communicator (ncclCommAbort; the
 * next ad_exchange returns AD_E_STATE until ad_comm_init), so a failing rank exits instead of waiting. */
int ad_exchange(ad_ctx* ctx, const ad_deps_result* res_dev, const int64_t* txn_index_dev, const uint64_t* dest_first,
                uint64_t txn_base, uint64_t n_owned, void* stream, ad_merged* out, ad_exchange_stats* stats);

/* ---- exchange plan: where every transfer of a step starts and ends ---------------------------
 * Shared by ad_exchange and ad_exchange_local, exported for hosts that move the parts with a
 * transport of their own. Pure host code (no device call).
 * Exchange table: one row per rank s (slice order) of `world`, AD_XROW_WORDS(world) uint64 each:
 *   row[4 d + a]     units of array a (0 parts, 1 key words, 2 ids, 3 k2t ints) that s sends to rank d,
 *                    in s's send buffers grouped by destination (the order ad_parts_export writes)
 *   row[4 W + 0]     AD_XROW_MAGIC
 *   row[4 W + 1]     s's id format (AD_IDS_*): every rank must use the same one (else AD_E_STATE)
 *   row[4 W + 2]     status: 0, or -(AD_E_* code) of s's failure before the move (then AD_E_PEER)
 *   row[4 W + 3]     reserved, 0
 *   row[4 W + 4 + a] capacity of s's send buffer of array a, in units
 *   row[4 W + 8 + a] capacity of s's receive buffer of array a, in units
 * Output for `rank`: xfers[a * world + p] = bytes to send to / receive from peer p (offsets into this
 * rank's send / receive buffer of array a; receive side in source order, so K3 sees slice order);
 * recv_units[a] = units this rank receives; src_parts[p] = parts from peer p (ad_parts_merge's
 * src_parts); flags: AD_XPLAN_GROW if any rank's buffers are too small for the step (every rank can
 * tell, so all take the same growth round). Every rank computes the same verdict from the same table. */
#define AD_XROW_HDR 12
#define AD_XROW_WORDS(world) (4u * (uint32_t)(world) + AD_XROW_HDR)
#define AD_XROW_MAGIC 0x41445852ull        /* "ADXR" */
#define AD_XPLAN_GROW 1u
typedef struct ad_xfer {
    uint64_t send_off, send_bytes;   /* this rank's send buffer: the run going to the peer        */
    uint64_t recv_off, recv_bytes;   /* this rank's receive buffer: the run coming from the peer  */
} ad_xfer;
int ad_exchange_plan(const uint64_t* table, uint32_t world, uint32_t rank, ad_xfer* xfers /* [4 * world] */,
                     uint64_t* recv_units /* [4] */, uint64_t* src_parts /* [world] */, uint32_t* flags);

/* Copy device memory owned by the library (results) into a host buffer: for hosts without a
 * HIP binding of their own (the Panama FFM wrapper). */
int ad_copy_to_host(ad_ctx* ctx, void* dst, const void* src_dev, uint64_t bytes);

/* ---- execution ordering (config 5): topological apply levels -------------------------
 * Txn i: executeAt (msb/lsb/node), kind, keys [key_off[i],key_off[i+1]) and direct deps
 * [dep_off[i], dep_off[i+1]) (indices of txns it waits on regardless of key).
 * level[i] = 0 if T_i waits on nothing, else 1 + max level of what it waits on, where on
 * each shared key T waits for every earlier (by executeAt) committed txn its kind witnesses
 * (Txn.Kind.witnesses, Txn.java:221-235; CommandsForKey.notifyManaged :1193-1274;
 * Commands.updateWaitingOn :700-775). */
typedef struct ad_graph_soa {
    uint64_t n_txns;
    const uint64_t* exec_msb;
    const uint64_t* exec_lsb;
    const int32_t*  exec_node;
    const uint8_t*  kind;
    const uint64_t* key_off;
    const int64_t*  keys;
    const uint64_t* dep_off;         /* NULL = no direct deps */
    const uint32_t* deps;
} ad_graph_soa;

int ad_levels(ad_ctx* ctx, const ad_graph_soa* g, uint32_t* level_out, ad_stats* stats);

/* As ad_levels with every array of g and level_out in device memory (HBM); the work is
 * enqueued on `stream` (NULL = the ctx stream) and complete on return. key_off[0] must be 0.
 * Errors: AD_E_DUP_EXEC (two txns with equal executeAt), AD_E_INVAL (dep index >= n_txns). */
int ad_levels_device(ad_ctx* ctx, const ad_graph_soa* g_dev, uint32_t* level_out_dev, void* stream, ad_stats* stats);

/* ---- PreAccept timestamp proposal ------------------------------------------
 * CommandStore.preaccept (CommandStore.java:322-347) for a batch of PreAccepts on one snapshot:
 * minNonConflicting = maxConflicts.get(keys) -- the Timestamp.max fold of a ReducingRangeMap over
 * the request's keys (ReducingRangeMap.foldl, ReducingRangeMap.java:123-157; MaxConflicts.java:46-50)
 * -- and the decisions that need no clock. A ReducingRangeMap as SoA: interval i covers
 * [starts[i], starts[i+1]) (inclusive_ends = 0) or (starts[i], starts[i+1]] (inclusive_ends = 1),
 * starts ascending key ordinals (RoutingKey order), value i = {msb, lsb, node}, present[i] = 0
 * for a null value. */
typedef struct ad_range_map_soa {
    uint64_t        n_values;
    const int64_t*  starts;          /* [n_values + 1] */
    const uint64_t* msb;
    const uint64_t* lsb;
    const int32_t*  node;
    const uint8_t*  present;         /* NULL = all present */
    uint32_t        inclusive_ends;
} ad_range_map_soa;

/* per-request result flags of ad_preaccept_device */
#define AD_PA_FAST     1u   /* witnessedAt = txnId (permitFastPath, txnId >= minNonConflicting, epoch)  */
#define AD_PA_REJECTED 2u   /* rejectBefore holds an id above txnId on a key: reply uniqueNow(txnId).asRejected() */
#define AD_PA_ESP      4u   /* ExclusiveSyncPoint: witnessedAt = txnId (markExclusiveSyncPoint on the host) */

/* Install the store's maxConflicts and rejectBefore maps (NULL = empty). Host arrays, copied. */
int ad_preaccept_maps_load(ad_ctx* ctx, const ad_range_map_soa* max_conflicts, const ad_range_map_soa* reject_before);

/* For every request of q_dev (device arrays; keys ascending): out_msb/lsb/node[i] =
 * minNonConflicting (Timestamp.NONE = zeros when no key has a value), out_flags[i] = AD_PA_*.
 * Without FAST/REJECTED/ESP the host replies time.uniqueNow(minNonConflicting); with REJECTED
 * the node's clock-based expiry (preAcceptTimeout) is still the host's. Outputs in device memory;
 * enqueued on `stream` and complete on return. */
int ad_preaccept_device(ad_ctx* ctx, const ad_query_soa* q_dev, uint32_t permit_fast_path, uint64_t node_epoch,
                        void* stream, uint64_t* out_msb, uint64_t* out_lsb, int32_t* out_node, uint8_t* out_flags,
                        ad_stats* stats);

/* ---- recovery scans ---------------------------------------------------------
 * The four CommandsForKey.mapReduceFull scans BeginRecovery runs for a recovering txnId
 * (BeginRecovery.java:132-144, :329-380; CommandsForKey.mapReduceFull CommandsForKey.java:809-908,
 * InMemorySafeStore.mapReduceFull InMemoryCommandStore.java:874-882), batched: request i recovers
 * txnId i (testTxnId; executeAt and min_epoch are not read) over its keys, testKind =
 * txnId.kind().witnessedBy() (Txn.java:247-262).
 *
 * TxnInfo.missing() (CommandsForKey.java:332-341): the ids each entry's deps do not hold. Entry e of
 * the loaded ad_cfk_soa has missing ids [off[e], off[e+1]) (ascending); without a load every entry
 * has NO_TXNIDS. Loading a new ad_cfk_soa clears them. CommandsForKey.loadingPruned is empty (no
 * pruned ids are being loaded), as it is once a store has caught up. */
typedef struct ad_cfk_missing_soa {
    uint64_t n_entries;             /* == n_entries of the loaded ad_cfk_soa */
    const uint64_t* off;            /* [n_entries + 1] */
    const uint64_t* msb;
    const uint64_t* lsb;
    const int32_t*  node;
} ad_cfk_missing_soa;

int ad_cfk_missing_load(ad_ctx* ctx, const ad_cfk_missing_soa* missing);

/* which scan (BeginRecovery.java): the result is the Deps its map lambda builds; for the two
 * boolean scans the answer is "the request's result holds a pair" (the lambda returns true on the
 * first (key, txnId) the scan visits) and the pairs are the witnesses. */
#define AD_RECOVER_STARTED_BEFORE_ACCEPTED_NO_WITNESS 0  /* acceptedOrCommittedStartedBeforeWithoutWitnessing :329-342:
                                                          * STARTED_BEFORE, WITHOUT, IS_PROPOSED            */
#define AD_RECOVER_STARTED_BEFORE_STABLE_WITNESS      1  /* stableStartedBeforeAndWitnessed :344-352:
                                                          * STARTED_BEFORE, WITH, IS_STABLE                 */
#define AD_RECOVER_STARTED_AFTER_ACCEPTED_NO_WITNESS  2  /* hasAcceptedOrCommittedStartedAfterWithoutWitnessing
                                                          * :354-367: STARTED_AFTER, WITHOUT, IS_PROPOSED    */
#define AD_RECOVER_EXECUTES_AFTER_STABLE_NO_WITNESS   3  /* hasStableExecutesAfterWithoutWitnessing :369-380:
                                                          * ANY, WITHOUT, IS_STABLE                         */

/* What the recovery scans read of the store's live range commands (InMemorySafeStore.mapReduceFull ->
 * mapReduceRangesInternal, InMemoryCommandStore.java:884-958): per command of the last
 * ad_range_cmds_load (same order; historical and erased ones are not read), its status class, whether
 * it knows deps (known().deps.hasProposedOrDecidedDeps()), executeAtOrTxnId, and the TxnIds t for
 * which partialDeps().intersects(t, the command's ranges) holds (ascending) -- the witness test of
 * :946. A scan then tests, per range command whose ranges hold one of the request's keys:
 * STARTED_AFTER txnId > testTxnId; STARTED_BEFORE txnId < testTxnId and executeAtOrTxnId >=
 * testTxnId; ANY executeAtOrTxnId >= testTxnId; the status class; testKind; deps known; WITH: the
 * list holds testTxnId, WITHOUT: it does not; the pairs (range, txnId) go to rangeDeps (scan 0's
 * lambda also wants executeAt > testTxnId, :335). */
#define AD_RS_PROPOSED 1   /* Status PreCommitted, Committed or Accepted (IS_PROPOSED, :917-925)   */
#define AD_RS_STABLE   2   /* Stable <= Status < Truncated (IS_STABLE, :926-928)                   */
typedef struct ad_range_cmds_recovery_soa {
    uint64_t n_cmds;                /* == n_cmds of the loaded ad_range_cmds_soa */
    const uint8_t*  status;         /* AD_RS_* (0: neither)                       */
    const uint8_t*  has_deps;
    const uint64_t* exec_msb;       /* executeAtOrTxnId                           */
    const uint64_t* exec_lsb;
    const int32_t*  exec_node;
    const uint64_t* dep_off;        /* [n_cmds + 1]                               */
    const uint64_t* dep_msb;
    const uint64_t* dep_lsb;
    const int32_t*  dep_node;
} ad_range_cmds_recovery_soa;

int ad_range_cmds_recovery_load(ad_ctx* ctx, const ad_range_cmds_recovery_soa* rec);

/* Host buffers in, host result out (as ad_deps_batch). A store with live range commands needs
 * their recovery facts (ad_range_cmds_recovery_load after the last ad_range_cmds_load), else
 * AD_E_STATE. Range-domain requests (ad_query_soa.range_*: a recovering sync point or range txn, whose
 * Seekables BeginRecovery hands to mapReduceFull) scan every CommandsForKey inside their ranges sliced
 * to the store (InMemoryCommandStore.java:289-304) and the range commands whose ranges intersect them
 * (:884-958); RedundantBefore takes no part in these scans. */
int ad_recovery_batch(ad_ctx* ctx, const ad_query_soa* q, uint32_t scan, ad_deps_result** out);
/* Device buffers in and out, as ad_deps_batch_device (result valid until the next batch call). */
int ad_recovery_batch_device(ad_ctx* ctx, const ad_query_soa* q_dev, uint32_t scan, void* stream, ad_deps_result* out);

/* ---- device-resident CommandsForKey maintenance ----------------------------
 * CommandsForKey.update (CommandsForKey.java:972-1042) for a batch of status transitions, applied to
 * the snapshot in HBM (no host ingest, no re-upload). Update i raises the byId entry of txnId i in
 * the CommandsForKey of keys[i] to InternalStatus status[i] with executeAt i and the command's
 * ballot (acceptedOrCommitted) i. The entry is replaced (:1013-1036) iff the new status is above its
 * current one, or equal with status.hasInfo and a ballot above the entry's TxnInfo.ballot(), or is
 * PREACCEPTED_OR_ACCEPTED_INVALIDATE over ACCEPTED with a higher ballot; the replacing TxnInfo
 * (TxnInfo.create :254-262) keeps executeAt i only when the status has an executeAt (ACCEPTED ..
 * APPLIED; txnId otherwise) and the ballot only when it has a ballot (PREACCEPTED_OR_ACCEPTED_INVALIDATE
 * .. COMMITTED; Ballot.ZERO otherwise). Updates of one entry apply in batch order. committedByExecuteAt,
 * maxAppliedWriteByExecuteAt and every derived device array follow (:642-681).
 * The caller filters what the Java drops before the search (txnId < shardRedundantBefore, :995).
 * A txnId the key's byId does not hold is inserted at its byId position (:1002-1007, -1 - binarySearch).
 * Ids the store's id dictionary does not hold (txnIds and executeAts) join it: appended when newer
 * than every id of the store, otherwise merged, which renumbers every id rank on the device (a
 * monotone remap: nothing is re-sorted). A key without a CommandsForKey gets one (the store creates
 * it before the update; key indices renumbered, key hash and KeyLines follow). Errors (nothing
 * applied): AD_E_INVAL (status > 7, live range-domain id), AD_E_INCONSISTENT_ID, AD_E_DUP_EXEC (two
 * committed entries of a key with one executeAt, :1439); AD_E_PARTIAL (the explicit updates applied,
 * the deps-derived part not: ad_cfk_update_status). Ids and keys added by a failed batch stay
 * (an unreferenced id or an empty CommandsForKey changes no answer). Host copies (ad_cfk_entries, recovery views, SEQUENTIAL batches)
 * follow on demand. */
/* TxnInfo.missing() and the deps-derived additions (Updating.insertOrUpdate, Updating.java:99-470):
 * a batch carrying deps (dep_off non-NULL) keeps every entry's missing() list on the device, as the
 * reference's sequence of updates leaves it -- an update with deps derives its TxnInfo's list
 * (computeInfoAndAdditions :194-287: the key's entries below depsKnownBefore its kind witnesses, not
 * COMMITTED or later, not in its deps), other entries lose ids that became COMMITTED or INVALID and
 * gain the batch's insertions below COMMITTED under their depsKnownBefore that they witness
 * (Utils.java:68-352) -- and inserts the deps the key's byId lacks as TRANSITIVELY_KNOWN entries:
 * those the command's kind witnesses, and every dep above the key's last txnId as the update sees it
 * (past byId's end the Java adds without the witness test, :253-262). Additions below the key's
 * prunedBefore are dropped (removePrunedAdditions, :111-117) and handed back by ad_cfk_load_pruned
 * for the host's Pruning.loadPruned / PostProcess.LoadPruned (:171). The lists start from the last
 * ad_cfk_missing_load (NO_TXNIDS without one). A batch without deps hands them back to the host copy,
 * where entries leaving ACCEPTED..APPLIED or moved mark them stale (ad_cfk_missing_load again). The
 * additions are a second internal batch: when only it fails, the explicit updates stand. */
typedef struct ad_cfk_update_soa {
    uint64_t n;
    const int64_t*  keys;
    const uint64_t* txn_msb;
    const uint64_t* txn_lsb;
    const int32_t*  txn_node;
    const uint64_t* exec_msb;
    const uint64_t* exec_lsb;
    const int32_t*  exec_node;
    const uint8_t*  status;          /* AD_ST_* = InternalStatus.from(command.saveStatus()) */
    const uint64_t* ballot_msb;      /* command.acceptedOrCommitted(); all three NULL = Ballot.ZERO
                                      * (all three or none: AD_E_INVAL otherwise) */
    const uint64_t* ballot_lsb;
    const int32_t*  ballot_node;
    /* command.partialDeps().txnIds(key) past redundantBefore.shardRedundantBefore() (the cursor of
     * Updating.computeInfoAndAdditions :184-185), ascending: deps of update i are
     * [dep_off[i], dep_off[i+1]); read for updates with ACCEPTED..APPLIED. NULL: no deps (see below). */
    const uint64_t* dep_off;         /* [n + 1] */
    const uint64_t* dep_msb;
    const uint64_t* dep_lsb;
    const int32_t*  dep_node;
} ad_cfk_update_soa;

/* Host buffers (staged to the device). n_applied (may be null): updates that changed an entry;
 * stats (may be null): ms_stage[0] dictionary append + locate + apply + insertion, ms_stage[1]
 * re-derivation, ms_device total, n_keys[0] entries inserted, n_keys[1] ids added to the dictionary,
 * n_keys[2] TRANSITIVELY_KNOWN entries inserted from deps. */
int ad_cfk_update(ad_ctx* ctx, const ad_cfk_update_soa* u, uint64_t* n_applied, ad_stats* stats);
/* Device buffers, on `stream` (null: the context's stream). Synchronous on return. */
int ad_cfk_update_device(ad_ctx* ctx, const ad_cfk_update_soa* u_dev, void* stream, uint64_t* n_applied, ad_stats* stats);
/* What the last ad_cfk_update[_device] left: *applied = 1 when its explicit updates stand (AD_OK, or
 * AD_E_PARTIAL), 0 when nothing was applied (every other error); *failed_update = the batch index of the
 * update a failure names, -1 for none. AD_E_PARTIAL: a batch with deps whose update *failed_update
 * carried a dep its kind does not witness that is absent from the key's byId and not an
 * ExclusiveSyncPoint (Updating.java:239-249, where the Java throws) -- or a device failure in that
 * second part: every explicit update stands (the Java would have applied those before the throwing
 * one and none after it: the caller re-applies nothing, and fixes or drops the offending dep), no
 * addition was inserted, and the missing() lists ask for a reload (ad_cfk_missing: AD_E_STATE until
 * ad_cfk_missing_load). */
int ad_cfk_update_status(const ad_ctx* ctx, int* applied, int64_t* failed_update);
/* The LoadPruned requests of the last ad_cfk_update[_device] (Updating.java:111-117,171): for each
 * addition dropped below its key's prunedBefore, the update (batch index) whose deps held it, the key
 * and the TxnId -- the host issues the loads (Pruning.loadPruned). Batch order of the updates. Views
 * owned by the context, valid until its next update batch. */
int ad_cfk_load_pruned(ad_ctx* ctx, uint64_t* n, const uint64_t** update, const int64_t** keys, const uint64_t** msb,
                       const uint64_t** lsb, const int32_t** node);
/* TxnInfo.missing() of every entry as it stands (load order): ids [off[e], off[e+1]) ascending.
 * AD_E_STATE when the lists are stale (updates without deps moved entries after a load). Views
 * owned by the context, valid until its next call. */
int ad_cfk_missing(ad_ctx* ctx, uint64_t* n_entries, const uint64_t** off, const uint64_t** msb, const uint64_t** lsb,
                   const int32_t** node);
/* The store's entries as they stand (load order): status and executeAt per entry. Views owned by
 * the context, valid until its next call. */
int ad_cfk_entries(ad_ctx* ctx, uint64_t* n_entries, const uint8_t** status, const uint64_t** exec_msb,
                   const uint64_t** exec_lsb, const int32_t** exec_node);
/* TxnInfo.ballot() of every entry of the loaded ad_cfk_soa (TxnInfoExtra, CommandsForKey.java:273-283;
 * Ballot.ZERO where the TxnInfo has none). Without a load every entry holds Ballot.ZERO; loading a new
 * ad_cfk_soa clears them. */
int ad_cfk_ballots_load(ad_ctx* ctx, uint64_t n_entries, const uint64_t* msb, const uint64_t* lsb, const int32_t* node);
/* The entries' ballots as they stand (views as ad_cfk_entries). */
int ad_cfk_ballots(ad_ctx* ctx, uint64_t* n_entries, const uint64_t** msb, const uint64_t** lsb, const int32_t** node);

/* Pruning.maybePrune (Pruning.java:164-199) -> pruneBefore (:205-331) on the device, for the
 * CommandsForKey of each listed key (key ordinals, host array; keys == NULL: every key), as
 * SafeCommandsForKey.update runs it after an Applied command updated the key
 * (SafeCommandsForKey.java:73-78; prune_interval = agent.cfkPruneInterval(), min_hlc_delta =
 * agent.cfkHlcPruneDelta()). Per key: with maxAppliedWriteByExecuteAt >= prune_interval, the new
 * prunedBefore is the latest APPLIED Write before it in committedByExecuteAt whose executeAt.hlc()
 * <= that Write's executeAt.hlc() - min_hlc_delta, taken when its TxnId is above the current
 * prunedBefore and it is not byId[0]; below it, INVALID_OR_TRUNCATED entries and APPLIED entries
 * executing before it leave byId and committedByExecuteAt (a key where nothing would leave is left as
 * it was, prunedBefore included). Every TxnInfo.missing() is NO_TXNIDS in this model: with lists
 * loaded (ad_cfk_missing_load) AD_E_STATE. Removed ids stay in the id dictionary. n_removed: entries
 * removed; stats (may be null): ms_device, n_keys[0] entries removed, n_keys[1] keys pruned. */
int ad_cfk_prune(ad_ctx* ctx, const int64_t* keys, uint64_t n_keys, int32_t prune_interval, int64_t min_hlc_delta,
                 uint64_t* n_removed, ad_stats* stats);
/* The store's CommandsForKeys as they stand: keys, byId segments ([seg[k], seg[k+1]) of the entry
 * arrays, n_keys + 1 offsets), every entry's TxnId and each key's prunedBefore as an index into its
 * byId (-1: none). Views owned by the context, valid until its next call. */
int ad_cfk_byid(ad_ctx* ctx, uint64_t* n_keys, const int64_t** keys, const uint64_t** seg, uint64_t* n_entries,
                const uint64_t** txn_msb, const uint64_t** txn_lsb, const int32_t** txn_node, const int64_t** pruned_before);

/* ---- debug invariant checks ---------------------------------------------------
 * Structural invariants the reference asserts, checked in HBM without copying anything back.
 * ad_check_result_device: every request and map of a device result (ad_deps_batch_device,
 * ad_recovery_batch_device; not AD_PARTS_ONLY) against RelationMultiMap.checkValid
 * (RelationMultiMap.java:1074-1097) and the builder's layout (:147-260): keys strictly ascending,
 * txnIds strictly ascending and inside ad_dict, keysToTxnIds = nKeys strictly increasing absolute end
 * offsets from above nKeys to its length, each key's values strictly ascending and below nTxnIds,
 * every TxnId some key's value, offsets monotone. *first = request * 3 + map of the first violation.
 * ad_check_snapshot: the prepared snapshot as it stands (after ad_cfk_update batches too): keys
 * strictly ascending, each key's byId strictly increasing by TxnId (CommandsForKey.java:1438) with
 * dictionary member ranks and its cached last txnId, committed Writes by strictly increasing
 * executeAt (:1439), the id dictionary strictly ascending (Timestamp.compareTo). *first = the first
 * failing key index (n_keys + i: dictionary ids i, i + 1). first may be NULL; ~0 = none. */
int ad_check_result_device(ad_ctx* ctx, const ad_deps_result* res_dev, void* stream, uint64_t* n_violations,
                           uint64_t* first);
int ad_check_snapshot(ad_ctx* ctx, uint64_t* n_violations, uint64_t* first);

#ifdef __cplusplus
}
#endif
#endif /* ACCORD_DEPS_H */
