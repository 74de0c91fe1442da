/*
 * refcpu — CPU restatement of the reference (Apache Cassandra Accord, Java) dependency
 * calculation for PreAccept/Accept.  TEST INFRASTRUCTURE ONLY: it is the parity oracle and
 * the CPU baseline, never part of the product (libaccord_deps.so does not link it).
 *
 * Pinning: the Java reference cannot run in this image (no JDK) and ships
 * no golden vectors; the restatement is pinned by the reference's own known-answer tests
 * (PreAcceptTest.java:114,209,241,283) and by ports of its model-based tests
 * (KeyDepsTest, RangeDepsTest, SearchableRangeListTest, DepsTest) under tests/.
 *
 * Data formats are the ones of include/accord_deps.h (shared struct layouts only).
 */
#ifndef ACCORD_REFCPU_H
#define ACCORD_REFCPU_H

#include "../include/accord_deps.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct rc_store rc_store;

/* Fully materialised result: TxnIds as {msb,lsb,node}, range keys as (start,end). */
typedef struct rc_result {
    uint64_t  n_txns;
    uint64_t* keys_off[AD_NMAPS];
    int64_t*  keys[AD_NMAPS];        /* key ordinal, or range start for AD_MAP_RANGE      */
    int64_t*  keys_end[AD_NMAPS];    /* range end for AD_MAP_RANGE, NULL otherwise        */
    uint64_t* txn_off[AD_NMAPS];
    uint64_t* txn_msb[AD_NMAPS];
    uint64_t* txn_lsb[AD_NMAPS];
    int32_t*  txn_node[AD_NMAPS];
    uint64_t* k2t_off[AD_NMAPS];
    int32_t*  k2t[AD_NMAPS];
    uint64_t  scan_entries;          /* sum over probes of CommandsForKey scan length `end` */
} rc_result;

int  rc_store_create(const ad_config* cfg, rc_store** out);
void rc_store_destroy(rc_store* s);
const char* rc_last_error(const rc_store* s);

int rc_cfk_load(rc_store* s, const ad_cfk_soa* cfk);
int rc_range_cmds_load(rc_store* s, const ad_range_cmds_soa* cmds);
int rc_range_cmds_update(rc_store* s, const ad_range_cmds_soa* in);
int rc_redundant_load(rc_store* s, const ad_redundant_soa* rb);
int rc_redundant_advance(rc_store* s, const ad_redundant_soa* in);
/* the store's slice sets that ad_query_soa.slice_set names (ad_slice_sets_load) */
int rc_slice_sets_load(rc_store* s, uint32_t n_sets, const uint64_t* off, const int64_t* start, const int64_t* end);

/* Resolve queries [first, first+count) of q (count == 0: all). */
int  rc_deps_batch(rc_store* s, const ad_query_soa* q, uint32_t flags, uint64_t first,
                   uint64_t count, rc_result** out);
void rc_result_free(rc_result* r);

/* request-wise PartialDeps.with over the results of several CommandStores (multi-GPU oracle) */
int rc_result_merge(const rc_result* const* parts, int n_parts, rc_result** out);

int rc_levels(const ad_graph_soa* g, uint32_t* level_out);

/* CommandStore.preaccept (CommandStore.java:322-347) minus the clock: minNonConflicting and the
 * AD_PA_* flags per request (include/accord_deps.h, ad_preaccept_device). */
int rc_preaccept(const ad_range_map_soa* max_conflicts, const ad_range_map_soa* reject_before, const ad_query_soa* q,
                 uint32_t permit_fast_path, uint64_t node_epoch, uint64_t* out_msb, uint64_t* out_lsb, int32_t* out_node,
                 uint8_t* out_flags);

/* TxnInfo.missing() per entry of the loaded CommandsForKey snapshot (rc_cfk_load order) and the
 * four BeginRecovery mapReduceFull scans (AD_RECOVER_*; include/accord_deps.h) */
int rc_cfk_missing_load(rc_store* s, const ad_cfk_missing_soa* m);
int rc_recovery_batch(rc_store* s, const ad_query_soa* q, uint32_t scan, uint64_t first, uint64_t count,
                      rc_result** out);
/* the range commands' recovery facts (ad_range_cmds_recovery_load) */
int rc_range_cmds_recovery_load(rc_store* s, const ad_range_cmds_recovery_soa* rec);

/* exposed for the tests */
int rc_tid_cmp(uint64_t amsb, uint64_t alsb, int32_t anode, uint64_t bmsb, uint64_t blsb, int32_t bnode);

#ifdef __cplusplus
}
#endif
#endif
