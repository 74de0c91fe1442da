// exchange.hpp — launch interface of the multi-GPU export / merge kernels (exchange.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "common.hpp"

namespace adx {

// Export of one store's batch result (device CSR of ad_deps_result) into the transport format
// of ad_parts (accord_deps.h).
struct ExportArgs {
    uint64_t n;                                   // requests of the batch
    const uint64_t* keys_off[3]; const int64_t* keys[3];
    const uint64_t* txn_off[3];  const uint32_t* txns[3];
    const uint64_t* k2t_off[3];  const int32_t* k2t[3];
    const int64_t* txn_index;                     // [n] global request index (ascending)
    const uint64_t* dict_msb; const uint64_t* dict_lsb; const int32_t* dict_node;   // raw ids
    const int64_t* rt_start; const int64_t* rt_end;                                // range table
    bool rank_ids;                                // ids as uint32 global ranks (the dictionary is the global one), else triplets
    const uint8_t* reg; const uint64_t* t_reg;    // parts-only batch: per-request regions (null: packed arrays)
    uint32_t* sz;                                 // [n] parts (non-empty maps) per request
    uint64_t* off;                                // [n+1] their exclusive scan
    int64_t* hdr; int64_t* okeys; int64_t* oids; int32_t* ok2t;
    // the parts this store keeps (requests [self_lo, self_hi): it owns them) go straight to its own
    // receive arrays, at their send position + self_delta[array] units (no send-buffer copy, no move)
    uint64_t self_lo, self_hi;
    uint64_t ids_per_req;                         // average ids per request (lanes per request of the export)
    int64_t self_delta[4];
    int64_t* rhdr; int64_t* rkeys; int64_t* rids; int32_t* rk2t;
};

// Merge (K3) of received parts for requests [txn_base, txn_base + n_owned).
struct MergeArgs {
    uint64_t n_parts, n_owned, txn_base;
    uint64_t n_elems;                             // received key words + ids + keysToTxnIds (lanes per part)
    uint32_t n_src;
    const uint64_t* src_first;                    // [n_src+1] part boundaries per source
    const int64_t* hdr; const int64_t* keys; const int64_t* ids; const int32_t* k2t;
    uint32_t* psz;                                // [3][n_parts] key words, ids, k2t
    uint64_t* poff;                               // [3][n_parts+1]
    int32_t* slot;                                // [3*n_owned][n_src] part index or -1 (rmerge: [n_owned][n_src]
                                                  // first part of the request in each source)
    uint32_t* dup;                                // [n_ids] exclusive per-part dup prefix | dup bit
    uint32_t* pinfo;                              // rmerge: [n_parts][8] part record (k_rmerge_slots)
    uint32_t* heavy; uint32_t* n_heavy;           // rmerge: groups beyond the LDS merge (r << 2 | map), their count
    uint32_t* gsz;                                // [3][3*n_owned] key words, union ids, k2t (rmerge: [3 k][3 m][n_owned],
                                                  // keys counted in keys)
    uint64_t* goff;                               // [3][3*n_owned+1] (rmerge: [9][n_owned+1], per map from 0)
    uint32_t* error;
    uint64_t* o_keys_off; uint64_t* o_txn_off; uint64_t* o_k2t_off;   // [3][n_owned+1]
    int64_t* o_keys; int64_t* o_ids; int32_t* o_k2t;
    // AD_IDS_RANK parts: ids are uint32 global ranks
    uint32_t* u;                                  // [n_ids] union index of each received id | DUP_BIT
    uint32_t* ppre;                               // [2][n_parts] key words / pairs of earlier parts of its group
                                                  // (rmerge: [n_parts][4] keys and pairs before it, group keys, parts)
    uint64_t n_global;
    // ad_parts_union (keys of different sources may overlap): per received key word / k2t entry
    uint32_t* kdp; uint32_t* kuk; uint32_t* khead;   // [n_key_words]: dup prefix, union key index | DUP_BIT, head
    uint32_t* pdp; uint32_t* ppos;                   // [n_k2t]: pairs' dup prefix, body position | DUP_BIT
};

hipError_t run_export_sizes(const ExportArgs& a, hipStream_t st);
hipError_t run_export_emit(const ExportArgs& a, hipStream_t st);
hipError_t run_export_bounds(const ExportArgs& a, const uint64_t* dest_first, uint32_t n_dest, uint64_t* counts,
                             hipStream_t st);
// the exchange table row of this rank (ad_exchange_plan's layout): counts = k_export_bounds' cumulative
// [n_dest + 1][4], header words after the n_dest x 4 per-destination units
constexpr uint32_t XROW_HDR = 12;
struct XRowHdr { uint64_t w[XROW_HDR]; };
hipError_t run_x_row(const uint64_t* counts, uint32_t n_dest, const XRowHdr& h, uint64_t* row, hipStream_t st);
hipError_t run_merge_prepare(const MergeArgs& a, hipStream_t st);
hipError_t run_merge_slots(const MergeArgs& a, hipStream_t st);
hipError_t run_merge_count(const MergeArgs& a, hipStream_t st);
hipError_t run_merge_emit(const MergeArgs& a, hipStream_t st);
hipError_t run_merge_bases(const MergeArgs& a, uint64_t* out, hipStream_t st);
// AD_IDS_RANK merge: union ranks per group (wave per group), then thread-per-part emission
hipError_t run_merge_rank(const MergeArgs& a, hipStream_t st);
hipError_t run_merge_emit_rank(const MergeArgs& a, hipStream_t st);
// AD_IDS_RANK merge of up to RM_MAX_SRC sources: a 16-lane group per owned request sizes its three
// merged maps (slot = [n_owned][n_src] first part of each source), then emits them after the scan
constexpr uint32_t RM_MAX_SRC = 16;
hipError_t run_rmerge_slots(const MergeArgs& a, hipStream_t st);
hipError_t run_rmerge_size(const MergeArgs& a, hipStream_t st);
// bases of the three maps in the outputs (into `bases`, 12 entries) and the copy pass
hipError_t run_rmerge_copy(const MergeArgs& a, const uint64_t* bases, hipStream_t st);
// ad_parts_union: general union (overlapping keys), rank-format ids
hipError_t run_union_rank(const MergeArgs& a, hipStream_t st);
hipError_t run_union_emit(const MergeArgs& a, hipStream_t st);

}  // namespace adx
