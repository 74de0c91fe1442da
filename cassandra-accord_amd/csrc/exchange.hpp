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
    const uint32_t* gmap;                         // [n_dict] global rank of each dictionary id (null: triplets)
    const uint8_t* reg; const uint64_t* t_reg;    // parts-only batch: per-request regions (null: packed arrays)
    uint32_t* sz;                                 // [n] parts (non-empty maps) per request
    uint64_t* off;                                // [n+1] their exclusive scan
    int64_t* hdr; int64_t* okeys; int64_t* oids; int32_t* ok2t;
};

// Merge (K3) of received parts for requests [txn_base, txn_base + n_owned).
struct MergeArgs {
    uint64_t n_parts, n_owned, txn_base;
    uint32_t n_src;
    const uint64_t* src_first;                    // [n_src+1] part boundaries per source
    const int64_t* hdr; const int64_t* keys; const int64_t* ids; const int32_t* k2t;
    uint32_t* psz;                                // [3][n_parts] key words, ids, k2t
    uint64_t* poff;                               // [3][n_parts+1]
    int32_t* slot;                                // [3*n_owned][n_src] part index or -1
    uint32_t* dup;                                // [n_ids] exclusive per-part dup prefix | dup bit
    uint32_t* gsz;                                // [3][3*n_owned] key words, union ids, k2t
    uint64_t* goff;                               // [3][3*n_owned+1]
    uint32_t* error;
    uint64_t* o_keys_off; uint64_t* o_txn_off; uint64_t* o_k2t_off;   // [3][n_owned+1]
    int64_t* o_keys; int64_t* o_ids; int32_t* o_k2t;
    // AD_IDS_RANK parts: ids are uint32 global ranks
    uint32_t* u;                                  // [n_ids] union index of each received id | DUP_BIT
    uint32_t* ppre;                               // [2][n_parts] key words / pairs of earlier parts of its group
    uint64_t n_global;
    const uint64_t* g_msb; const uint64_t* g_lsb; const int32_t* g_node;   // the global dictionary
    // ad_parts_union (keys of different sources may overlap): per received key word / k2t entry
    uint32_t* kdp; uint32_t* kuk; uint32_t* khead;   // [n_key_words]: dup prefix, union key index | DUP_BIT, head
    uint32_t* pdp; uint32_t* ppos;                   // [n_k2t]: pairs' dup prefix, body position | DUP_BIT
};

// global rank of each local dictionary id (binary search in the global dictionary)
hipError_t run_global_map(const uint64_t* l_msb, const uint64_t* l_lo_norm, const int32_t* l_node, uint64_t n_local,
                          const uint64_t* g_msb, const uint64_t* g_lsb, const int32_t* g_node, uint64_t n_global,
                          uint32_t* map, uint32_t* err, hipStream_t st);

hipError_t run_export_sizes(const ExportArgs& a, hipStream_t st);
hipError_t run_export_emit(const ExportArgs& a, hipStream_t st);
hipError_t run_export_bounds(const ExportArgs& a, const uint64_t* dest_first, uint32_t n_dest, uint64_t* counts,
                             hipStream_t st);
hipError_t run_merge_prepare(const MergeArgs& a, hipStream_t st);
hipError_t run_merge_slots(const MergeArgs& a, hipStream_t st);
hipError_t run_merge_count(const MergeArgs& a, hipStream_t st);
hipError_t run_merge_emit(const MergeArgs& a, hipStream_t st);
hipError_t run_merge_bases(const MergeArgs& a, uint64_t* out, hipStream_t st);
// AD_IDS_RANK merge: union ranks per group (wave per group), then thread-per-part emission
hipError_t run_merge_rank(const MergeArgs& a, hipStream_t st);
hipError_t run_merge_emit_rank(const MergeArgs& a, hipStream_t st);
// ad_parts_union: general union (overlapping keys), rank-format ids
hipError_t run_union_rank(const MergeArgs& a, hipStream_t st);
hipError_t run_union_emit(const MergeArgs& a, hipStream_t st);

}  // namespace adx
