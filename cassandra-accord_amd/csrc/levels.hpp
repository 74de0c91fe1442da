// levels.hpp — K5: execution-ordering levels and the device LSD radix sort it
// uses. Host launch interface of levels.hip.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

namespace adx {

// The waitingOn graph of a batch of committed transactions (device pointers; ad_graph_soa).
struct LevelsIn {
    uint64_t n;
    const uint64_t* exec_msb;
    const uint64_t* exec_lsb;
    const int32_t* exec_node;
    const uint8_t* kind;
    const uint64_t* key_off;     // [n+1]
    const int64_t* keys;
    const uint64_t* dep_off;     // [n+1] or null
    const uint32_t* deps;
};

struct LevelsOut {
    uint64_t n_levels = 0;       // 1 + max level (0 for an empty graph)
    uint64_t n_edges = 0;        // edges of the sparsified waitingOn DAG (key chains + direct deps)
    uint64_t n_occ = 0;          // txn-key occurrences
    uint64_t n_launch = 0;       // frontier-step launches (incl. the empty tail of the last chunk)
    bool packed = false;         // the packed path ran (keys-only sorts, predecessor records)
    double ms_build = 0;         // exec ranking + key chains + CSR of successors (HIP events)
    double ms_frontier = 0;      // frontier loop
    double ms_total = 0;
};

struct LevelsWork;
LevelsWork* levels_work_create();
void levels_work_destroy(LevelsWork* w);

// level_out (device, [n]): level[i] of txn i. Returns 0 or an AD_E_* code (message in *err).
int run_levels(LevelsWork* w, const LevelsIn& in, uint32_t* level_out, hipStream_t st, LevelsOut* out,
               std::string* err);

// Stable LSD radix sort of (key, val) pairs by the key bits in `digit_mask` (bit d = sort on
// bits [8d, 8d+8)); the result ends in (*k_res, *v_res). k_tmp/v_tmp: scratch of n entries,
// hist: radix_hist_entries(n) u32, off: that + 1 u64, bsum: scan scratch (per-pass path only).
// Count / scan / scatter kernels per digit.
hipError_t radix_sort_pairs(uint64_t* k_in, uint32_t* v_in, uint64_t* k_tmp, uint32_t* v_tmp, uint64_t n,
                            uint32_t digit_mask, uint32_t* hist, uint64_t* off, uint64_t* bsum, hipStream_t st,
                            uint64_t** k_res, uint32_t** v_res);
uint64_t radix_hist_entries(uint64_t n);

}  // namespace adx
