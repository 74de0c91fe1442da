// kernels.hpp — host-side launch interface of the gfx950 kernels (kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <cstddef>
#include <cstdint>

#include "common.hpp"

namespace adx {

// Device-side control block of one batch: arena bump pointers, overflow and error flags.
struct BatchCtl {
    unsigned long long key_top, key_cap;      // K1 arena (u32 elements)
    unsigned long long rng_top, rng_cap;      // K4 arena (u64 elements)
    unsigned long long scr_top, scr_cap;      // K2 big-txn scratch (bytes)
    unsigned long long reg_top, reg_cap;      // K2 per-request output regions (bytes)
    unsigned long long n_deferred;            // requests the fused kernel hands to the split kernels
    unsigned int overflow;                    // bit0 key arena, bit1 range arena, bit2 scratch, bit3 regions
    unsigned int error;                       // AD_E_* (negated) of the first failure, 0 = none
    unsigned long long n_deferred1;           // lean pass 1 -> pass 2 list slots (reserved in chunks)
    unsigned long long n_deferred2;           // lean pass 2 -> general fused kernel list slots
    unsigned long long n_real1, n_real2;      // requests on those lists
    unsigned long long tot[9];                // totals of the 9 per-request size arrays (after the offsets scan)
    unsigned long long n_big;                 // k_build -> k_build_big: requests with a list family > K2_BIG
    unsigned long long n_wide1;               // wide lean pass 1: requests it took with 33..64 raw emissions
};
constexpr unsigned OVF_PACK = 16u;            // BatchCtl.overflow: a packed output array is too small

constexpr uint64_t NO_RB = ~0ull;
constexpr uint32_t K2_BIG = 512;     // elements in a list family from which k_build_big takes a request (= the LDS path's K2_CAP)
constexpr unsigned ERR_INVAL = 1u;   // BatchCtl.error codes
constexpr unsigned ERR_STATE = 8u;
constexpr unsigned ERR_SLICE = 16u;  // a request's slice_set beyond the store's slice sets

// Per-batch device buffers (sized by the host before the launches).
struct BatchBufs {
    // queries (device pointers; q_* borrowed from the caller or staged by ad_deps_batch)
    uint64_t n_txns, n_probes;
    const uint64_t* q_txn_msb; const uint64_t* q_txn_lsb; const int32_t* q_txn_node;
    const uint64_t* q_exec_msb; const uint64_t* q_exec_lsb; const int32_t* q_exec_node;
    const int64_t* q_min_epoch;      // may be null
    const uint64_t* q_key_off;
    const int64_t* q_keys;
    const uint32_t* q_slice_set;     // per request its slice set (SLICE_STORE: the store's slices); null = all the store's
    // Range-domain requests (run_range_expand): per probe its kind (PK_*; null: every probe is a key of
    // its request) and, for range and redundant-before probes, the range [q_keys[p], q_keys_hi[p])
    const uint8_t* p_kind;
    const int64_t* q_keys_hi;
    uint32_t* p_slot;                // lean passes without range commands: per probe its KeyLine (LS_NONE: outside the slice)
    // K0
    uint32_t* t_S; uint32_t* t_self; uint32_t* t_kinds; int64_t* t_epoch;
    uint32_t* p_txn; uint4* p_rec;
    uint4* q_rec;                    // fused path: per request {key_off, S rank, np | cls << 16 | flags, self rank} (k_prepare)
    // K1
    uint32_t* arena; uint32_t* p_off; uint32_t* p_c0; uint32_t* p_c1;
    // K4
    uint64_t* rarena; uint32_t* p_roff; uint32_t* p_rcnt; uint64_t* p_rb;
    // K2
    uint32_t* sz;                    // [9][n_txns]: per map m: keys, txns, k2t
    uint64_t* off;                   // [9][n_txns+1]
    uint64_t* bsum;                  // [9][ceil(n_txns/1024)] scan block sums
    uint64_t* t_reg;                 // [3][n_txns] byte offset of each request's map region
    uint8_t* reg;                    // per-request output regions
    uint8_t* scratch;                // big-request scratch
    uint32_t* deferred;              // [n_txns] requests deferred by k_resolve
    uint32_t* big;                   // [n_txns] requests k_build hands to k_build_big (one workgroup each)
    uint32_t k2_big;                 // list-family size from which it does (K2_BIG; tests lower it)
    uint32_t kb_sort;                // k_build_big merges a map in LDS up to this many elements (tests: 0 = never)
    uint32_t kb_merge;               // k_build_big's LDS merge as a merge tree (else the rank merge; tests: AD_KB_MERGE)
    uint32_t pack_even;              // pack copy: k_pack_even (few heavy requests) instead of k_pack_tiles's waves
    uint32_t* deferred1;             // requests deferred by lean pass 1 (+ chunk holes)
    uint32_t* deferred2;             // requests deferred by lean pass 2 (+ chunk holes)
    const uint32_t* req_list;        // k_resolve: resolve only these requests (count *req_count); null = all
    const unsigned long long* req_count;
    int64_t* o_keys[3]; uint32_t* o_txns[3]; int32_t* o_k2t[3];
    uint64_t o_cap[9];               // capacities (elements) of the packed arrays, [3 * map + array]
    uint64_t* lb_agg;                // [9][tiles] size sums per tile (k_tile_sums)
    uint64_t* lb_inc;                // [9][tiles] exclusive prefixes of the tile sums (k_tile_scan)
    BatchCtl* ctl;
    // fused path: k_prepare's first block writes the control block (zeros and these arena capacities:
    // key, range, scratch, regions) instead of a host copy before the batch
    uint32_t ctl_init;
    uint64_t init_cap[4];
};
static_assert(sizeof(BatchCtl) % 8 == 0 && offsetof(BatchCtl, key_cap) == 8 && offsetof(BatchCtl, rng_cap) == 24 &&
                  offsetof(BatchCtl, scr_cap) == 40 && offsetof(BatchCtl, reg_cap) == 56,
              "k_prepare's control-block init writes 8-byte words");

// recovery scans: the CommandsForKey entries in load order, for mapReduceFull
struct RecoveryView {
    const uint4* ent;        // per entry {txnId rank, executeAt rank, status | kind << 8 | n_missing << 12, missing off}
    const uint32_t* seg;     // [n_keys + 1] entry range of each key index
    const uint32_t* pruned;  // [n_keys] prunedBefore rank, 0 = none
    const uint32_t* miss;    // TxnInfo.missing() as ranks, ascending per entry
    // 64-ary max trees over the entries (load order) of the executeAt ranks in each status set
    // (0: ACCEPTED/COMMITTED, 1: STABLE/APPLIED; other entries 0): lvl[s][l][j] = max over entries
    // [j * 64^l, (j + 1) * 64^l), l >= 1
    const uint32_t* lvl[2][MAX_LEVELS];
    int n_levels;            // including the entry level
    // per key, its entries' (missing() id, entry) pairs sorted: [inv_off[k], inv_off[k + 1])
    const uint64_t* inv_off;
    const uint2* inv;
    // live range commands (ad_range_cmds_recovery_load): per range entry of the snapshot its command
    // (load order) or ~0u; per command AD_RS_* | has_deps << 2, executeAtOrTxnId and the ids t with
    // partialDeps().intersects(t, its ranges) (ascending), normalised for norm_cmp
    const uint32_t* r_cmd;
    const uint32_t* rc_flags;
    const uint64_t* rc_ex_hi; const uint64_t* rc_ex_lo; const int32_t* rc_ex_node;
    const uint32_t* rc_dep_off;
    const uint64_t* rc_dep_hi; const uint64_t* rc_dep_lo; const int32_t* rc_dep_node;
    bool ranges;             // the store has live range commands
};
constexpr uint32_t RV_MISS_SHIFT = 12;
constexpr uint32_t RV_MAX_MISS = (1u << 20) - 1;

// The RecoveryView of a live store, from the device state ad_cfk_update keeps current (no host copy):
// per entry {txnId rank, executeAt rank, status | kind << 8 | #missing << 12, offset of its list in the
// device missing() ids}, per key its segment start and prunedBefore rank; the two per-status-set max
// trees; the per-key inverted missing() index. mref / moff: the device lists (null: no lists).
// *err gets 1 when a list exceeds RV_MAX_MISS.
struct RvDevIn {
    uint64_t n_ent, n_keys;
    const uint2* ent; const KeyRec* krec; const uint8_t* status; const uint32_t* xrank; const uint32_t* ekey;
    const uint32_t* mref; const uint64_t* moff; const uint32_t* mids;
};
hipError_t run_rv_entries(const RvDevIn& in, uint4* ent, uint32_t* seg, uint32_t* pruned, uint32_t* cnt, uint32_t* err,
                          hipStream_t st);
// levels l >= 1 of the two trees: lvl[set][l] (l < n_levels), lvl_n[l] nodes each
hipError_t run_rv_trees(const RvDevIn& in, uint32_t* const* lvl0, uint32_t* const* lvl1, const uint64_t* lvl_n, int n_levels,
                        hipStream_t st);
// the inverted pairs in entry order (key << 32 | miss rank, entry) at eoff[e] (exclusive scan of cnt)
hipError_t run_rv_inv_pairs(const RvDevIn& in, const uint64_t* eoff, uint64_t* key, uint32_t* val, hipStream_t st);
// inv_off[k] = eoff[segment start of k], inv_off[n_keys] = eoff[n_ent]; inv[p] = {rank, entry} of the sorted pairs
hipError_t run_rv_inv_finish(const RvDevIn& in, const uint64_t* eoff, const uint64_t* skey, const uint32_t* sval,
                             uint64_t n_pairs, uint64_t* inv_off, uint2* inv, hipStream_t st);

// Probe kinds of an expanded batch (a batch with Range-domain requests, run_range_expand): a key of a
// key-domain request (K1 + K4 by key); a CommandsForKey key inside a Range-domain request's sliced ranges
// (K1 only); one sliced range of such a request (K4: range commands whose range intersects it); one
// unsliced range of it (K4: the RedundantBefore entries intersecting it)
constexpr uint8_t PK_KEY = 0, PK_RANGE_KEY = 1, PK_RANGE = 2, PK_RANGE_RB = 3;
// per request its probe count (cnt) and error flag (*err = 1: keys and ranges together, or ranges
// not normalised); then, from the exclusive scan `off`, the probes
// (err[1]: the Range-domain requests, their indices appended to `list`); then, from the exclusive scan `off`,
// the probes: a key-domain request's keys one thread per request, a listed request's one wave each
// sset: per request its slice set (null: the store's slices)
hipError_t run_range_count(const DevSnapshot& s, uint64_t n, const uint64_t* key_off, const uint64_t* range_off,
                           const int64_t* range_start, const int64_t* range_end, const uint32_t* sset, uint32_t* cnt,
                           uint32_t* err, uint32_t* list, uint64_t max_list, bool with_rb, hipStream_t st);
hipError_t run_range_fill(const DevSnapshot& s, uint64_t n, const uint64_t* key_off, const int64_t* keys,
                          const uint64_t* range_off, const int64_t* range_start, const int64_t* range_end,
                          const uint32_t* sset, const uint64_t* off, int64_t* pkeys, int64_t* pkeys_hi, uint8_t* pkind,
                          const uint32_t* list, uint32_t n_list, bool with_rb, hipStream_t st);

hipError_t build_cfk_trees(const DevSnapshot& s, hipStream_t st);
hipError_t build_range_trees(const DevSnapshot& s, hipStream_t st);

hipError_t run_encode(const DevSnapshot& s, const BatchBufs& b, hipStream_t st);
hipError_t run_scan(const DevSnapshot& s, const BatchBufs& b, hipStream_t st);
hipError_t run_range(const DevSnapshot& s, const BatchBufs& b, hipStream_t st);
hipError_t run_build(const DevSnapshot& s, const BatchBufs& b, hipStream_t st);
hipError_t run_recovery(const DevSnapshot& s, const RecoveryView& v, const BatchBufs& b, uint32_t scan, hipStream_t st);
hipError_t run_offsets(const BatchBufs& b, hipStream_t st);
hipError_t run_scan_arrays(const uint32_t* in, uint64_t* out, uint64_t n, int n_arrays, uint64_t* bsum, hipStream_t st);
// off: 9 arrays of n1 offsets back to back; array a += base[a] (a slice's offsets made relative to its batch)
hipError_t run_add_bases(uint64_t* off, uint64_t n1, const uint64_t* base, hipStream_t st);
// ad_deps_batch_into's copy-out: up to OUT_SEGS device -> host-mapped segments in one launch
constexpr int OUT_SEGS = 18;
struct OutSeg {
    const void* src;
    void* dst;                 // device-mapped address of pinned host memory
    uint64_t bytes;            // of the source
    uint64_t add;              // mode 1: every u64 word gets `add`
    uint32_t mode;             // 0 copy, 1 u64 + add, 2 u32 -> u16 (the wire form of k2t)
    uint32_t pad;
};
// the wire form of a slice's keyDeps (ad_deps_batch_into): each output key as its index among the
// request's query keys (u8), and whether every request's k2t segment and unique-txn count fit u16
// (flag[0] bit 0: a key not found or past index 255; bit 1: a k2t value past 65535)
hipError_t run_key_index(uint64_t n, const uint64_t* q_key_off, const int64_t* q_keys, const uint64_t* off,
                         const int64_t* o_keys, uint8_t* idx, uint32_t* flag, hipStream_t st);
struct OutSegs {
    OutSeg s[OUT_SEGS];
    uint32_t n;
};
hipError_t run_copy_out(const OutSegs& g, hipStream_t st);
hipError_t run_pack(const BatchBufs& b, hipStream_t st);
// offsets of the 9 size arrays + totals (+ the packed arrays when `copy`): tile sums, one-block scan
// of the tile sums, then a streaming per-tile scan + pack; no host round trip between resolve and pack
constexpr uint32_t LB_TILE = 256;
inline uint64_t lb_tiles(uint64_t n) { return (n + LB_TILE - 1) / LB_TILE; }
hipError_t run_pack_lb(const BatchBufs& b, bool copy, hipStream_t st);
hipError_t run_collect_totals(const BatchBufs& b, hipStream_t st);

// fused per-request path (resolve.hip)
constexpr uint32_t SLOT_NONE = 0x7FFFFFFFu;    // p_slot: key has no CommandsForKey in this store
constexpr uint32_t SLOT_IN_SLICE = 0x80000000u;
constexpr uint32_t DEFER_HOLE = 0xFFFFFFFFu;      // unused slot of a wave's deferral chunk
constexpr uint32_t DEFER_CHUNK = 64;              // deferral slots a lean wave reserves at a time
constexpr uint32_t REC_FAST = 1u << 24;          // q_rec: lean path applies (<= 8 keys, valid kind, 32-bit key offsets)
constexpr uint32_t REC_SPLIT = 1u << 25;         // q_rec: a Range-domain request of a mixed batch (the split kernels resolve it)
hipError_t run_prepare(const DevSnapshot& s, const BatchBufs& b, hipStream_t st);
// pass 1 with rpw1 = 2 on a store without range commands: wide1 selects the wide kernel (requests of up to
// 64 raw emissions) over the narrow one (up to 32; the rest to pass 2)
hipError_t run_resolve_lean(const DevSnapshot& s, const BatchBufs& b, int pass, uint32_t rpw1, bool wide1, hipStream_t st);

// ---- PreAccept timestamp proposal (preaccept.hip)
struct DevRangeMap {            // a ReducingRangeMap<Timestamp> in HBM (ad_range_map_soa)
    uint64_t n;                 // values; starts has n + 1
    const int64_t* starts;
    const uint64_t* msb; const uint64_t* lsb; const int32_t* node;
    const uint8_t* present;     // null = all present
    uint32_t inclusive_ends;
};

struct PreacceptArgs {
    uint64_t n;
    const uint64_t* txn_msb; const uint64_t* txn_lsb; const int32_t* txn_node;
    const uint64_t* key_off; const int64_t* keys;
    DevRangeMap mc, rb;         // maxConflicts, rejectBefore
    uint32_t permit_fast_path;
    uint64_t node_epoch;
    uint64_t* out_msb; uint64_t* out_lsb; int32_t* out_node; uint8_t* out_flags;
    // the snapshot's key index (null khash: none): a key found there takes its values from
    // key_val[2 * key index] (maxConflicts, rejectBefore): one 64-byte line per key
    const KeySlot* khash; uint64_t khash_mask;
    const struct PaValue* key_val;
};

struct alignas(32) PaValue {     // a map's value at one key (present = 0: none)
    uint64_t msb, lsb;
    int32_t node;
    uint32_t present;
    uint64_t pad;
};

hipError_t run_preaccept(const PreacceptArgs& a, hipStream_t st);
// key_val[2i], key_val[2i+1] = the values of snapshot key i in maxConflicts / rejectBefore
hipError_t run_preaccept_key_values(const DevRangeMap& mc, const DevRangeMap& rb, const int64_t* keys, uint64_t n_keys,
                                    PaValue* key_val, hipStream_t st);
hipError_t run_resolve(const DevSnapshot& s, const BatchBufs& b, hipStream_t st);
hipError_t run_defer_counts(const BatchBufs& b, const uint32_t* deferred, uint64_t nd, uint32_t* cnt, hipStream_t st);
hipError_t run_defer_gather(const BatchBufs& b, const uint32_t* deferred, uint64_t nd, const uint64_t* sub_off,
                            const BatchBufs& sub, uint64_t* o_tm, uint64_t* o_tl, int32_t* o_tn, uint64_t* o_em,
                            uint64_t* o_el, int32_t* o_en, int64_t* o_me, uint64_t* o_ko, int64_t* o_k, int64_t* o_khi,
                            uint8_t* o_kind, uint32_t* o_ss, hipStream_t st);
hipError_t run_defer_scatter(const BatchBufs& b, const uint32_t* deferred, uint64_t nd, const uint32_t* sub_sz,
                             const uint64_t* sub_reg, hipStream_t st);

int device_cu_count();
// the KeyLine table (table_slots lines) from s.kent / cand / cwr; kslot[k] = the line of key k (its
// perfect-hash index), kcell[k] = its stabbing cell (NO_CELL; null: none)
// per key its KeyLine (the perfect hash under the displacements)
hipError_t run_key_slots(const int64_t* keys, uint64_t nk, const uint32_t* disp, uint64_t nb, uint64_t m, uint32_t* kslot,
                         hipStream_t st);
hipError_t run_build_klines(const DevSnapshot& s, const uint32_t* kslot, const uint32_t* kcell, KeyLine* table,
                            uint64_t table_slots, hipStream_t st);
// bytes of the KeyLine table allocation: the lines, then one LeanQuads per line
inline uint64_t kline_table_bytes(uint64_t slots) { return (sizeof(KeyLine) + sizeof(LeanQuads)) * slots; }
inline const LeanQuads* kline_quads(const KeyLine* table, uint64_t slots)
{
    return reinterpret_cast<const LeanQuads*>(table + slots);
}
// the two-level sample of s's dictionary into hi/lo/node (dict_sample_entries(s.n_dict) entries)
hipError_t run_dict_sample(const DevSnapshot& s, uint64_t* hi, uint64_t* lo, int32_t* node, hipStream_t st);
hipError_t run_dict_buckets(const DevSnapshot& s, uint32_t* B, uint32_t lg, hipStream_t st);

}  // namespace adx
