// common.hpp — shared definitions of libaccord_deps (host runtime + gfx950 kernels).
//
// Device representation:
//   * every TxnId/Timestamp of a store snapshot is replaced by its rank in a sorted id
//     dictionary: member i -> 2i+1 (odd); a foreign id falling between members i-1 and i
//     -> 2i (even). Rank order == Timestamp.compareTo order (Timestamp.java:208-217) and rank
//     equality == Timestamp.equals (:244-249), so all kernels compare u32 ranks.
//   * CommandsForKey byId entries (CommandsForKey.java:621) are `uint2 {tau, txw}`:
//       txw = rank | kind << 29
//       tau = elision threshold key: 0 for TRANSITIVELY_KNOWN/INVALID (never emitted),
//             executeAt rank for committed Read/Write (emitted iff executeAt >= M),
//             0xFFFFFFFF otherwise (never elided)                      (:930-950)
//   * per witness class a 64-ary max tree over tau restricted to the class' kinds
//     prunes byId[0,end) down to the emitted entries.
#pragma once
#include <cstdint>
#include <cstddef>

namespace adx {

constexpr uint32_t RANK_BITS = 29;
constexpr uint32_t RANK_MASK = (1u << RANK_BITS) - 1;
constexpr uint64_t MAX_DICT = (1ull << 28) - 1;     // 2*MAX_DICT+1 < 2^29
constexpr uint32_t TAU_NEVER_ELIDED = 0xFFFFFFFFu;
constexpr uint32_t CLASS_DIRECT_BIT = 0x80000000u;   // K1 output: rank | direct-key-deps bit
constexpr int NCLASS = 3;                             // Ws, RsOrWs, AnyGloballyVisible
constexpr int MAX_LEVELS = 8;                         // 64^8 > 2^32 entries
constexpr int WAVE = 64;

// Txn.Kind.Kinds as masks over Kind ordinals (Txn.java:114-152)
constexpr uint32_t KINDS_WS = 1u << 1;
constexpr uint32_t KINDS_RS_OR_WS = (1u << 0) | (1u << 1);
constexpr uint32_t KINDS_ANY_GLOBALLY_VISIBLE = (1u << 0) | (1u << 1) | (1u << 3) | (1u << 4);
constexpr uint32_t CLASS_KINDS[NCLASS] = {KINDS_WS, KINDS_RS_OR_WS, KINDS_ANY_GLOBALLY_VISIBLE};

// Txn.Kind.witnesses() (Txn.java:221-235); 0 = AssertionError (invalid kind for a query)
__host__ __device__ inline uint32_t kind_witnesses(uint32_t kind)
{
    switch (kind)
    {
        case 0: case 2: return KINDS_WS;                    // Read, EphemeralRead
        case 1: case 3: return KINDS_RS_OR_WS;              // Write, SyncPoint
        case 4: return KINDS_ANY_GLOBALLY_VISIBLE;          // ExclusiveSyncPoint
        default: return 0;
    }
}

// smallest witness class whose kind set contains `kinds`
__host__ __device__ inline int kinds_class(uint32_t kinds)
{
    if ((kinds & ~KINDS_WS) == 0) return 0;
    if ((kinds & ~KINDS_RS_OR_WS) == 0) return 1;
    return 2;
}

// normalised, order-preserving form of a Timestamp: (hi, lo, node) compared lexicographically,
// hi unsigned, lo unsigned, node signed (Timestamp.compareTo)
struct NormTid { uint64_t hi, lo; int32_t node; };

__host__ __device__ inline NormTid norm_tid(uint64_t msb, uint64_t lsb, int32_t node)
{
    NormTid t;
    t.hi = msb;
    t.lo = ((lsb >> 16) << 4) | ((lsb >> 1) & 0xF);        // lowHlc, then lsb & IDENTITY_FLAGS
    t.node = node;
    return t;
}

__host__ __device__ inline int norm_cmp(const NormTid& a, const NormTid& b)
{
    if (a.hi != b.hi) return a.hi < b.hi ? -1 : 1;
    if (a.lo != b.lo) return a.lo < b.lo ? -1 : 1;
    if (a.node != b.node) return a.node < b.node ? -1 : 1;
    return 0;
}

// Per-key record of the CommandsForKey index (one 32-byte load per probe).
struct KeyRec {
    uint32_t seg_lo, seg_hi;       // byId entries [seg_lo, seg_hi) in ent
    uint32_t w_lo, w_hi;           // committed Writes by executeAt [w_lo, w_hi) in w
    uint32_t last_txn;             // rank of byId[seg_hi-1] (0 if empty): tail fast path of insertPos
    uint32_t last_wexec;           // w[w_hi-1].x (0 if none): tail fast path of maxCommittedWriteBefore
    uint32_t pruned;               // rank of prunedBefore, 0 = NONE
    int32_t  maw;                  // absolute index into w of maxAppliedWriteByExecuteAt, -1 = none
};

// Per-probe record written by K0: {key index (NO_KEY if absent/outside the slice), S rank,
// self rank (0 = none), kinds | class << 8 | in_slice << 12}
constexpr uint32_t NO_KEY = 0xFFFFFFFFu;

// Open-addressing hash of key ordinal -> key index (one 16-byte probe per lookup, linear probing)
struct KeySlot {
    int64_t key;
    uint32_t idx;       // KEY_EMPTY = free slot
    uint32_t cell;      // the key's cell in the range stabbing index (NO_CELL: none)
};
constexpr uint32_t NO_CELL = 0xFFFFFFFFu;
constexpr uint32_t KEY_EMPTY = 0xFFFFFFFFu;

// Fused path: one 128-byte hash slot (= one cache line) per key carries the key's KeyRec and
// its emission lists: per witness class c the entries that are never elided
// (`cand`: tau = never-elided, kind in class c, byId order) and the committed Read/Write entries by
// executeAt (`cwr`, shared by the classes that witness Reads). A probe newer than the whole
// CommandsForKey (S > last txnId and S > last committed Write's executeAt) emits exactly
//   cand_c  and  { Ws: the last committed Write | RsOrWs/AnyGloballyVisible: cwr[cwr_tail, cwr_hi) }
// (minus the request's own id): the mapReduceActive loop (CommandsForKey.java:930-950) with
// end = byId.length and M = the last committed Write's executeAt.
// Indexed by key index (dense: 64 B per CommandsForKey, so hot entries pack into the caches):
// q0 the newest test + the Ws emission, q1+c the lists of witness class c. The lean kernel loads
// q0 and one class quarter; the tree path's KeyRec is the separate krec[] array.
struct KeyClassLists {
    uint32_t cand_lo, cand_hi;     // never-elided entries of class c: cand[cand_lo, cand_hi)
    uint32_t cwr_tail, cwr_hi;     // committed R/W from the last committed Write on: cwr[cwr_tail, cwr_hi)
};
struct alignas(64) KeyEntry {
    uint32_t last_txn;             // q0.x  rank of byId's last txnId (0 if empty)
    uint32_t last_wexec;           // q0.y  executeAt rank of the last committed Write (0 if none)
    uint32_t last_w_txn;           // q0.z  txn rank of that Write (0 if none)
    uint32_t pad;
    KeyClassLists cl[NCLASS];      // q1..q3
};
static_assert(sizeof(KeyEntry) == 64, "KeyEntry is half a cache line");

__host__ __device__ inline uint64_t key_hash(int64_t k)
{
    uint64_t z = (uint64_t)k + 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

// Per-store device snapshot, passed to kernels by value.
struct DevSnapshot {
    // id dictionary (normalised)
    const uint64_t* dict_hi;
    const uint64_t* dict_lo;
    const int32_t*  dict_node;
    uint64_t n_dict;
    uint64_t dict_last_hi, dict_last_lo;   // the newest dictionary id (request fast path: newer than all)
    int32_t dict_last_node;
    // CommandsForKey
    uint64_t n_keys;
    const int64_t*  keys;          // [n_keys]
    const KeyRec*   krec;          // [n_keys]
    const KeySlot*  khash;         // [khash_mask + 1]
    const KeyEntry* kent;          // [n_keys] newest-test fields + list bounds (fused kernels)
    const uint32_t* cand;          // never-elided entries per key and class: txw (rank | kind << 29)
    const uint32_t* cwr;           // committed Read/Write entries per key by executeAt: txw
    uint64_t khash_mask;
    uint64_t n_ent;
    const uint2*    ent;           // {tau, txw}
    const uint2*    w;             // committed Writes by executeAt: {exec rank, txn rank}
    const uint32_t* lvl[NCLASS][MAX_LEVELS];   // [c][l], l >= 1 (lvl[c][0] unused)
    uint64_t lvl_n[MAX_LEVELS];
    int n_levels;                  // number of levels incl. leaf
    // range commands (flattened (range, command) entries sorted by (start, end, rank))
    uint64_t n_rent;
    const int64_t*  r_start;
    const int64_t*  r_end;
    const uint32_t* r_txw;         // rank | kind << 29
    const uint32_t* r_rid;         // range id (index into the range table)
    const int64_t*  rlvl[NCLASS][MAX_LEVELS];  // max end per 64^l block
    uint64_t rlvl_n[MAX_LEVELS];
    int n_rlevels;
    // stabbing index of the range entries (null when not built): endpoints, per-cell lists
    uint64_t n_cell_E;
    const int64_t*  cell_E;        // distinct endpoints, ascending
    const uint32_t* cell_off;      // [n_cell_E + 2]
    const uint64_t* cell_ent;      // rid << 32 | txw, per cell in (Range.compare, TxnId) order
    // redundant-before (disjoint, ascending)
    uint64_t n_rb;
    const int64_t*  rb_start;
    const int64_t*  rb_end;
    const int64_t*  rb_e0;
    const int64_t*  rb_e1;
    const uint32_t* rb_wm;         // rank of shardAppliedOrInvalidatedBefore (0 = NONE / not > NONE)
    const uint32_t* rb_rid;
    // store slice
    uint64_t n_slices;
    const int64_t* slice_start;
    const int64_t* slice_end;
    int start_inclusive;
    int elide;
};

// Range.contains(key) (Range.java:40-56 EndInclusive, :84-100 StartInclusive)
__host__ __device__ inline bool range_contains(int start_inclusive, int64_t s, int64_t e, int64_t key)
{
    return start_inclusive ? (s <= key && key < e) : (s < key && key <= e);
}

}  // namespace adx
