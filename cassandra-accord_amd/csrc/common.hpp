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

// The lean kernels' per-key record: one 128-byte line (one L2 line) per key in a table indexed by a
// perfect hash of the key ordinal (kl_index), so a (request, key) probe costs one random line: the
// key test, the newest test, the emission counts and -- for keys whose emissions fit -- the
// emissions themselves.
//   [0, 8)    key
//   [8, 16)   the key's entries in the range stabbing index: cell_ent[cell_lo, cell_hi)
//   [16, 28)  last txnId rank, last committed Write's executeAt rank and txnId rank (0: none)
//   [28, 32)  meta: KL_USED | KL_INLINE | KL_NOLEAN | inline offset of the cwr tail << 24 | KL_CELLINL |
//             inline u64 offset of the stabbing-cell entries << 20 | #cwr tail
//   [32, 56)  per witness class c: {#never-elided entries of class c, their start in cand}
//   [56, 64)  start of the cwr tail in cwr, rank of prunedBefore (0: none)
//   [64, 128) inline emissions when #class-2 entries + #cwr tail <= KL_INL: the never-elided
//             entries nested by class -- Writes, then Reads, then SyncPoints/ExclusiveSyncPoints
//             (class c's list is the first n_c of them) -- then the cwr tail; then, when they fit
//             (KL_CELLINL), the key's stabbing-cell entries (rid << 32 | txw, u64-aligned) -- a range
//             probe then reads them from the line it already has instead of a line of cell_ent
struct KeyClassSpan { uint32_t n, base; };
struct alignas(128) KeyLine {
    int64_t key;
    uint32_t cell_lo, cell_hi;
    uint32_t last_txn, last_wexec, last_w_txn, meta;
    KeyClassSpan cls[NCLASS];
    uint32_t cwr_tail, pruned;
    uint32_t inl[16];
};
static_assert(sizeof(KeyLine) == 128, "KeyLine is one cache line");
constexpr uint32_t KL_INL = 16;
constexpr uint32_t KL_USED = 1u << 31;
constexpr uint32_t KL_INLINE = 1u << 30;
constexpr uint32_t KL_NOLEAN = 1u << 29;          // counts beyond the meta fields: the general kernel serves it
constexpr uint32_t KL_NCWR_MASK = (1u << 20) - 1;
constexpr uint32_t KL_CELLINL = 1u << 23;         // the cell entries are inline, at u64 offset (meta >> 20) & 7
constexpr uint32_t KL_CELL_SHIFT = 20;
constexpr uint32_t KL_INL_SHIFT = 24;             // 5 bits (<= KL_INL)

// Per key line, beside its KeyLine (same perfect-hash index): what one (request, key) probe of witness
// class c needs in one 16-byte load -- {thr, counts, base1, base2}: the request is served lean iff
// S > thr (thr = max(last committed Write's executeAt, prunedBefore) ranks; ~0 when the lean path cannot
// serve the key), its raw emissions are n1 = counts & 0x7F entries at base1 (class c's never-elided list)
// then n2 = (counts >> 8) & 0x7F at base2 (class Ws: the last committed Write itself, base2 being its txw;
// else the cwr tail); LQ_INLINE: both runs are word indices into the KeyLine table (its inline part) instead
// of cand / cwr. key / used: the slot's key (k_prepare's membership test).
constexpr uint32_t LQ_INLINE = 1u << 16;
constexpr uint32_t LQ_NMAX = 0x7F;
struct alignas(64) LeanQuads {
    uint4 q[NCLASS];
    int64_t key;
    uint32_t used, pad;
};
static_assert(sizeof(LeanQuads) == 64, "LeanQuads is half a cache line");

__host__ __device__ inline uint64_t key_hash(int64_t k)
{
    uint64_t z = (uint64_t)k + 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

// Perfect hash of a snapshot's keys onto KeyLine indices (hash and displace): key k lives at
// kl_index(key_hash2(k), disp[kl_bucket(key_hash(k))]); the displacements are chosen at ingest so
// that no two keys share a line. One small (cache-resident) lookup, then exactly one line.
__host__ __device__ inline uint64_t key_hash2(int64_t k)
{
    uint64_t z = (uint64_t)k ^ 0xD1B54A32D192ED03ULL;
    z = (z ^ (z >> 33)) * 0xFF51AFD7ED558CCDULL;
    z = (z ^ (z >> 33)) * 0xC4CEB9FE1A85EC53ULL;
    return z ^ (z >> 33);
}
__host__ __device__ inline uint64_t mulhi64(uint64_t a, uint64_t b)
{
#ifdef __HIP_DEVICE_COMPILE__
    return __umul64hi(a, b);
#else
    return (uint64_t)(((unsigned __int128)a * b) >> 64);
#endif
}
__host__ __device__ inline uint64_t kl_bucket(uint64_t h, uint64_t n_buckets) { return mulhi64(h, n_buckets); }
__host__ __device__ inline uint64_t kl_index(uint64_t g, uint32_t d, uint64_t n_lines)
{
    return mulhi64(g ^ ((uint64_t)d * 0x9E3779B97F4A7C15ULL), n_lines);
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
    // every DICT_SAMP-th dictionary id (cache-resident): a rank search touches HBM only inside one
    // DICT_SAMP-id window of the dictionary
    // (n_samp entries), then from entry dict_samp2_base(n_samp) every DICT_SAMP2-th id (n_samp2
    // entries, 0 = none): a search then reads one 16-id window of that level and one of the dictionary
    const uint64_t* ds_hi;
    const uint64_t* ds_lo;
    const int32_t*  ds_node;
    uint64_t n_samp, n_samp2;
    // bucket index over the first sample level (dict_bucket; nullptr = none): DB_HDR header words, then
    // 2^lg + 1 bucket starts
    const uint32_t* ds_bkt;
    // CommandsForKey
    uint64_t n_keys;
    const int64_t*  keys;          // [n_keys]
    const KeyRec*   krec;          // [n_keys]
    const KeySlot*  khash;         // [khash_mask + 1]
    const KeyEntry* kent;          // [n_keys] newest-test fields + list bounds (fused kernels)
    const KeyLine*  kline;         // [kl_lines] the lean kernels' per-key lines (perfect hash)
    const LeanQuads* kquad;        // [kl_lines] beside them: per class the probe's 16 bytes, the key
    const uint32_t* kl_disp;       // [kl_buckets] displacements
    uint64_t kl_lines, kl_buckets;
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
    // per-request slices (ad_slice_sets_load): set k = [sset_start, sset_end)[sset_off[k], sset_off[k + 1])
    uint64_t n_ssets;
    const uint64_t* sset_off;
    const int64_t* sset_start;
    const int64_t* sset_end;
    int start_inclusive;
    int elide;
    // range ids below 2^26 and id ranks below 2^26: the lean kernels' rangeDeps build sorts 32-bit keys
    // (range id << 6 | lane, rank << 6 | pair) instead of 64-bit (range id << 32 | rank, rank << 8 | pair)
    int rng32;
};

constexpr uint64_t DICT_SAMP = 256, DICT_SAMP2 = 16;
inline uint64_t dict_samples(uint64_t n_dict) { return (n_dict + DICT_SAMP - 1) / DICT_SAMP; }
inline uint64_t dict_samples2(uint64_t n_dict) { return (n_dict + DICT_SAMP2 - 1) / DICT_SAMP2; }
// start of the second level in the sample arrays: a whole number of 16-entry (128-byte) windows in
__host__ __device__ inline uint64_t dict_samp2_base(uint64_t n_samp) { return (n_samp + DICT_SAMP2 - 1) & ~(DICT_SAMP2 - 1); }
// entries of the sample arrays (both levels) for a dictionary of n_dict ids
inline uint64_t dict_sample_entries(uint64_t n_dict) { return dict_samp2_base(dict_samples(n_dict)) + dict_samples2(n_dict); }

// First index i in [a, b) where the monotone predicate pred(k, i) (true ... true false ... false) is false
// (b when there is none), for N independent binary searches of one thread advanced in lockstep: their
// loads of a round go out together, so an Accept's two ids cost one chain of round trips instead of two.
// A finished (or unwanted) search evaluates index 0 (the arrays are non-empty when any search runs) and
// keeps its bounds. (Measured: three pivots per round -- a quaternary search -- made k_prepare slower on the
// request mix, 0.18 -> 0.21 ms: it is bound by the lines it reads as much as by the chain.)
#ifndef DICT_PIVOTS
#define DICT_PIVOTS 1
#endif
template <int N, class Pred>
__device__ inline void lockstep_partition(uint64_t (&a)[N], uint64_t (&b)[N], Pred pred)
{
    for (;;)
    {
        bool any = false;
#pragma unroll
        for (int k = 0; k < N; ++k) any = any || a[k] < b[k];
        if (!any) return;
        if (DICT_PIVOTS == 3)
        {
            // quaternary rounds (three pivots per search; measurement switch)
            uint64_t p1[N], p2[N], p3[N];
            bool c1[N], c2[N], c3[N];
#pragma unroll
            for (int k = 0; k < N; ++k)
            {
                const bool on = a[k] < b[k];
                const uint64_t len = on ? b[k] - a[k] : 0;
                p1[k] = on ? a[k] + (len >> 2) : 0;
                p2[k] = on ? a[k] + (len >> 1) : 0;
                p3[k] = on ? a[k] + ((3 * len) >> 2) : 0;
            }
#pragma unroll
            for (int k = 0; k < N; ++k)
            {
                c1[k] = pred(k, p1[k]);
                c2[k] = pred(k, p2[k]);
                c3[k] = pred(k, p3[k]);
            }
#pragma unroll
            for (int k = 0; k < N; ++k)
            {
                const bool on = a[k] < b[k];
                const uint64_t na = c3[k] ? p3[k] + 1 : (c2[k] ? p2[k] + 1 : (c1[k] ? p1[k] + 1 : a[k]));
                const uint64_t nb = c3[k] ? b[k] : (c2[k] ? p3[k] : (c1[k] ? p2[k] : p1[k]));
                a[k] = on ? na : a[k];
                b[k] = on ? nb : b[k];
            }
            continue;
        }
        uint64_t m[N];
        bool c[N];
#pragma unroll
        for (int k = 0; k < N; ++k) m[k] = a[k] < b[k] ? (a[k] + b[k]) >> 1 : 0;
#pragma unroll
        for (int k = 0; k < N; ++k) c[k] = pred(k, m[k]);
#pragma unroll
        for (int k = 0; k < N; ++k)
        {
            const bool on = a[k] < b[k];
            a[k] = on && c[k] ? m[k] + 1 : a[k];
            b[k] = on && !c[k] ? m[k] : b[k];
        }
    }
}

// The first sample level's bucket index (round 6): bucket f(t) = min((t - first) >> shift, 2^lg - 1) over the
// 128-bit (hi, lo) of a normalised id (0 below the first), monotone in the id order, so the samples <= t number
// between start[f(t)] (the samples of lower buckets) and start[f(t) + 1]. A rank search reads its bucket's two
// starts (one line) and searches only the samples between them -- instead of ~16 rounds of binary search over
// all of them (each an L2 round trip). Header: first id's hi (2 words), lo (2), shift, lg, n_samp built for.
constexpr uint32_t DB_HDR = 8;
__host__ __device__ inline uint32_t bitlen128(uint64_t hi, uint64_t lo)
{
    return hi ? 128u - (uint32_t)__builtin_clzll(hi) : (lo ? 64u - (uint32_t)__builtin_clzll(lo) : 0u);
}
__host__ __device__ inline uint32_t dict_bucket_of(uint64_t mh, uint64_t ml, uint32_t sh, uint32_t lg, uint64_t hi, uint64_t lo)
{
    if (hi < mh || (hi == mh && lo < ml)) return 0;
    const unsigned __int128 d = ((((unsigned __int128)hi << 64) | lo) - (((unsigned __int128)mh << 64) | ml)) >> sh;
    const uint64_t nb = 1ull << lg;
    return d >= nb ? (uint32_t)(nb - 1) : (uint32_t)d;
}

// Ranks of up to N arbitrary ids in the dictionary (member i -> 2i+1, else 2 * lower bound; above every
// member: 2 * n_dict without a load), searched in lockstep (lockstep_partition): the first-level sample, then the
// second-level window of it, then one DICT_SAMP2-id window of the dictionary. want[k] false: r[k] = 0.
template <int N, class Snap>
__device__ inline void dict_rank_sampled_n(const Snap& s, const NormTid (&t)[N], const bool (&want)[N], uint32_t (&r)[N])
{
    const NormTid last{s.dict_last_hi, s.dict_last_lo, s.dict_last_node};
    bool act[N];
    uint64_t a[N], b[N];
#pragma unroll
    for (int k = 0; k < N; ++k)
    {
        r[k] = 0;
        act[k] = want[k] && s.n_dict != 0;
        if (act[k])
        {
            const int cl = norm_cmp(last, t[k]);
            if (cl < 0) { r[k] = (uint32_t)(2 * s.n_dict); act[k] = false; }
            else if (cl == 0) { r[k] = (uint32_t)(2 * s.n_dict - 1); act[k] = false; }
        }
        a[k] = 0;
        b[k] = act[k] ? s.n_samp : 0;
    }
    bool any = false;
#pragma unroll
    for (int k = 0; k < N; ++k) any = any || act[k];
    if (s.ds_bkt && any)
    {
        // the bucket's samples only (dict_bucket_of; the header words are the same for every thread)
        const uint32_t* B = s.ds_bkt;
        const uint64_t mh = B[0] | ((uint64_t)B[1] << 32), ml = B[2] | ((uint64_t)B[3] << 32);
        const uint32_t sh = B[4], lg = B[5];
#pragma unroll
        for (int k = 0; k < N; ++k)
        {
            const uint32_t f = act[k] ? dict_bucket_of(mh, ml, sh, lg, t[k].hi, t[k].lo) : 0u;
            const uint2 ab = act[k] ? make_uint2(B[DB_HDR + f], B[DB_HDR + f + 1]) : make_uint2(0, 0);
            a[k] = ab.x;
            b[k] = ab.y;
        }
    }
    // first level: the samples <= t
    lockstep_partition<N>(a, b, [&](int k, uint64_t m) {
        const NormTid d{s.ds_hi[m], s.ds_lo[m], s.ds_node[m]};
        return norm_cmp(d, t[k]) <= 0;
    });
    uint64_t lo[N], hi[N], j0[N], j1[N];
    const uint64_t base = dict_samp2_base(s.n_samp);
#pragma unroll
    for (int k = 0; k < N; ++k)
    {
        lo[k] = a[k] ? (a[k] - 1) * DICT_SAMP : 0;
        hi[k] = a[k] < s.n_samp ? a[k] * DICT_SAMP : s.n_dict;
        // second level: the samples j*DICT_SAMP2 inside [lo, hi) -- one 128-byte window of hi / lo words
        // -- narrow the window to DICT_SAMP2 ids (pos in [(c-1)*DICT_SAMP2, c*DICT_SAMP2] for c = the
        // samples <= t; all of them <= t: pos <= hi as before)
        j0[k] = lo[k] / DICT_SAMP2;
        j1[k] = min((hi[k] + DICT_SAMP2 - 1) / DICT_SAMP2, s.n_samp2);
        a[k] = j0[k];
        b[k] = act[k] && s.n_samp2 ? j1[k] : j0[k];
    }
    lockstep_partition<N>(a, b, [&](int k, uint64_t m) {
        const NormTid d{s.ds_hi[base + m], s.ds_lo[base + m], s.ds_node[base + m]};
        return norm_cmp(d, t[k]) <= 0;
    });
#pragma unroll
    for (int k = 0; k < N; ++k)
    {
        if (act[k] && s.n_samp2)
        {
            if (a[k] > j0[k]) lo[k] = (a[k] - 1) * DICT_SAMP2;
            if (a[k] < j1[k]) hi[k] = a[k] * DICT_SAMP2;
        }
        a[k] = lo[k];
        b[k] = act[k] ? hi[k] : lo[k];
    }
    // the window: lower bound of t (the three words of a probe loaded together)
    lockstep_partition<N>(a, b, [&](int k, uint64_t m) {
        const NormTid d{s.dict_hi[m], s.dict_lo[m], s.dict_node[m]};
        return norm_cmp(d, t[k]) < 0;
    });
#pragma unroll
    for (int k = 0; k < N; ++k)
    {
        const uint64_t e = act[k] && a[k] < s.n_dict ? a[k] : 0;
        const NormTid d{s.dict_hi[e], s.dict_lo[e], s.dict_node[e]};
        const bool eq = act[k] && a[k] < s.n_dict && norm_cmp(d, t[k]) == 0;
        r[k] = act[k] ? (uint32_t)(2 * a[k] + (eq ? 1 : 0)) : r[k];
    }
}

// Rank of one arbitrary id (dict_rank_sampled_n with N = 1)
template <class Snap>
__device__ inline uint32_t dict_rank_sampled(const Snap& s, const NormTid& t)
{
    const NormTid tt[1] = {t};
    const bool w[1] = {true};
    uint32_t r[1];
    dict_rank_sampled_n<1>(s, tt, w, r);
    return r[0];
}

// Range.contains(key) (Range.java:40-56 EndInclusive, :84-100 StartInclusive)
__host__ __device__ inline bool range_contains(int start_inclusive, int64_t s, int64_t e, int64_t key)
{
    return start_inclusive ? (s <= key && key < e) : (s < key && key <= e);
}

// The Ranges a request's scan is sliced to -- SafeCommandStore.mapReduceActive's `slice`
// (SafeCommandStore.java:292): PreAccept / Accept / GetDeps pass safeStore.ranges().allBetween(minUnsyncedEpoch,
// txnId | executeAt) (PreAccept.java:100,130, Accept.java:115, CommandStores.java:233-242), which differs by epoch
// during a topology change. A request names one of the store's slice sets (ad_query_soa.slice_set,
// ad_slice_sets_load), or SLICE_STORE: the store's own slices (ad_config; none = every key).
constexpr uint32_t SLICE_STORE = 0xFFFFFFFFu;
struct SliceView {
    const int64_t* st;
    const int64_t* en;
    uint64_t n;
    bool all;          // no slicing: every key
};
__device__ __forceinline__ SliceView request_slice(const DevSnapshot& s, const uint32_t* sset, uint64_t t)
{
    const uint32_t k = sset ? sset[t] : SLICE_STORE;
    if (k == SLICE_STORE) return SliceView{s.slice_start, s.slice_end, s.n_slices, s.n_slices == 0};
    if (k >= s.n_ssets) return SliceView{nullptr, nullptr, 0, false};       // rejected (ERR_SLICE): no key
    const uint64_t a = s.sset_off[k];
    return SliceView{s.sset_start + a, s.sset_end + a, s.sset_off[k + 1] - a, false};
}
// Ranges.contains(key) of the slice (InMemoryCommandStore.java:280)
__device__ __forceinline__ bool slice_has(int start_inclusive, const SliceView& v, int64_t key)
{
    if (v.all) return true;
    for (uint64_t i = 0; i < v.n; ++i)
        if (range_contains(start_inclusive, v.st[i], v.en[i], key)) return true;
    return false;
}

}  // namespace adx
