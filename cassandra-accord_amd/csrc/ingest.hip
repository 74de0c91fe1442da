// ingest.hip — the CommandsForKey snapshot built on the device: the id dictionary
// and every entry's ranks, validated, from the raw SoA columns the caller loaded (ad_cfk_load);
// the derived arrays (cand / cwr / w lists, KeyEntry, trees) then come from the same derivation the
// device updates use (cfk_update.hip cfk_derive). Replaces the host loops of abi.cpp build_snapshot
// for a store without an installed node-wide dictionary.
//
// Reference: CommandsForKey's constructor over byId (CommandsForKey.java:642-681) with the
// invariants it asserts -- byId strictly increasing (:1438); Timestamp order / identity
// (Timestamp.java:208-217,244-249): ids equal under equals() must be bit-identical here.
//
//   1. records: every txnId, every executeAt that differs from its txnId, every extra id (range
//      command txnIds, RedundantBefore watermarks) -> normalised (hi, lo, node) + raw lsb
//   2. LSD radix sort of the record indices by node, then lo, then hi (digits constant over the
//      batch skipped: levels.hip radix_sort_pairs)
//   3. unique flags (+ the flag-bit identity check) -> scan -> dictionary member i = rank 2i+1, and
//      every record's rank
//   4. per entry: key index (search of seg), txw, executeAt rank, status / domain / byId-order checks;
//      per key: KeyRec {segment, last txnId, prunedBefore rank}, keys ascending
#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>

#include "../../include/accord_deps.h"
#include "common.hpp"
#include "ingest.hpp"
#include "kernels.hpp"
#include "levels.hpp"
#include "wave.hpp"

namespace adx {

namespace {

struct IngCtl {
    unsigned long long diff[3];    // OR of (word ^ word of record 0): node, lo, hi
    unsigned long long n_diff;     // executeAts that differ from their txnIds
    unsigned int code, pad;        // first failure (AD_E_* negated) and where
    unsigned long long bad;
};

__device__ inline void ing_fail(IngCtl* c, int code, uint64_t where)
{
    if (atomicCAS(&c->code, 0u, (unsigned)(-code)) == 0u) c->bad = where;
}

__device__ inline bool raw_eq(uint64_t am, uint64_t al, int32_t an, uint64_t bm, uint64_t bl, int32_t bn)
{
    return am == bm && al == bl && an == bn;
}

// executeAt differs from the txnId (bits): it gets a record of its own
__global__ __launch_bounds__(256) void k_ing_differs(IngestIn in, uint32_t* f)
{
    const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= in.ne) return;
    f[e] = raw_eq(in.tm[e], in.tl[e], in.tn[e], in.em[e], in.el[e], in.en[e]) ? 0u : 1u;
}

// the records: [0, ne) txnIds, [ne, ne + nd) differing executeAts (entry order), then the extras.
// Grid-stride over entries and extras (a bounded grid: one OR per block and word for the digit masks)
constexpr unsigned ING_RED_BLOCKS = 1024;
__global__ __launch_bounds__(256) void k_ing_records(IngestIn in, const uint32_t* f, const uint64_t* fpos, uint64_t nd,
                                                     IngRec r, IngCtl* ctl)
{
    __shared__ uint64_t red[3][4];
    uint64_t d0 = 0, d1 = 0, d2 = 0;
    const NormTid z = norm_tid(in.ne ? in.tm[0] : in.xm[0], in.ne ? in.tl[0] : in.xl[0], in.ne ? in.tn[0] : in.xn[0]);
    auto put = [&](uint64_t slot, uint64_t m, uint64_t l, int32_t nd_) {
        const NormTid t = norm_tid(m, l, nd_);
        r.hi[slot] = t.hi;
        r.lo[slot] = t.lo;
        r.node[slot] = t.node;
        r.lsb[slot] = l;
        d0 |= (uint64_t)((uint32_t)t.node ^ (uint32_t)z.node);
        d1 |= t.lo ^ z.lo;
        d2 |= t.hi ^ z.hi;
    };
    const uint64_t n = in.ne + in.nx;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    {
        if (i < in.ne)
        {
            put(i, in.tm[i], in.tl[i], in.tn[i]);
            if (f[i]) put(in.ne + fpos[i], in.em[i], in.el[i], in.en[i]);     // entry i's differing executeAt
        }
        else
        {
            const uint64_t x = i - in.ne;
            put(in.ne + nd + x, in.xm[x], in.xl[x], in.xn[x]);
        }
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1)
    {
        d0 |= __shfl_xor(d0, d, 64);
        d1 |= __shfl_xor(d1, d, 64);
        d2 |= __shfl_xor(d2, d, 64);
    }
    const uint32_t w = threadIdx.x >> 6;
    if (lane_id() == 0) { red[0][w] = d0; red[1][w] = d1; red[2][w] = d2; }
    __syncthreads();
    if (threadIdx.x < 3)
    {
        const uint64_t v = red[threadIdx.x][0] | red[threadIdx.x][1] | red[threadIdx.x][2] | red[threadIdx.x][3];
        if (v) atomicOr(&ctl->diff[threadIdx.x], (unsigned long long)v);
    }
}

// sort words: word 0 the node (sign flipped: signed order), 1 lo, 2 hi, of record v[i]
__global__ __launch_bounds__(256) void k_ing_word(IngRec r, const uint32_t* v, uint64_t n, int word, uint64_t* key)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t x = v ? v[i] : (uint32_t)i;
    key[i] = word == 0 ? (uint64_t)((uint32_t)r.node[x] ^ 0x80000000u) : (word == 1 ? r.lo[x] : r.hi[x]);
}

__global__ void k_iota32(uint32_t* v, uint64_t n)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) v[i] = (uint32_t)i;
}

// the records in sorted order (one gather), so that the unique test and the dictionary read them
// contiguously
__global__ __launch_bounds__(256) void k_ing_gather(IngRec r, const uint32_t* v, uint64_t n, IngRec so)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t a = v[i];
    so.hi[i] = r.hi[a];
    so.lo[i] = r.lo[a];
    so.node[i] = r.node[a];
    so.lsb[i] = r.lsb[a];
}

// sorted position i starts a new dictionary member unless it equals its predecessor (Timestamp.equals);
// equal ids must carry the same flag bits (the library's identity: AD_E_INCONSISTENT_ID)
__global__ __launch_bounds__(256) void k_ing_unique(IngRec so, const uint32_t* v, uint64_t n, uint32_t* u, IngCtl* ctl)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    bool first = i == 0;
    if (!first)
    {
        first = so.hi[i] != so.hi[i - 1] || so.lo[i] != so.lo[i - 1] || so.node[i] != so.node[i - 1];
        if (!first && so.lsb[i] != so.lsb[i - 1]) ing_fail(ctl, AD_E_INCONSISTENT_ID, v[i]);
    }
    u[i] = first ? 1u : 0u;
}

// dictionary members and every record's rank
__global__ __launch_bounds__(256) void k_ing_dict(IngRec so, const uint32_t* v, uint64_t n, const uint32_t* u,
                                                  const uint64_t* upos, IngestOut o)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t m = upos[i] + u[i] - 1;            // member index (inclusive count - 1)
    if (u[i])
    {
        o.dict_hi[m] = so.hi[i];
        o.dict_lo[m] = so.lo[i];
        o.dict_node[m] = so.node[i];
        o.dict_lsb_raw[m] = so.lsb[i];
    }
    o.rec_rank[v[i]] = (uint32_t)(2 * m + 1);
}

// per entry: its key (last key whose segment starts at or before it), txw, executeAt rank, checks
__global__ __launch_bounds__(256) void k_ing_entries(IngestIn in, const uint32_t* f, const uint64_t* fpos, IngestOut o,
                                                     IngCtl* ctl)
{
    const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= in.ne) return;
    uint64_t lo = 0, hi = in.nk + 1;                 // upper_bound(seg, e) - 1
    while (lo < hi)
    {
        const uint64_t mid = (lo + hi) >> 1;
        if (in.seg[mid] <= e) lo = mid + 1;
        else hi = mid;
    }
    const uint32_t k = (uint32_t)(lo - 1);
    const uint32_t st = in.status[e];
    const uint64_t l = in.tl[e];
    const uint32_t kind = (uint32_t)((l >> 1) & 7), dom = (uint32_t)(l & 1);
    const uint32_t tr = o.rec_rank[e];
    const uint32_t xr = f[e] ? o.rec_rank[in.ne + fpos[e]] : tr;
    if (st > 7) ing_fail(ctl, AD_E_INVAL, k);
    else if (dom && !(st == AD_ST_TRANSITIVELY_KNOWN || st == AD_ST_INVALID_OR_TRUNCATED_OR_UNMANAGED_COMMITTED))
        ing_fail(ctl, AD_E_INVAL, k);                // a live range-domain id in a CommandsForKey
    if (e > in.seg[k] && tr <= o.rec_rank[e - 1]) ing_fail(ctl, AD_E_ORDER, k);   // CommandsForKey.java:1438
    o.ent[e] = make_uint2(0u, tr | (kind << RANK_BITS));
    o.xrank[e] = xr;
    o.ekey[e] = k;
}

__global__ __launch_bounds__(256) void k_ing_keys(IngestIn in, IngestOut o, IngCtl* ctl)
{
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= in.nk) return;
    if (k > 0 && in.keys[k - 1] >= in.keys[k]) ing_fail(ctl, AD_E_INVAL, k);
    KeyRec r{};
    r.seg_lo = (uint32_t)in.seg[k];
    r.seg_hi = (uint32_t)in.seg[k + 1];
    r.last_txn = r.seg_hi > r.seg_lo ? o.rec_rank[r.seg_hi - 1] : 0u;
    r.maw = -1;
    if (in.pruned && in.pruned[k] >= 0)
    {
        const uint64_t idx = r.seg_lo + (uint64_t)in.pruned[k];
        if (idx >= r.seg_hi) ing_fail(ctl, AD_E_STATE, k);      // prunedBefore not in byId
        else r.pruned = o.rec_rank[idx];
    }
    o.krec[k] = r;
}

// per key: its cell in the range stabbing index (cell(x) = #endpoints < x, or <= x StartInclusive)
__global__ __launch_bounds__(256) void k_ing_kcell(const int64_t* keys, uint64_t nk, const int64_t* cell_E, uint64_t m,
                                                   int start_inclusive, uint32_t* kcell)
{
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nk) return;
    const int64_t x = keys[k];
    uint32_t c = NO_CELL;
    if (cell_E)
    {
        uint64_t lo = 0, hi = m;
        while (lo < hi)
        {
            const uint64_t mid = (lo + hi) >> 1;
            if (start_inclusive ? cell_E[mid] <= x : cell_E[mid] < x) lo = mid + 1;
            else hi = mid;
        }
        c = (uint32_t)lo;
    }
    kcell[k] = c;
}

__global__ __launch_bounds__(256) void k_ing_khash_clear(KeySlot* h, uint64_t n)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) h[i] = KeySlot{0, KEY_EMPTY, NO_CELL};
}

// open addressing, linear probing: a key claims the first free slot from its hash (CAS on the index)
__global__ __launch_bounds__(256) void k_ing_khash_fill(const int64_t* keys, uint64_t nk, const uint32_t* kcell, KeySlot* h,
                                                        uint64_t hcap)
{
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nk) return;
    const int64_t key = keys[k];
    const uint64_t mask = hcap - 1;
    uint64_t i = key_hash(key) & mask;
    while (atomicCAS(&h[i].idx, KEY_EMPTY, (uint32_t)k) != KEY_EMPTY) i = (i + 1) & mask;
    h[i].key = key;
    h[i].cell = kcell[k];
}

unsigned nblk(uint64_t n) { return (unsigned)std::max<uint64_t>(1, (n + 255) / 256); }

uint32_t digits(uint64_t diff)
{
    uint32_t m = 0;
    for (int d = 0; d < 8; ++d)
        if ((diff >> (8 * d)) & 0xFF) m |= 1u << d;
    return m;
}

}  // namespace

struct IngestWork {
    IngDBuf ctl, f, fpos, bsum, hi, lo, node, lsb, ka, kb, va, vb, hist, hoff, u, upos, so_node, so_lsb;
    IngCtl* h_ctl = nullptr;
    ~IngestWork()
    {
        if (h_ctl) (void)hipHostFree(h_ctl);
    }
};

IngestWork* ingest_work_create() { return new IngestWork(); }
void ingest_work_destroy(IngestWork* w) { delete w; }

#define ICHK(expr)                                                                                \
    do {                                                                                          \
        hipError_t _e = (expr);                                                                   \
        if (_e != hipSuccess) { *err = std::string(#expr) + ": " + hipGetErrorString(_e); return AD_E_DEVICE; } \
    } while (0)
#define IALLOC(buf, bytes)                                                                        \
    do {                                                                                          \
        if (!(buf).ensure(bytes)) { *err = "device allocation (ingest)"; return AD_E_NOMEM; }     \
    } while (0)

uint64_t ingest_records(const IngestIn& in) { return 2 * in.ne + in.nx; }

int ingest_dictionary(IngestWork* w, const IngestIn& in, IngestOut& o, hipStream_t st, uint64_t* n_dict, uint64_t* bad,
                      std::string* err)
{
    const uint64_t ne = in.ne;
    IALLOC(w->ctl, sizeof(IngCtl));
    IngCtl* ctl = w->ctl.as<IngCtl>();
    if (!w->h_ctl) ICHK(hipHostMalloc((void**)&w->h_ctl, sizeof(IngCtl), hipHostMallocDefault));
    ICHK(hipMemsetAsync(ctl, 0, sizeof(IngCtl), st));
    // 1. which executeAts need records of their own, then all records
    IALLOC(w->f, 4 * std::max<uint64_t>(ne, 1));
    IALLOC(w->fpos, 8 * (ne + 1));
    IALLOC(w->bsum, 8 * ((std::max<uint64_t>(2 * ne + in.nx, 1) + 1023) / 1024 * 4 + radix_hist_entries(2 * ne + in.nx + 1) / 1024 + 64));
    if (ne) k_ing_differs<<<nblk(ne), 256, 0, st>>>(in, w->f.as<uint32_t>());
    ICHK(run_scan_arrays(w->f.as<uint32_t>(), w->fpos.as<uint64_t>(), ne, 1, w->bsum.as<uint64_t>(), st));
    ICHK(hipMemcpyAsync(&ctl->n_diff, w->fpos.as<uint64_t>() + ne, 8, hipMemcpyDeviceToDevice, st));
    ICHK(d2h(w->h_ctl, ctl, sizeof(IngCtl), st));
    ICHK(hipStreamSynchronize(st));
    const uint64_t nd = w->h_ctl->n_diff, n = ne + nd + in.nx;
    IALLOC(w->hi, 8 * std::max<uint64_t>(n, 1));
    IALLOC(w->lo, 8 * std::max<uint64_t>(n, 1));
    IALLOC(w->node, 4 * std::max<uint64_t>(n, 1));
    IALLOC(w->lsb, 8 * std::max<uint64_t>(n, 1));
    IngRec r{w->hi.as<uint64_t>(), w->lo.as<uint64_t>(), w->node.as<int32_t>(), w->lsb.as<uint64_t>()};
    if (n) k_ing_records<<<std::min<unsigned>(nblk(ne + in.nx), ING_RED_BLOCKS), 256, 0, st>>>(in, w->f.as<uint32_t>(), w->fpos.as<uint64_t>(), nd, r, ctl);
    ICHK(hipGetLastError());
    ICHK(d2h(w->h_ctl, ctl, sizeof(IngCtl), st));
    ICHK(hipStreamSynchronize(st));
    // 2. LSD over node, lo, hi (digits that vary only)
    IALLOC(w->ka, 8 * std::max<uint64_t>(n, 1));
    IALLOC(w->kb, 8 * std::max<uint64_t>(n, 1));
    IALLOC(w->va, 4 * std::max<uint64_t>(n, 1));
    IALLOC(w->vb, 4 * std::max<uint64_t>(n, 1));
    const uint64_t hn = radix_hist_entries(std::max<uint64_t>(n, 1));
    IALLOC(w->hist, 4 * hn);
    IALLOC(w->hoff, 8 * (hn + 1));
    uint64_t* kcur = w->ka.as<uint64_t>();
    uint32_t* vcur = w->va.as<uint32_t>();
    if (n) k_iota32<<<nblk(n), 256, 0, st>>>(vcur, n);
    for (int word = 0; word < 3; ++word)
    {
        const uint32_t dm = digits(w->h_ctl->diff[word]);
        if (!dm || n < 2) continue;
        k_ing_word<<<nblk(n), 256, 0, st>>>(r, vcur, n, word, kcur);
        uint64_t* kt = kcur == w->ka.as<uint64_t>() ? w->kb.as<uint64_t>() : w->ka.as<uint64_t>();
        uint32_t* vt = vcur == w->va.as<uint32_t>() ? w->vb.as<uint32_t>() : w->va.as<uint32_t>();
        ICHK(radix_sort_pairs(kcur, vcur, kt, vt, n, dm, w->hist.as<uint32_t>(), w->hoff.as<uint64_t>(), w->bsum.as<uint64_t>(),
                              st, &kcur, &vcur));
    }
    // 3. members and ranks
    IALLOC(w->u, 4 * std::max<uint64_t>(n, 1));
    IALLOC(w->upos, 8 * (n + 1));
    // sorted copies of the records: the radix key buffers are free now (n x 8 B each) plus two more
    IALLOC(w->so_node, 4 * std::max<uint64_t>(n, 1));
    IALLOC(w->so_lsb, 8 * std::max<uint64_t>(n, 1));
    uint64_t* so_hi = kcur == w->ka.as<uint64_t>() ? w->kb.as<uint64_t>() : w->ka.as<uint64_t>();
    uint64_t* so_lo = kcur;
    IngRec so{so_hi, so_lo, w->so_node.as<int32_t>(), w->so_lsb.as<uint64_t>()};
    if (n) k_ing_gather<<<nblk(n), 256, 0, st>>>(r, vcur, n, so);
    if (n) k_ing_unique<<<nblk(n), 256, 0, st>>>(so, vcur, n, w->u.as<uint32_t>(), ctl);
    ICHK(run_scan_arrays(w->u.as<uint32_t>(), w->upos.as<uint64_t>(), n, 1, w->bsum.as<uint64_t>(), st));
    if (n) k_ing_dict<<<nblk(n), 256, 0, st>>>(so, vcur, n, w->u.as<uint32_t>(), w->upos.as<uint64_t>(), o);
    ICHK(hipGetLastError());
    uint64_t nm = 0;
    ICHK(d2h(w->h_ctl, ctl, sizeof(IngCtl), st));
    ICHK(d2h(&nm, w->upos.as<uint64_t>() + n, 8, st));
    ICHK(hipStreamSynchronize(st));
    *n_dict = nm;
    o.n_diff = nd;
    if (w->h_ctl->code)
    {
        *bad = w->h_ctl->bad;
        *err = "ids equal under Timestamp.equals differ in flag bits";
        return -(int)w->h_ctl->code;
    }
    return AD_OK;
}

int ingest_entries(IngestWork* w, const IngestIn& in, const IngestOut& o, hipStream_t st, uint64_t* bad, std::string* err)
{
    IngCtl* ctl = w->ctl.as<IngCtl>();
    ICHK(hipMemsetAsync(ctl, 0, sizeof(IngCtl), st));
    if (in.ne) k_ing_entries<<<nblk(in.ne), 256, 0, st>>>(in, w->f.as<uint32_t>(), w->fpos.as<uint64_t>(), o, ctl);
    if (in.nk) k_ing_keys<<<nblk(in.nk), 256, 0, st>>>(in, o, ctl);
    ICHK(hipGetLastError());
    ICHK(d2h(w->h_ctl, ctl, sizeof(IngCtl), st));
    ICHK(hipStreamSynchronize(st));
    if (w->h_ctl->code)
    {
        const int code = -(int)w->h_ctl->code;
        *bad = w->h_ctl->bad;
        *err = code == AD_E_ORDER ? "byId strict order (CommandsForKey.java:1438)"
               : code == AD_E_STATE ? "prunedBefore is not in byId"
                                    : "status range / key-domain ids / keys ascending";
        return code;
    }
    return AD_OK;
}

hipError_t ingest_keys(const int64_t* keys, uint64_t nk, const int64_t* cell_E, uint64_t n_cell_E, int start_inclusive,
                       uint32_t* kcell, KeySlot* khash, uint64_t hcap, hipStream_t st)
{
    k_ing_khash_clear<<<nblk(hcap), 256, 0, st>>>(khash, hcap);
    if (nk)
    {
        k_ing_kcell<<<nblk(nk), 256, 0, st>>>(keys, nk, cell_E, n_cell_E, start_inclusive, kcell);
        k_ing_khash_fill<<<nblk(nk), 256, 0, st>>>(keys, nk, kcell, khash, hcap);
    }
    return hipGetLastError();
}

}  // namespace adx
