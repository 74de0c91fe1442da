// exchange.hip — multi-GPU path: export of one CommandStore's per-request
// PartialDeps for an all-to-all over RCCL, and K3, the on-GPU merge of the partials a GPU
// receives for the requests it owns.
//
// The merge is PartialDeps.with (PartialDeps.java:73-81) folded over the stores in slice order,
// as CommandStores.mapReduce reduces per-store results (CommandStores.java:576-593,
// PreAccept.reduce PreAccept.java:140-156). Slices are disjoint and ascending, so each map's
// keys concatenate in source order; the TxnId lists need a union: RelationMultiMap.linearUnion
// (RelationMultiMap.java:561-816) restated as a rank computation — the union index of an id x is
//     u(x) = sum over parts q of ( lb_q(x) - dupsBefore_q(lb_q(x)) )
// where lb_q is the lower bound of x in part q's (sorted, unique) id list and an element is a
// dup when an earlier part of the same request holds an equal id (Timestamp.equals). Each
// distinct id is counted once, in the first part holding it, so u is the id's position in the
// sorted union, and every copy of an id maps to the same u (keysToTxnIds remap for free).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "../../include/accord_deps.h"
#include "common.hpp"
#include "exchange.hpp"
#include "kernels.hpp"
#include "wave.hpp"

namespace adx {

namespace {

constexpr int XWAVES = 4;              // waves per block
constexpr uint32_t DUP_BIT = 0x80000000u;

struct Tid3 { uint64_t msb, lsb; int32_t node; };

__device__ __forceinline__ Tid3 load_tid(const int64_t* ids, uint64_t i)
{
    const int64_t* p = ids + 3 * i;
    return Tid3{(uint64_t)p[0], (uint64_t)p[1], (int32_t)p[2]};
}

__device__ __forceinline__ int tid_cmp3(const Tid3& a, const Tid3& b)
{
    return norm_cmp(norm_tid(a.msb, a.lsb, a.node), norm_tid(b.msb, b.lsb, b.node));
}

// first i in [0, n) with !(ids[base + i] < x)
__device__ __forceinline__ uint32_t lb_tid(const int64_t* ids, uint64_t base, uint32_t n, const Tid3& x)
{
    uint32_t lo = 0, hi = n;
    while (lo < hi)
    {
        const uint32_t mid = (lo + hi) >> 1;
        if (tid_cmp3(load_tid(ids, base + mid), x) < 0) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// ---------------------------------------------------------------------------------------
// export
// ---------------------------------------------------------------------------------------
// per request: number of non-empty maps (its parts); the part index is their exclusive scan
__global__ void k_export_sizes(ExportArgs a)
{
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= a.n) return;
    uint32_t live = 0;
#pragma unroll
    for (int m = 0; m < 3; ++m) live += a.keys_off[m][r + 1] > a.keys_off[m][r] ? 1u : 0u;
    a.sz[r] = live;
}

// offsets of request r's first part in the four transport arrays: the part scan, and for key
// words / ids / k2t the sums of the three maps' packed CSR offsets (maps are exported in order)
struct PartBase { uint64_t P, KW, ID, KO; };

__device__ __forceinline__ PartBase part_base(const ExportArgs& a, uint64_t r)
{
    PartBase b{a.off[r], 0, 0, 0};
#pragma unroll
    for (int m = 0; m < 3; ++m)
    {
        b.KW += (m == AD_MAP_RANGE ? 2 : 1) * a.keys_off[m][r];
        b.ID += a.txn_off[m][r];
        b.KO += a.k2t_off[m][r];
    }
    return b;
}

// Export by request groups: G lanes per request copy its parts' key words, ids and keysToTxnIds
// lane-strided (a part's elements are contiguous at both ends), with no block scans, LDS or owner searches --
// parts are small (a store's share of a request: a few keys, tens of ids), so a load-balanced copy over
// blocks of 128 requests (round 2's k_export_tiles: per-element owner search, block-wide barriers) cost more
// than the copy (1.11 against 0.77 ms for the W = 8 node's exports; deleted in round 6).
// Every lane of a group reads the request's offsets (same addresses: one line per group).
template <uint32_t G>
__global__ void __launch_bounds__(256) k_export_groups(ExportArgs a)
{
    const uint64_t r = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / G;
    const uint32_t sl = threadIdx.x % G;
    if (r >= a.n) return;                                 // whole groups (G divides the block)
    const bool kept = r >= a.self_lo && r < a.self_hi;
    int64_t* hdr = kept ? a.rhdr + 4 * a.self_delta[0] : a.hdr;
    int64_t* okeys = kept ? a.rkeys + a.self_delta[1] : a.okeys;
    int64_t* oids = kept ? a.rids + (a.rank_ids ? 0 : 3 * a.self_delta[2]) : a.oids;
    uint32_t* oids32 = reinterpret_cast<uint32_t*>(kept ? a.rids : a.oids) + (kept && a.rank_ids ? a.self_delta[2] : 0);
    int32_t* ok2t = kept ? a.rk2t + a.self_delta[3] : a.ok2t;
    uint64_t k0[3], t0[3], o0[3];
    uint32_t nk[3], nt[3], no[3];
#pragma unroll
    for (int m = 0; m < 3; ++m)
    {
        k0[m] = a.keys_off[m][r];
        nk[m] = (uint32_t)(a.keys_off[m][r + 1] - k0[m]);
        t0[m] = a.txn_off[m][r];
        nt[m] = (uint32_t)(a.txn_off[m][r + 1] - t0[m]);
        o0[m] = a.k2t_off[m][r];
        no[m] = (uint32_t)(a.k2t_off[m][r + 1] - o0[m]);
    }
    uint64_t P = a.off[r], KW = 0, ID = 0, KO = 0;
#pragma unroll
    for (int m = 0; m < 3; ++m)
    {
        KW += (m == AD_MAP_RANGE ? 2 : 1) * k0[m];
        ID += t0[m];
        KO += o0[m];
    }
    const int64_t tix = a.txn_index[r];
#pragma unroll
    for (int m = 0; m < 3; ++m)
    {
        if (!nk[m]) continue;
        const uint32_t w = m == AD_MAP_RANGE ? 2u : 1u;
        for (uint32_t h = sl; h < 4; h += G)
            hdr[4 * P + h] = h == 0 ? ((tix << 2) | m) : (int64_t)(h == 1 ? nk[m] : (h == 2 ? nt[m] : no[m]));
        const int64_t* sk;
        const uint32_t* si;
        const int32_t* so;
        if (a.reg)
        {
            const uint8_t* base = a.reg + a.t_reg[(uint64_t)m * a.n + r];
            sk = reinterpret_cast<const int64_t*>(base);
            si = reinterpret_cast<const uint32_t*>(base + 8ull * nk[m]);
            so = reinterpret_cast<const int32_t*>(base + 8ull * nk[m] + 4ull * nt[m]);
        }
        else
        {
            sk = a.keys[m] + k0[m];
            si = a.txns[m] + t0[m];
            so = a.k2t[m] + o0[m];
        }
        if (m == AD_MAP_RANGE)
            for (uint32_t i = sl; i < 2 * nk[m]; i += G)
            {
                const int64_t rid = sk[i >> 1];
                okeys[KW + i] = (i & 1) ? a.rt_end[rid] : a.rt_start[rid];
            }
        else
            for (uint32_t i = sl; i < nk[m]; i += G) okeys[KW + i] = sk[i];
        if (a.rank_ids)
            for (uint32_t i = sl; i < nt[m]; i += G) oids32[ID + i] = si[i];
        else
            for (uint32_t i = sl; i < nt[m]; i += G)
            {
                const uint32_t d = si[i];
                int64_t* o = oids + 3 * (ID + i);
                o[0] = (int64_t)a.dict_msb[d];
                o[1] = (int64_t)a.dict_lsb[d];
                o[2] = (int64_t)a.dict_node[d];
            }
        for (uint32_t i = sl; i < no[m]; i += G) ok2t[KO + i] = so[i];
        P += 1;
        KW += w * nk[m];
        ID += nt[m];
        KO += no[m];
    }
}

__global__ void k_export_bounds(ExportArgs a, const uint64_t* dest_first, uint32_t n_dest, uint64_t* counts)
{
    const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
    if (d > n_dest) return;
    const PartBase b = part_base(a, dest_first[d]);
    counts[4 * d + 0] = b.P;
    counts[4 * d + 1] = b.KW;
    counts[4 * d + 2] = b.ID;
    counts[4 * d + 3] = b.KO;
}

// This rank's row of the exchange table (accord_deps.h, ad_exchange_plan): per destination the units of
// each array (differences of the cumulative bounds k_export_bounds wrote), then the row header.
__global__ void k_x_row(const uint64_t* counts, uint32_t n_dest, XRowHdr h, uint64_t* row)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < 4 * n_dest) row[i] = counts[i + 4] - counts[i];
    else if (i < 4 * n_dest + XROW_HDR) row[i] = h.w[i - 4 * n_dest];
}

// ---------------------------------------------------------------------------------------
// merge (K3)
// ---------------------------------------------------------------------------------------
__global__ void k_merge_part_sizes(MergeArgs a)
{
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= a.n_parts) return;
    const int64_t* h = a.hdr + 4 * p;
    const int m = (int)(h[0] & 3);
    a.psz[0 * a.n_parts + p] = (uint32_t)(h[1] * (m == AD_MAP_RANGE ? 2 : 1));
    a.psz[1 * a.n_parts + p] = (uint32_t)h[2];
    a.psz[2 * a.n_parts + p] = (uint32_t)h[3];
}

__global__ void k_merge_slots(MergeArgs a)
{
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= a.n_parts) return;
    uint32_t s = 0;
    while (s + 1 < a.n_src && a.src_first[s + 1] <= p) ++s;
    const int64_t h0 = a.hdr[4 * p];
    const int m = (int)(h0 & 3);
    const int64_t t = h0 >> 2;
    if (m > 2 || t < (int64_t)a.txn_base || t >= (int64_t)(a.txn_base + a.n_owned) || a.hdr[4 * p + 1] <= 0)
    {
        atomicOr(a.error, 1u);
        return;
    }
    // a source exports its parts by ascending (request, map): one part per group and source
    // exactly when each part's (request, map) is above its predecessor's in the same source
    if (p > a.src_first[s])
    {
        const int64_t hp = a.hdr[4 * (p - 1)];
        if (((hp >> 2) << 2 | (hp & 3)) >= ((t << 2) | m)) atomicOr(a.error, 2u);
    }
    const uint64_t g = (uint64_t)m * a.n_owned + (uint64_t)(t - (int64_t)a.txn_base);
    a.slot[g * a.n_src + s] = (int32_t)p;
}

// The parts of group g in source order, staged in wave-private LDS so that lanes in divergent
// code can read any part's bounds (no cross-lane shuffles from inactive lanes).
struct PartInfo {
    uint64_t ibase, kbase, obase;     // offsets of the part's ids / key words / k2t in the receive buffers
    uint32_t ni, kw, no, nk;          // sizes: ids, key words, k2t ints, keys
    uint32_t p;                       // part index
};

__device__ __forceinline__ PartInfo load_part_info(const MergeArgs& a, uint64_t p)
{
    const uint64_t P1 = a.n_parts + 1;
    PartInfo pi;
    pi.kbase = a.poff[0 * P1 + p];
    pi.kw = (uint32_t)(a.poff[0 * P1 + p + 1] - pi.kbase);
    pi.ibase = a.poff[1 * P1 + p];
    pi.ni = (uint32_t)(a.poff[1 * P1 + p + 1] - pi.ibase);
    pi.obase = a.poff[2 * P1 + p];
    pi.no = (uint32_t)(a.poff[2 * P1 + p + 1] - pi.obase);
    pi.nk = (uint32_t)a.hdr[4 * p + 1];
    pi.p = (uint32_t)p;
    return pi;
}

__device__ __forceinline__ uint32_t stage_parts(const MergeArgs& a, uint64_t g, PartInfo* info)
{
    const uint32_t l = lane_id();
    const int32_t v = l < a.n_src ? a.slot[g * a.n_src + l] : -1;
    const uint64_t live = ballot(v >= 0);
    const uint32_t np = __popcll(live);
    if (v >= 0) info[mbcnt(live)] = load_part_info(a, (uint64_t)v);
    wave_lds_sync();
    return np;
}

// keys of consecutive parts must ascend (disjoint, ordered slices)
__device__ __forceinline__ bool keys_ordered(int m, int64_t prev_s, int64_t prev_e, int64_t first_s, int64_t first_e)
{
    if (m == AD_MAP_RANGE) return prev_s < first_s || (prev_s == first_s && prev_e < first_e);
    return prev_s < first_s;
}

// pass 1: dup flags with exclusive per-part dup prefix; sizes of the merged group
__global__ void __launch_bounds__(64 * XWAVES) k_merge_count(MergeArgs a)
{
    __shared__ PartInfo s_info[XWAVES][64];
    PartInfo* info = s_info[threadIdx.x >> 6];
    const uint64_t n_groups = 3 * a.n_owned;
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t n_waves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    const uint32_t l = lane_id();
    for (uint64_t g = wave; g < n_groups; g += n_waves)
    {
        const int m = (int)(g / a.n_owned);
        const int w = m == AD_MAP_RANGE ? 2 : 1;
        wave_lds_sync();
        const uint32_t np = stage_parts(a, g, info);
        uint64_t kw = 0, ids = 0, k2t = 0, dups = 0;
        if (l == 0)
            for (uint32_t j = 1; j < np; ++j)
            {
                const PartInfo& pp = info[j - 1];
                const PartInfo& pj = info[j];
                const int64_t ls = a.keys[pp.kbase + pp.kw - w], le = w == 2 ? a.keys[pp.kbase + pp.kw - 1] : 0;
                const int64_t fs = a.keys[pj.kbase], fe = w == 2 ? a.keys[pj.kbase + 1] : 0;
                if (!keys_ordered(m, ls, le, fs, fe)) atomicOr(a.error, 4u);
            }
        for (uint32_t j = 0; j < np; ++j)
        {
            const PartInfo pj = info[j];
            uint32_t run = 0;
            for (uint32_t e0 = 0; e0 < pj.ni; e0 += 64)
            {
                const uint32_t e = e0 + l;
                bool dup = false;
                if (e < pj.ni && j > 0)
                {
                    const Tid3 x = load_tid(a.ids, pj.ibase + e);
                    for (uint32_t q = 0; q < j && !dup; ++q)
                    {
                        const uint64_t qb = info[q].ibase;
                        const uint32_t qn = info[q].ni;
                        const uint32_t pos = lb_tid(a.ids, qb, qn, x);
                        dup = pos < qn && tid_cmp3(load_tid(a.ids, qb + pos), x) == 0;
                    }
                }
                const uint64_t bm = ballot(dup);
                if (e < pj.ni) a.dup[pj.ibase + e] = (run + mbcnt(bm)) | (dup ? DUP_BIT : 0u);
                run += __popcll(bm);
            }
            kw += pj.kw;
            ids += pj.ni;
            k2t += pj.no;
            dups += run;
        }
        if (l == 0)
        {
            a.gsz[0 * n_groups + g] = (uint32_t)kw;
            a.gsz[1 * n_groups + g] = (uint32_t)(ids - dups);
            a.gsz[2 * n_groups + g] = (uint32_t)k2t;
        }
    }
}

// u(x) for an id x of part j whose lower bound in its own part is pos_j
__device__ __forceinline__ uint32_t union_index(const MergeArgs& a, const PartInfo* info, uint32_t np, uint32_t j,
                                                uint32_t pos_j, const Tid3& x)
{
    uint32_t u = 0;
    for (uint32_t q = 0; q < np; ++q)
    {
        const uint64_t qb = info[q].ibase;
        const uint32_t qn = info[q].ni;
        const uint32_t lb = q == j ? pos_j : lb_tid(a.ids, qb, qn, x);
        uint32_t dp;
        if (lb < qn) dp = a.dup[qb + lb] & ~DUP_BIT;
        else
        {
            const uint32_t d = qn ? a.dup[qb + qn - 1] : 0u;
            dp = qn ? (d & ~DUP_BIT) + (d >> 31) : 0u;
        }
        u += lb - dp;
    }
    return u;
}

// pass 2: emit keys (concatenated), the sorted id union and the remapped keysToTxnIds
__global__ void __launch_bounds__(64 * XWAVES) k_merge_emit(MergeArgs a)
{
    __shared__ PartInfo s_info[XWAVES][64];
    PartInfo* info = s_info[threadIdx.x >> 6];
    const uint64_t n_groups = 3 * a.n_owned;
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t n_waves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    const uint32_t l = lane_id();
    const uint64_t G1 = n_groups + 1;
    for (uint64_t g = wave; g < n_groups; g += n_waves)
    {
        const int m = (int)(g / a.n_owned);
        const uint64_t r = g - (uint64_t)m * a.n_owned;
        const uint64_t mb = (uint64_t)m * a.n_owned;
        const int w = m == AD_MAP_RANGE ? 2 : 1;
        const uint64_t KW = a.goff[0 * G1 + g], ID = a.goff[1 * G1 + g], KO = a.goff[2 * G1 + g];
        if (l == 0)
        {
            const uint64_t O = (uint64_t)m * (a.n_owned + 1) + r;
            a.o_keys_off[O] = (KW - a.goff[0 * G1 + mb]) / w;
            a.o_txn_off[O] = ID - a.goff[1 * G1 + mb];
            a.o_k2t_off[O] = KO - a.goff[2 * G1 + mb];
            if (r + 1 == a.n_owned)
            {
                a.o_keys_off[O + 1] = (a.goff[0 * G1 + g + 1] - a.goff[0 * G1 + mb]) / w;
                a.o_txn_off[O + 1] = a.goff[1 * G1 + g + 1] - a.goff[1 * G1 + mb];
                a.o_k2t_off[O + 1] = a.goff[2 * G1 + g + 1] - a.goff[2 * G1 + mb];
            }
        }
        wave_lds_sync();
        const uint32_t np = stage_parts(a, g, info);
        if (np == 0) continue;
        uint64_t nkeys_total = 0;
        {
            uint64_t at = KW;
            for (uint32_t j = 0; j < np; ++j)
            {
                const PartInfo pj = info[j];
                for (uint32_t e = l; e < pj.kw; e += 64) a.o_keys[at + e] = a.keys[pj.kbase + e];
                at += pj.kw;
                nkeys_total += pj.nk;
            }
        }
        const uint64_t n_union = a.goff[1 * G1 + g + 1] - ID;
        uint64_t keys_before = 0, pairs_before = 0;
        for (uint32_t j = 0; j < np; ++j)
        {
            const PartInfo pj = info[j];
            for (uint32_t e = l; e < pj.ni; e += 64)
            {
                if (a.dup[pj.ibase + e] & DUP_BIT) continue;
                const Tid3 x = load_tid(a.ids, pj.ibase + e);
                const uint32_t u = union_index(a, info, np, j, e, x);
                if (u >= n_union) { atomicOr(a.error, 8u); continue; }     // ids of a part not sorted/unique
                int64_t* o = a.o_ids + 3 * (ID + u);
                o[0] = (int64_t)x.msb;
                o[1] = (int64_t)x.lsb;
                o[2] = (int64_t)x.node;
            }
            const uint32_t nk = pj.nk;
            const uint32_t pairs = pj.no - nk;
            for (uint32_t e = l; e < nk; e += 64)
                a.o_k2t[KO + keys_before + e] =
                    (int32_t)((uint64_t)a.k2t[pj.obase + e] - nk + nkeys_total + pairs_before);
            for (uint32_t v = l; v < pairs; v += 64)
            {
                const uint32_t idx = (uint32_t)a.k2t[pj.obase + nk + v];
                if (idx >= pj.ni) { atomicOr(a.error, 8u); continue; }
                const Tid3 x = load_tid(a.ids, pj.ibase + idx);
                a.o_k2t[KO + nkeys_total + pairs_before + v] = (int32_t)union_index(a, info, np, j, idx, x);
            }
            keys_before += nk;
            pairs_before += pairs;
        }
    }
}

// ---------------------------------------------------------------------------------------
// AD_IDS_RANK: parts carry uint32 ranks of one global dictionary (the dictionary every store's
// snapshot was built over, ad_set_global_dict), so the union of a group's id lists is integer work. Pass 1 (wave per group): the union index u of every received id -- the
// number of distinct ranks below it in the group -- and whether an earlier part already holds it
// (Timestamp.equals), plus per part the key words and pairs of the earlier parts of its group.
// Pass 2 (thread per part): keys concatenated in source order, union ids materialised from the
// global dictionary at u, keysToTxnIds remapped through u (RelationMultiMap.linearUnion restated,
// RelationMultiMap.java:561-816).
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t lb_u32(const uint32_t* v, uint64_t base, uint32_t n, uint32_t x)
{
    uint32_t lo = 0, hi = n;
    while (lo < hi)
    {
        const uint32_t mid = (lo + hi) >> 1;
        if (v[base + mid] < x) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

__global__ void __launch_bounds__(64 * XWAVES) k_merge_rank(MergeArgs a)
{
    __shared__ PartInfo s_info[XWAVES][64];
    __shared__ uint32_t s_ist[XWAVES][64];
    PartInfo* info = s_info[threadIdx.x >> 6];
    uint32_t* ist = s_ist[threadIdx.x >> 6];
    const uint64_t n_groups = 3 * a.n_owned;
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t n_waves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    const uint32_t l = lane_id();
    const uint32_t* ids = reinterpret_cast<const uint32_t*>(a.ids);
    // one owned request per iteration: the slots of its three maps in one load (3 * n_src <= 64),
    // so maps without parts cost nothing more
    const bool combined = 3 * a.n_src <= 64;
    for (uint64_t r = wave; r < a.n_owned; r += n_waves)
    {
      int32_t v = -1;
      if (combined && l < 3 * a.n_src)
      {
          const uint32_t ml = l / a.n_src, sl = l - ml * a.n_src;
          v = a.slot[((uint64_t)ml * a.n_owned + r) * a.n_src + sl];
      }
      const uint64_t live_all = ballot(v >= 0);
      for (int m = 0; m < 3; ++m)
      {
        const uint64_t g = (uint64_t)m * a.n_owned + r;
        const int w = m == AD_MAP_RANGE ? 2 : 1;
        wave_lds_sync();
        uint32_t np;
        if (combined)
        {
            const uint64_t mmask = ((1ull << a.n_src) - 1) << (m * a.n_src);
            const uint64_t live = live_all & mmask;
            np = __popcll(live);
            if (v >= 0 && ((mmask >> l) & 1)) info[__popcll(live & ((1ull << l) - 1))] = load_part_info(a, (uint64_t)v);
            wave_lds_sync();
        }
        else
            np = stage_parts(a, g, info);
        if (np == 0)
        {
            if (l == 0)
            {
                a.gsz[0 * n_groups + g] = 0;
                a.gsz[1 * n_groups + g] = 0;
                a.gsz[2 * n_groups + g] = 0;
            }
            continue;
        }
        // per part (lane j < np): sizes, exclusive prefixes, source-order key check
        const bool pl = l < np;
        const uint32_t ni_l = pl ? info[l].ni : 0u, kw_l = pl ? info[l].kw : 0u;
        const uint32_t pr_l = pl ? info[l].no - info[l].nk : 0u, no_l = pl ? info[l].no : 0u;
        const uint32_t ii = wave_incl_scan(ni_l), ki = wave_incl_scan(kw_l), pi = wave_incl_scan(pr_l);
        const uint32_t T = uniform(__shfl(ii, (int)np - 1, 64));
        const uint32_t KWt = uniform(__shfl(ki, (int)np - 1, 64));
        const uint32_t NOt = uniform(wave_sum(no_l));
        if (pl)
        {
            ist[l] = ii - ni_l;
            a.ppre[2 * (uint64_t)info[l].p] = ki - kw_l;
            a.ppre[2 * (uint64_t)info[l].p + 1] = pi - pr_l;
            if (l > 0)
            {
                const PartInfo& pp = info[l - 1];
                const PartInfo& pj = info[l];
                const int64_t ls = a.keys[pp.kbase + pp.kw - w], le = w == 2 ? a.keys[pp.kbase + pp.kw - 1] : 0;
                const int64_t fs = a.keys[pj.kbase], fe = w == 2 ? a.keys[pj.kbase + 1] : 0;
                if (!keys_ordered(m, ls, le, fs, fe)) atomicOr(a.error, 4u);
            }
        }
        wave_lds_sync();
        uint32_t n_dup = 0;
        if (T <= 64)
        {
            // one id per lane; u = number of distinct ranks below it, from a rank count over the
            // group (wave-uniform broadcasts) minus the duplicates below it
            const bool live = l < T;
            uint32_t j = 0;
            for (uint32_t q = 1; q < np; ++q)
                if (l >= ist[q]) j = q;
            const uint32_t idx = l - ist[j];
            const uint64_t at = info[j].ibase + idx;
            const uint32_t x = live ? ids[at] : 0xFFFFFFFFu;
            if (live && idx > 0 && ids[at - 1] >= x) atomicOr(a.error, 8u);        // part not sorted / unique
            if (live && x >= a.n_global) atomicOr(a.error, 16u);
            uint32_t lt = 0;
            bool dup = false;
            for (uint32_t s2 = 0; s2 < T; ++s2)
            {
                const uint32_t y = (uint32_t)__builtin_amdgcn_readlane((int)x, (int)s2);
                lt += y < x ? 1u : 0u;
                dup = dup || (y == x && s2 < l);
            }
            const uint64_t dm = ballot(live && dup);
            for (uint64_t b = dm; b; b &= b - 1)
            {
                const uint32_t s2 = (uint32_t)(__ffsll((unsigned long long)b) - 1);
                const uint32_t y = (uint32_t)__builtin_amdgcn_readlane((int)x, (int)s2);
                lt -= y < x ? 1u : 0u;
            }
            if (live) a.u[at] = lt | (dup ? DUP_BIT : 0u);
            n_dup = __popcll(dm);
        }
        else
        {
            // large group: per part, dup flags against the earlier parts with an exclusive dup
            // prefix (binary searches), then u(x) = sum over parts q of lb_q(x) - dupsBefore_q(lb_q(x))
            for (uint32_t jj = 0; jj < np; ++jj)
            {
                const PartInfo pj = info[jj];
                uint32_t run = 0;
                for (uint32_t e0 = 0; e0 < pj.ni; e0 += 64)
                {
                    const uint32_t e = e0 + l;
                    bool dup = false;
                    if (e < pj.ni)
                    {
                        const uint32_t x = ids[pj.ibase + e];
                        if (e > 0 && ids[pj.ibase + e - 1] >= x) atomicOr(a.error, 8u);
                        if (x >= a.n_global) atomicOr(a.error, 16u);
                        for (uint32_t q = 0; q < jj && !dup; ++q)
                        {
                            const uint32_t pos = lb_u32(ids, info[q].ibase, info[q].ni, x);
                            dup = pos < info[q].ni && ids[info[q].ibase + pos] == x;
                        }
                    }
                    const uint64_t bm = ballot(dup);
                    if (e < pj.ni) a.dup[pj.ibase + e] = (run + mbcnt(bm)) | (dup ? DUP_BIT : 0u);
                    run += __popcll(bm);
                }
                n_dup += run;
            }
            __threadfence();
            for (uint32_t jj = 0; jj < np; ++jj)
            {
                const PartInfo pj = info[jj];
                for (uint32_t e = l; e < pj.ni; e += 64)
                {
                    const uint32_t x = ids[pj.ibase + e];
                    uint32_t u = 0;
                    for (uint32_t q = 0; q < np; ++q)
                    {
                        const uint64_t qb = info[q].ibase;
                        const uint32_t qn = info[q].ni;
                        const uint32_t lb = q == jj ? e : lb_u32(ids, qb, qn, x);
                        uint32_t dp;
                        if (lb < qn) dp = a.dup[qb + lb] & ~DUP_BIT;
                        else
                        {
                            const uint32_t d = qn ? a.dup[qb + qn - 1] : 0u;
                            dp = qn ? (d & ~DUP_BIT) + (d >> 31) : 0u;
                        }
                        u += lb - dp;
                    }
                    a.u[pj.ibase + e] = u | (a.dup[pj.ibase + e] & DUP_BIT);
                }
            }
        }
        if (l == 0)
        {
            a.gsz[0 * n_groups + g] = KWt;
            a.gsz[1 * n_groups + g] = T - n_dup;
            a.gsz[2 * n_groups + g] = NOt;
        }
      }
    }
}

// 8 lanes per part: its slice of the group's keys, union ids and keysToTxnIds
constexpr uint32_t EMIT_LANES = 8;

__global__ void k_merge_emit_rank(MergeArgs a)
{
    const uint64_t p = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / EMIT_LANES;
    const uint32_t j8 = threadIdx.x % EMIT_LANES;
    if (p >= a.n_parts) return;
    const uint64_t n_groups = 3 * a.n_owned, G1 = n_groups + 1, P1 = a.n_parts + 1;
    const int64_t h0 = a.hdr[4 * p];
    const int m = (int)(h0 & 3);
    const uint64_t g = (uint64_t)m * a.n_owned + (uint64_t)((h0 >> 2) - (int64_t)a.txn_base);
    const uint32_t w = m == AD_MAP_RANGE ? 2u : 1u;
    const uint32_t nk = (uint32_t)a.hdr[4 * p + 1], ni = (uint32_t)a.hdr[4 * p + 2], no = (uint32_t)a.hdr[4 * p + 3];
    const uint64_t kbase = a.poff[0 * P1 + p], ibase = a.poff[1 * P1 + p], obase = a.poff[2 * P1 + p];
    const uint64_t KW = a.goff[0 * G1 + g], ID = a.goff[1 * G1 + g], KO = a.goff[2 * G1 + g];
    const uint32_t nkeys_total = a.gsz[0 * n_groups + g] / w;
    const uint32_t kwb = a.ppre[2 * p], prb = a.ppre[2 * p + 1];
    for (uint32_t e = j8; e < nk * w; e += EMIT_LANES) a.o_keys[KW + kwb + e] = a.keys[kbase + e];
    const uint32_t* ids = reinterpret_cast<const uint32_t*>(a.ids);
    for (uint32_t e = j8; e < ni; e += EMIT_LANES)
    {
        const uint32_t uu = a.u[ibase + e];
        if (uu & DUP_BIT) continue;
        reinterpret_cast<uint32_t*>(a.o_ids)[ID + uu] = ids[ibase + e];     // the global rank
    }
    const uint32_t kb = kwb / w;
    for (uint32_t e = j8; e < nk; e += EMIT_LANES)
        a.o_k2t[KO + kb + e] = (int32_t)((uint64_t)a.k2t[obase + e] - nk + nkeys_total + prb);
    for (uint32_t v = j8; v < no - nk; v += EMIT_LANES)
    {
        const uint32_t idx = (uint32_t)a.k2t[obase + nk + v];
        if (idx >= ni)
        {
            atomicOr(a.error, 8u);
            continue;
        }
        a.o_k2t[KO + nkeys_total + prb + v] = (int32_t)(a.u[ibase + idx] & ~DUP_BIT);
    }
}

constexpr uint32_t SCAN_WAVES_RC = 4;      // waves of a k_rmerge_copy block

// exclusive scan over the RC_PARTS threads of a block; *total = the block's sum
__device__ __forceinline__ uint64_t block_excl_scan_rc(uint64_t v, uint64_t* wsum, uint64_t* total)
{
    uint64_t inc = v;
    const int l = lane_id();
#pragma unroll
    for (int d = 1; d < 64; d <<= 1)
    {
        const uint64_t tt = __shfl_up(inc, d, 64);
        if (l >= d) inc += tt;
    }
    const int w = threadIdx.x >> 6;
    if (l == 63) wsum[w] = inc;
    __syncthreads();
    uint64_t before = 0, all = 0;
    for (int k = 0; k < (int)SCAN_WAVES_RC; ++k)
    {
        const uint64_t x = wsum[k];
        if (k < w) before += x;
        all += x;
    }
    *total = all;
    __syncthreads();
    return inc - v + before;
}

// ---------------------------------------------------------------------------------------
// AD_IDS_RANK merge, G lanes per owned request (G = 8 for up to 8 sources, else 16; 64/G requests
// per wave). A request's parts are found through slot[r][s] (its first part in source s; a source
// sends a request's maps consecutively, ascending). Per map, the group's parts in source order are
// staged in the sub-group's LDS; a group of at most 4G ids is merged in LDS: an id is a duplicate
// when an earlier part holds it (binary search in the staged parts), and its union index is the
// number of first occurrences below it. Larger groups keep the per-part dup prefix in global
// memory and use the lower-bound formula of k_merge_rank. The size pass and the emit pass
// recompute the same staging, so nothing per id travels between them except the large groups'
// dup prefix. Offsets in the receive buffers are 32-bit (the host takes the per-group kernels
// beyond that).
// ---------------------------------------------------------------------------------------
constexpr uint32_t RM_WAVES = 4;                 // waves per block

struct RmPart {
    uint32_t kbase, ibase, obase;                // offsets in the receive buffers
    uint32_t kw, ni, no, nk;                     // key words, ids, k2t ints, keys
    uint32_t p;                                  // part index
};

template <uint32_t G>
struct RmLds {
    static constexpr uint32_t CAP = 4 * G;       // ids of a group merged in LDS
    RmPart info[G];
    uint32_t kst[G + 1], ist[G + 1], nst[G + 1], pst[G + 1];   // exclusive prefixes (+ total at np)
    uint32_t id[CAP];
    uint32_t u[CAP];                             // union index | DUP_BIT
    uint8_t pe[CAP];                             // part of each staged id
};

template <uint32_t G>
__device__ __forceinline__ uint64_t rm_ballot(bool p, uint32_t sub)
{
    if constexpr (G == 64) return ballot(p);
    else return (ballot(p) >> (sub * G)) & ((1ull << G) - 1);
}

__device__ __forceinline__ uint32_t rm_part_of(const uint32_t* st, uint32_t np, uint32_t e)
{
    uint32_t q = 0;
    for (uint32_t j = 1; j < np; ++j)
        if (st[j] <= e) q = j;
    return q;
}

// first i in [0, n) with !(v[i] < x), over LDS
__device__ __forceinline__ uint32_t rm_lb_lds(const uint32_t* v, uint32_t n, uint32_t x)
{
    uint32_t lo = 0, hi = n;
    while (lo < hi)
    {
        const uint32_t mid = (lo + hi) >> 1;
        if (v[mid] < x) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// The parts of owned request r held by source lane sl: a source's parts of one request are
// consecutive (k_rmerge_slots records the first), so the up to three records are loaded together
// (one round trip after the slot). rm_part_for then picks map m's (compile-time m: no scratch).
struct RmFound {
    uint4 A[3], B[3];
    bool ok[3];
    uint32_t p0;                                 // part index of A[0]
};

__device__ __forceinline__ void rm_find_parts(const MergeArgs& a, uint64_t r, uint32_t sl, RmFound& f)
{
#pragma unroll
    for (int k = 0; k < 3; ++k) f.ok[k] = false;
    if (sl >= a.n_src) return;
    const int32_t v = a.slot[r * a.n_src + sl];
    if (v == -1) return;
    const uint32_t p0 = (uint32_t)v & 0x3FFFFFFFu, cnt = ((uint32_t)v >> 30) + 1;
    const uint4* pi = reinterpret_cast<const uint4*>(a.pinfo);
#pragma unroll
    for (int k = 0; k < 3; ++k)
    {
        f.ok[k] = (uint32_t)k < cnt;
        f.A[k] = f.ok[k] ? pi[2 * ((uint64_t)p0 + k)] : make_uint4(0, 0, 0, 0);
        f.B[k] = f.ok[k] ? pi[2 * ((uint64_t)p0 + k) + 1] : make_uint4(0, 0, 0, 0xFFFFFFFFu);
    }
    f.p0 = p0;
}

__device__ __forceinline__ bool rm_part_for(const RmFound& f, int m, RmPart& q)
{
    bool has = false;
#pragma unroll
    for (int k = 0; k < 3; ++k)
        if (f.ok[k] && (int)(f.B[k].w & 3) == m)
        {
            q = RmPart{f.A[k].x, f.A[k].y, f.A[k].z, f.B[k].x, f.B[k].y, f.B[k].z, f.A[k].w, f.p0 + (uint32_t)k};
            has = true;
        }
    return has;
}

// Stage map m's parts of the request in source order; returns their number. Sets the prefix
// arrays (kst: key words, ist: ids, nst: keys, pst: pairs; entry np = totals).
template <uint32_t G>
__device__ __forceinline__ uint32_t rm_stage(const MergeArgs& a, RmLds<G>& L, const RmPart& mine, bool has, uint32_t sub,
                                             uint32_t sl, int m)
{
    const uint64_t live = rm_ballot<G>(has, sub);
    const uint32_t np = __popcll(live);
    if (np == 0) return 0;
    if (has) L.info[__popcll(live & ((1ull << sl) - 1))] = mine;
    wave_lds_sync();
    if (sl < np || sl == 0)
    {
        // lane sl: the prefix of part sl; lane 0 also the totals (entry np)
        const uint32_t upto = sl == 0 ? np : sl;
        uint32_t k = 0, i = 0, n = 0, pr = 0;
        for (uint32_t j = 0; j < upto; ++j)
        {
            k += L.info[j].kw;
            i += L.info[j].ni;
            n += L.info[j].nk;
            pr += L.info[j].no - L.info[j].nk;
        }
        L.kst[upto] = k;
        L.ist[upto] = i;
        L.nst[upto] = n;
        L.pst[upto] = pr;
        if (sl == 0) L.kst[0] = L.ist[0] = L.nst[0] = L.pst[0] = 0;
    }
    if (sl > 0 && sl < np)
    {
        // keys of consecutive parts ascend (disjoint slices in source order)
        const int w = m == AD_MAP_RANGE ? 2 : 1;
        const RmPart& pp = L.info[sl - 1];
        const RmPart& pj = L.info[sl];
        const int64_t ls = a.keys[pp.kbase + pp.kw - w], le = w == 2 ? a.keys[pp.kbase + pp.kw - 1] : 0;
        const int64_t fs = a.keys[pj.kbase], fe = w == 2 ? a.keys[pj.kbase + 1] : 0;
        if (!keys_ordered(m, ls, le, fs, fe)) atomicOr(a.error, 4u);
    }
    wave_lds_sync();
    return np;
}

// Ids of a group of T <= CAP into LDS, checked, with each id's dup bit (an earlier part holds it)
// in L.u. Returns the number of dups.
template <uint32_t G>
__device__ __forceinline__ uint32_t rm_stage_ids(const MergeArgs& a, RmLds<G>& L, uint32_t np, uint32_t T, uint32_t sub,
                                                 uint32_t sl)
{
    const uint32_t* ids = reinterpret_cast<const uint32_t*>(a.ids);
    for (uint32_t e = sl; e < T; e += G)
    {
        const uint32_t q = rm_part_of(L.ist, np, e);
        const uint32_t i = e - L.ist[q];
        const uint32_t x = ids[L.info[q].ibase + i];
        if (i > 0 && ids[L.info[q].ibase + i - 1] >= x) atomicOr(a.error, 8u);      // part not sorted / unique
        if (x >= a.n_global) atomicOr(a.error, 16u);
        L.id[e] = x;
    }
    wave_lds_sync();
    uint32_t dups = 0;
    for (uint32_t e0 = 0; e0 < T; e0 += G)
    {
        const uint32_t e = e0 + sl;
        bool dup = false;
        if (e < T)
        {
            const uint32_t q = rm_part_of(L.ist, np, e), x = L.id[e];
            for (uint32_t q2 = 0; q2 < q && !dup; ++q2)
            {
                const uint32_t* v = L.id + L.ist[q2];
                const uint32_t n = L.info[q2].ni;
                const uint32_t b = rm_lb_lds(v, n, x);
                dup = b < n && v[b] == x;
            }
            L.u[e] = dup ? DUP_BIT : 0u;
        }
        dups += __popcll(rm_ballot<G>(dup, sub));
    }
    wave_lds_sync();
    return dups;
}

// Large group: per part, dup flags against the earlier parts with the exclusive dup prefix of the
// part, in a.dup (global binary searches). Returns the number of dups.
template <uint32_t G>
__device__ __forceinline__ uint32_t rm_dups_global(const MergeArgs& a, RmLds<G>& L, uint32_t np, uint32_t sub, uint32_t sl)
{
    const uint32_t* ids = reinterpret_cast<const uint32_t*>(a.ids);
    uint32_t total = 0;
    for (uint32_t q = 0; q < np; ++q)
    {
        const RmPart pq = L.info[q];
        uint32_t run = 0;
        for (uint32_t e0 = 0; e0 < pq.ni; e0 += G)
        {
            const uint32_t e = e0 + sl;
            bool dup = false;
            if (e < pq.ni)
            {
                const uint32_t x = ids[pq.ibase + e];
                if (e > 0 && ids[pq.ibase + e - 1] >= x) atomicOr(a.error, 8u);
                if (x >= a.n_global) atomicOr(a.error, 16u);
                for (uint32_t q2 = 0; q2 < q && !dup; ++q2)
                {
                    const uint32_t pos = lb_u32(ids, L.info[q2].ibase, L.info[q2].ni, x);
                    dup = pos < L.info[q2].ni && ids[L.info[q2].ibase + pos] == x;
                }
            }
            const uint64_t bm = rm_ballot<G>(dup, sub);
            if (e < pq.ni) a.dup[pq.ibase + e] = (run + __popcll(bm & ((1ull << sl) - 1))) | (dup ? DUP_BIT : 0u);
            run += __popcll(bm);
        }
        total += run;
    }
    return total;
}

// union index of id x (position pos_j in its own part j) of a large group (after rm_dups_global)
template <uint32_t G>
__device__ __forceinline__ uint32_t rm_union_global(const MergeArgs& a, const RmLds<G>& L, uint32_t np, uint32_t j,
                                                    uint32_t pos_j, uint32_t x)
{
    const uint32_t* ids = reinterpret_cast<const uint32_t*>(a.ids);
    uint32_t u = 0;
    for (uint32_t q = 0; q < np; ++q)
    {
        const uint64_t qb = L.info[q].ibase;
        const uint32_t qn = L.info[q].ni;
        const uint32_t lb = q == j ? pos_j : lb_u32(ids, qb, qn, x);
        uint32_t dp;
        if (lb < qn) dp = a.dup[qb + lb] & ~DUP_BIT;
        else
        {
            const uint32_t d = qn ? a.dup[qb + qn - 1] : 0u;
            dp = qn ? (d & ~DUP_BIT) + (d >> 31) : 0u;
        }
        u += lb - dp;
    }
    return u;
}

__global__ void k_rmerge_slots(MergeArgs a)
{
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= a.n_parts) return;
    uint32_t s = 0;
    while (s + 1 < a.n_src && a.src_first[s + 1] <= p) ++s;
    const int64_t h0 = a.hdr[4 * p];
    const int m = (int)(h0 & 3);
    const int64_t t = h0 >> 2;
    if (m > 2 || t < (int64_t)a.txn_base || t >= (int64_t)(a.txn_base + a.n_owned) || a.hdr[4 * p + 1] <= 0)
    {
        atomicOr(a.error, 1u);
        reinterpret_cast<uint4*>(a.pinfo)[2 * p + 1] = make_uint4(0, 0, 0, 0xFFFFFFFFu);   // matches no request
        return;
    }
    bool first = p == a.src_first[s];
    if (!first)
    {
        const int64_t hp = a.hdr[4 * (p - 1)];
        if (((hp >> 2) << 2 | (hp & 3)) >= ((t << 2) | m)) atomicOr(a.error, 2u);
        first = (hp >> 2) != t;
    }
    const uint64_t rel = (uint64_t)(t - (int64_t)a.txn_base);
    if (first)
    {
        // the request's parts in this source (consecutive, at most one per map): p | (count - 1) << 30
        const uint64_t end = a.src_first[s + 1];
        uint32_t cnt = 1;
        if (p + 1 < end && (a.hdr[4 * (p + 1)] >> 2) == t)
        {
            cnt = 2;
            if (p + 2 < end && (a.hdr[4 * (p + 2)] >> 2) == t) cnt = 3;
        }
        a.slot[rel * a.n_src + s] = (int32_t)((uint32_t)p | ((cnt - 1) << 30));
    }
    // the part's record for the merge passes: offsets in the receive buffers, sizes, request and map
    const uint64_t P1 = a.n_parts + 1;
    const uint64_t k0 = a.poff[0 * P1 + p], i0 = a.poff[1 * P1 + p], o0 = a.poff[2 * P1 + p];
    uint4* pi = reinterpret_cast<uint4*>(a.pinfo);
    pi[2 * p] = make_uint4((uint32_t)k0, (uint32_t)i0, (uint32_t)o0, (uint32_t)a.hdr[4 * p + 1]);
    pi[2 * p + 1] = make_uint4((uint32_t)(a.poff[0 * P1 + p + 1] - k0), (uint32_t)(a.poff[1 * P1 + p + 1] - i0),
                               (uint32_t)(a.poff[2 * P1 + p + 1] - o0), (uint32_t)(rel << 2) | (uint32_t)m);
}

// Pass 1, G lanes per owned request: per map the merged sizes (keys, union ids, k2t) into
// gsz[k*3 + m][r], each part's place in its group (ppre[p] = {keys of the earlier parts, their
// pairs, the group's keys, parts}), and for groups of several parts every received id's union index
// (u[i] | DUP_BIT: an earlier part holds it).
template <uint32_t G>
__device__ __forceinline__ uint32_t sg_incl_scan(uint32_t v)
{
    const uint32_t sl = threadIdx.x % G;
#pragma unroll
    for (uint32_t d = 1; d < G; d <<= 1)
    {
        const uint32_t t = __shfl_up(v, d, G);
        if (sl >= d) v += t;
    }
    return v;
}

template <uint32_t G>
__device__ __forceinline__ uint32_t sg_sum(uint32_t v)
{
#pragma unroll
    for (uint32_t d = G / 2; d >= 1; d >>= 1) v += __shfl_xor(v, d, G);
    return v;
}

template <uint32_t G>
__global__ void __launch_bounds__(64 * RM_WAVES) k_rmerge_size(MergeArgs a)
{
    __shared__ RmLds<G> s_l[RM_WAVES * (64 / G)];
    const uint32_t sub = (threadIdx.x & 63) / G, sl = threadIdx.x % G;
    RmLds<G>& L = s_l[threadIdx.x / G];
    const uint64_t r = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / G;
    if (r >= a.n_owned || (*a.error & 3u)) return;     // malformed headers: nothing is read through them
    const uint64_t n = a.n_owned;
    const uint32_t* id = reinterpret_cast<const uint32_t*>(a.ids);
    RmFound f;
    rm_find_parts(a, r, sl, f);
    uint4* ppre = reinterpret_cast<uint4*>(a.ppre);
#pragma unroll 1
    for (int m = 0; m < 3; ++m)
    {
        // lane sl = source sl: the group's parts are the lanes holding one, in lane (= source) order
        RmPart q{};
        const bool h = rm_part_for(f, m, q);
        const uint32_t c_in = sg_incl_scan<G>(h ? 1u : 0u);
        const uint32_t np = __shfl(c_in, (int)(G - 1), G);
        uint32_t nk = 0, ids = 0, no = 0;
        bool heavy = false;
        if (np)
        {
            const uint32_t k_in = sg_incl_scan<G>(h ? q.nk : 0u), i_in = sg_incl_scan<G>(h ? q.ni : 0u);
            const uint32_t p_in = sg_incl_scan<G>(h ? q.no - q.nk : 0u);
            nk = __shfl(k_in, (int)(G - 1), G);
            const uint32_t T = __shfl(i_in, (int)(G - 1), G), PT = __shfl(p_in, (int)(G - 1), G);
            no = nk + PT;
            const uint32_t j = c_in - 1, i0 = i_in - (h ? q.ni : 0u);
            if (h) ppre[q.p] = make_uint4(k_in - q.nk, p_in - (q.no - q.nk), nk, np);
            uint32_t dups = 0;     // one part: its ids are the union (checked by the copy pass)
            heavy = np > 1 && T > RmLds<G>::CAP;
            if (np > 1 && T <= RmLds<G>::CAP)
            {
                // stage the group's ids, element-parallel: part j's at [ist[j], ist[j] + ni)
                wave_lds_sync();
                if (h)
                {
                    L.ist[j] = i0;
                    L.info[j].ni = q.ni;
                    L.info[j].ibase = q.ibase;
                }
                if (sl == 0) L.ist[np] = T;
                wave_lds_sync();
                for (uint32_t e = sl; e < T; e += G)
                {
                    const uint32_t qq = rm_part_of(L.ist, np, e);
                    const uint32_t x = id[L.info[qq].ibase + (e - L.ist[qq])];
                    if (x >= a.n_global) atomicOr(a.error, 16u);
                    L.id[e] = x;
                    L.pe[e] = (uint8_t)qq;
                }
                wave_lds_sync();
                // an id is a dup when an earlier part holds it (binary search in the staged parts)
                for (uint32_t e0 = 0; e0 < T; e0 += G)
                {
                    const uint32_t e = e0 + sl;
                    bool dup = false;
                    if (e < T)
                    {
                        const uint32_t qq = L.pe[e], x = L.id[e];
                        if (e > L.ist[qq] && L.id[e - 1] >= x) atomicOr(a.error, 8u);     // part not sorted / unique
                        for (uint32_t q2 = 0; q2 < qq && !dup; ++q2)
                        {
                            const uint32_t* v = L.id + L.ist[q2];
                            const uint32_t nn = L.info[q2].ni;
                            const uint32_t b = rm_lb_lds(v, nn, x);
                            dup = b < nn && v[b] == x;
                        }
                        L.u[e] = dup ? DUP_BIT : 0u;
                    }
                    dups += __popcll(rm_ballot<G>(dup, sub));
                }
                wave_lds_sync();
                // union index: first occurrences below the id
                for (uint32_t e = sl; e < T; e += G)
                {
                    const uint32_t x = L.id[e], qq = L.pe[e];
                    uint32_t u = 0;
                    for (uint32_t k = 0; k < T; ++k) u += (L.id[k] < x && !(L.u[k] & DUP_BIT)) ? 1u : 0u;
                    a.u[L.info[qq].ibase + (e - L.ist[qq])] = u | (L.u[e] & DUP_BIT);
                }
            }
            else if (np > 1 && sl == 0)
            {
                // more than CAP ids: k_rmerge_heavy sizes the union and places its ids
                const uint32_t at = atomicAdd(a.n_heavy, 1u);
                a.heavy[at] = (uint32_t)(r << 2) | (uint32_t)m;
            }
            if (np > 1)
            {
                // keys of consecutive parts ascend (disjoint slices in source order)
                const int w = m == AD_MAP_RANGE ? 2 : 1;
                const bool first = h && j == 0;
                // the previous part's last key, from the nearest lower lane holding a part
                const uint64_t holders = rm_ballot<G>(h, sub);
                const int64_t last_s = h ? a.keys[q.kbase + q.kw - w] : 0, last_e = (h && w == 2) ? a.keys[q.kbase + q.kw - 1] : 0;
                const uint64_t below = holders & ((1ull << sl) - 1);
                const int src = (h && !first && below) ? 63 - __clzll(below) : -1;
                const int64_t ps = __shfl(last_s, src < 0 ? (int)sl : src, G);
                const int64_t pe = __shfl(last_e, src < 0 ? (int)sl : src, G);
                if (h && !first)
                {
                    const int64_t fs = a.keys[q.kbase], fe = w == 2 ? a.keys[q.kbase + 1] : 0;
                    if (!keys_ordered(m, ps, pe, fs, fe)) atomicOr(a.error, 4u);
                }
            }
            ids = T - dups;
        }
        if (sl < 3 && !(sl == 1 && heavy))
        {
            const uint32_t v = sl == 0 ? nk : sl == 1 ? ids : no;
            a.gsz[(uint64_t)(sl * 3 + m) * n + r] = v;
        }
    }
}

// Groups of more than CAP ids (listed by k_rmerge_size): one wave per group, the sources in its
// lanes; dup prefix per part in global memory, union index of every id by lower bounds in the parts.
__global__ void __launch_bounds__(64 * RM_WAVES) k_rmerge_heavy(MergeArgs a)
{
    __shared__ RmLds<64> s_l[RM_WAVES];
    RmLds<64>& L = s_l[threadIdx.x >> 6];
    if (*a.error & 3u) return;
    const uint32_t sl = lane_id();
    const uint32_t nh = *a.n_heavy;
    const uint64_t n_waves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    const uint32_t* id = reinterpret_cast<const uint32_t*>(a.ids);
    for (uint64_t k = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; k < nh; k += n_waves)
    {
        const uint32_t e0 = a.heavy[k];
        const uint64_t r = e0 >> 2;
        const int m = (int)(e0 & 3);
        RmFound f;
        rm_find_parts(a, r, sl, f);
        RmPart q{};
        const bool h = rm_part_for(f, m, q);
        wave_lds_sync();
        const uint32_t np = rm_stage<64>(a, L, q, h, 0, sl, m);
        const uint32_t T = L.ist[np];
        const uint32_t dups = rm_dups_global<64>(a, L, np, 0, sl);
        __threadfence_block();
        for (uint32_t e = sl; e < T; e += 64)
        {
            const uint32_t qq = rm_part_of(L.ist, np, e), i = e - L.ist[qq];
            const uint64_t at = L.info[qq].ibase + i;
            a.u[at] = rm_union_global<64>(a, L, np, qq, i, id[at]) | (a.dup[at] & DUP_BIT);
        }
        if (sl == 0) a.gsz[(uint64_t)(1 * 3 + m) * a.n_owned + r] = T - dups;
    }
}

// bases[3*m + k]: offset of map m's first element in output array k (keys in words), m = 3: totals
__global__ void k_rmerge_bases(MergeArgs a, uint64_t* out)
{
    if (threadIdx.x != 0) return;
    const uint64_t n1 = a.n_owned + 1;
    uint64_t acc[3] = {0, 0, 0};
    for (int m = 0; m < 4; ++m)
    {
        for (int k = 0; k < 3; ++k) out[3 * m + k] = acc[k];
        if (m == 3) break;
        const uint64_t w = m == AD_MAP_RANGE ? 2 : 1;
        acc[0] += w * a.goff[(uint64_t)(0 * 3 + m) * n1 + a.n_owned];
        acc[1] += a.goff[(uint64_t)(1 * 3 + m) * n1 + a.n_owned];
        acc[2] += a.goff[(uint64_t)(2 * 3 + m) * n1 + a.n_owned];
    }
}

// Pass 2, load balanced over the receive buffers: a block takes 256 consecutive parts, places each
// (its group's offsets + its place in the group), then streams their keys, ids and keysToTxnIds to
// the merged arrays, thread per element (binary search of the owning part in LDS).
constexpr uint32_t RC_PARTS = 256;

struct RcLds {
    uint32_t kbase[RC_PARTS], ibase[RC_PARTS], obase[RC_PARTS];
    uint32_t ni[RC_PARTS], nk[RC_PARTS];
    uint32_t kdst[RC_PARTS], idst[RC_PARTS], hdst[RC_PARTS], pdst[RC_PARTS];
    int32_t add[RC_PARTS];                       // head adjustment: group keys + earlier pairs - own keys
    uint32_t flags[RC_PARTS];                    // bit 0: one-part group (ids copied), bit 1: range map (2 words)
    uint32_t kpre[RC_PARTS + 1], ipre[RC_PARTS + 1], opre[RC_PARTS + 1];
    uint64_t wsum[SCAN_WAVES_RC + 1];
};

__device__ __forceinline__ uint32_t rc_owner(const uint32_t* pre, uint32_t np, uint32_t e)
{
    // last j with pre[j] <= e
    uint32_t lo = 0, hi = np;
    while (hi - lo > 1)
    {
        const uint32_t mid = (lo + hi) >> 1;
        if (pre[mid] <= e) lo = mid;
        else hi = mid;
    }
    return lo;
}

__global__ void __launch_bounds__(RC_PARTS) k_rmerge_copy(MergeArgs a, const uint64_t* bases)
{
    __shared__ RcLds L;
    if (*a.error & 3u) return;
    const uint32_t t = threadIdx.x;
    const uint64_t p0 = (uint64_t)blockIdx.x * RC_PARTS;
    const uint32_t np = (uint32_t)min<uint64_t>(RC_PARTS, a.n_parts - p0);
    const uint64_t n1 = a.n_owned + 1;
    uint32_t kw = 0, ni = 0, no = 0;
    if (t < np)
    {
        const uint64_t p = p0 + t;
        const uint4* pi = reinterpret_cast<const uint4*>(a.pinfo);
        const uint4 A = pi[2 * p], B = pi[2 * p + 1];
        const uint4 pp = reinterpret_cast<const uint4*>(a.ppre)[p];
        const uint32_t m = B.w & 3, r = B.w >> 2;
        const uint32_t w = m == AD_MAP_RANGE ? 2u : 1u;
        const uint64_t K = a.goff[(uint64_t)(0 * 3 + m) * n1 + r], I = a.goff[(uint64_t)(1 * 3 + m) * n1 + r];
        const uint64_t O = a.goff[(uint64_t)(2 * 3 + m) * n1 + r];
        L.kbase[t] = A.x;
        L.ibase[t] = A.y;
        L.obase[t] = A.z;
        L.nk[t] = A.w;
        L.ni[t] = B.y;
        L.kdst[t] = (uint32_t)(bases[3 * m + 0] + w * (K + pp.x));
        L.idst[t] = (uint32_t)(bases[3 * m + 1] + I);
        L.hdst[t] = (uint32_t)(bases[3 * m + 2] + O + pp.x);
        L.pdst[t] = (uint32_t)(bases[3 * m + 2] + O + pp.z + pp.y);
        L.add[t] = (int32_t)(pp.z + pp.y) - (int32_t)A.w;
        L.flags[t] = (pp.w == 1 ? 1u : 0u) | (w == 2 ? 2u : 0u);
        kw = B.x;
        ni = B.y;
        no = B.z;
    }
    // exclusive prefixes of the parts' element counts (one block scan each)
    {
        uint64_t tot;
        uint64_t ex = block_excl_scan_rc(kw, L.wsum, &tot);
        L.kpre[t] = (uint32_t)ex;
        if (t == 0) L.kpre[RC_PARTS] = (uint32_t)tot;
        ex = block_excl_scan_rc(ni, L.wsum, &tot);
        L.ipre[t] = (uint32_t)ex;
        if (t == 0) L.ipre[RC_PARTS] = (uint32_t)tot;
        ex = block_excl_scan_rc(no, L.wsum, &tot);
        L.opre[t] = (uint32_t)ex;
        if (t == 0) L.opre[RC_PARTS] = (uint32_t)tot;
    }
    __syncthreads();
    const uint32_t KT = L.kpre[RC_PARTS], IT = L.ipre[RC_PARTS], OT = L.opre[RC_PARTS];
    const uint32_t* ids = reinterpret_cast<const uint32_t*>(a.ids);
    uint32_t* o_ids = reinterpret_cast<uint32_t*>(a.o_ids);
    for (uint32_t e = t; e < KT; e += RC_PARTS)
    {
        const uint32_t j = rc_owner(L.kpre, np, e), i = e - L.kpre[j];
        a.o_keys[L.kdst[j] + i] = a.keys[L.kbase[j] + i];
    }
    for (uint32_t e = t; e < IT; e += RC_PARTS)
    {
        const uint32_t j = rc_owner(L.ipre, np, e), i = e - L.ipre[j];
        const uint32_t at = L.ibase[j] + i, x = ids[at];
        if (L.flags[j] & 1u)
        {
            if (i > 0 && ids[at - 1] >= x) atomicOr(a.error, 8u);      // part not sorted / unique
            if (x >= a.n_global) atomicOr(a.error, 16u);
            o_ids[L.idst[j] + i] = x;
        }
        else
        {
            const uint32_t uu = a.u[at];
            if (!(uu & DUP_BIT)) o_ids[L.idst[j] + uu] = x;
        }
    }
    for (uint32_t e = t; e < OT; e += RC_PARTS)
    {
        const uint32_t j = rc_owner(L.opre, np, e), i = e - L.opre[j];
        const int32_t v = a.k2t[L.obase[j] + i];
        const uint32_t nk = L.nk[j];
        if (i < nk)
        {
            a.o_k2t[L.hdst[j] + i] = v + L.add[j];
            continue;
        }
        const uint32_t idx = (uint32_t)v;
        if (idx >= L.ni[j])
        {
            atomicOr(a.error, 8u);
            continue;
        }
        a.o_k2t[L.pdst[j] + (i - nk)] = (L.flags[j] & 1u) ? (int32_t)idx : (int32_t)(a.u[L.ibase[j] + idx] & ~DUP_BIT);
    }
}

// ---------------------------------------------------------------------------------------
// ad_parts_union: Deps.merge of replies whose key sets overlap (Deps.java:281-286 via
// PartialDeps.with / RelationMultiMap.linearUnion, RelationMultiMap.java:561-816). Every part
// holds three sorted, duplicate-free lists -- its keys, its ids, and its (key, id) pairs -- and
// the merged map is their union in each: an element's union index is
//     rank(x) = sum over parts q of ( lb_q(x) - dupsBefore_q(lb_q(x)) )
// (an element is a dup when an earlier part holds an equal one). Keys of range maps compare as
// (start, end) (Range.compare). Pass 1 (wave per group) ranks keys, then ids, then pairs (whose
// value is (key union index, id union index)), and sets each union key's head = union keys +
// distinct pairs with a smaller or equal key; pass 2 (8 lanes per part) writes them.
// ---------------------------------------------------------------------------------------
struct KeyV { int64_t a, b; };
__device__ __forceinline__ bool lt(const KeyV& x, const KeyV& y) { return x.a < y.a || (x.a == y.a && x.b < y.b); }
__device__ __forceinline__ bool eqv(const KeyV& x, const KeyV& y) { return x.a == y.a && x.b == y.b; }
__device__ __forceinline__ bool lt(uint64_t x, uint64_t y) { return x < y; }
__device__ __forceinline__ bool eqv(uint64_t x, uint64_t y) { return x == y; }

// the P lists of one group: val(q, i), len(q), and the scratch slot of element (q, i)
template <class V, class Val, class Len, class Slot>
struct UnionLists {
    uint32_t np; Val val; Len len; Slot slot;
    __device__ uint32_t lb(uint32_t q, const V& x) const
    {
        uint32_t lo = 0, hi = len(q);
        while (lo < hi)
        {
            const uint32_t mid = (lo + hi) >> 1;
            if (lt(val(q, mid), x)) lo = mid + 1;
            else hi = mid;
        }
        return lo;
    }
    // distinct elements of all lists below x (dp: per-list exclusive dup prefix | DUP_BIT)
    __device__ uint32_t rank_of(const V& x, const uint32_t* dp, uint32_t own_q = ~0u, uint32_t own_pos = 0) const
    {
        uint32_t r = 0;
        for (uint32_t q = 0; q < np; ++q)
        {
            const uint32_t n = len(q);
            const uint32_t b = q == own_q ? own_pos : lb(q, x);
            uint32_t before;
            if (b < n) before = dp[slot(q, b)] & ~DUP_BIT;
            else if (n == 0) before = 0;
            else
            {
                const uint32_t d = dp[slot(q, n - 1)];
                before = (d & ~DUP_BIT) + (d >> 31);
            }
            r += b - before;
        }
        return r;
    }
};

template <class V, class L>
__device__ uint32_t union_rank_all(const L& ls, uint32_t* dp, uint32_t* out, uint32_t* error)
{
    const uint32_t l = lane_id();
    uint32_t total = 0, dups = 0;
    for (uint32_t q = 0; q < ls.np; ++q)
    {
        const uint32_t n = ls.len(q);
        uint32_t run = 0;
        for (uint32_t e0 = 0; e0 < n; e0 += 64)
        {
            const uint32_t e = e0 + l;
            bool dup = false;
            if (e < n)
            {
                const V x = ls.val(q, e);
                if (e > 0 && !lt(ls.val(q, e - 1), x)) atomicOr(error, 8u);       // not sorted / unique
                for (uint32_t q2 = 0; q2 < q && !dup; ++q2)
                {
                    const uint32_t b = ls.lb(q2, x);
                    dup = b < ls.len(q2) && eqv(ls.val(q2, b), x);
                }
            }
            const uint64_t bm = ballot(dup);
            if (e < n) dp[ls.slot(q, e)] = (run + mbcnt(bm)) | (dup ? DUP_BIT : 0u);
            run += __popcll(bm);
        }
        total += n;
        dups += run;
    }
    __threadfence_block();      // written and read back by this wave only
    for (uint32_t q = 0; q < ls.np; ++q)
    {
        const uint32_t n = ls.len(q);
        for (uint32_t e = l; e < n; e += 64)
        {
            const V x = ls.val(q, e);
            const uint32_t s = ls.slot(q, e);
            out[s] = ls.rank_of(x, dp, q, e) | (dp[s] & DUP_BIT);
        }
    }
    __threadfence_block();      // written and read back by this wave only
    return total - dups;
}

template <class V, class Val, class Len, class Slot>
__device__ UnionLists<V, Val, Len, Slot> make_lists(uint32_t np, Val v, Len n, Slot s)
{
    return UnionLists<V, Val, Len, Slot>{np, v, n, s};
}

// wave-private staging of one group for the fast path (keys <= UN_KCAP, ids and pairs <= UN_ECAP)
constexpr uint32_t UN_KCAP = 64, UN_ECAP = 256;
struct UnionLds {
    uint32_t kst[64], ist[64], pst[64];          // per part: first key / id / pair of the group
    KeyV kv[UN_KCAP];
    uint32_t head[UN_KCAP], kdp[UN_KCAP], kuk[UN_KCAP];
    uint32_t iv[UN_ECAP], idp[UN_ECAP], iu[UN_ECAP];
    uint32_t pidx[UN_ECAP], pdp[UN_ECAP], ppos[UN_ECAP];
    uint64_t pv[UN_ECAP];
};

__global__ void __launch_bounds__(64 * XWAVES) k_union_rank(MergeArgs a)
{
    __shared__ UnionLds s_un[XWAVES];
    __shared__ PartInfo s_info[XWAVES][64];
    PartInfo* info = s_info[threadIdx.x >> 6];
    const uint64_t n_groups = 3 * a.n_owned;
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t n_waves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    const uint32_t l = lane_id();
    const uint32_t* ids = reinterpret_cast<const uint32_t*>(a.ids);
    for (uint64_t g = wave; g < n_groups; g += n_waves)
    {
        const int m = (int)(g / a.n_owned);
        const uint32_t w = m == AD_MAP_RANGE ? 2u : 1u;
        wave_lds_sync();
        const uint32_t np = stage_parts(a, g, info);
        if (np == 0)
        {
            if (l == 0)
            {
                a.gsz[0 * n_groups + g] = 0;
                a.gsz[1 * n_groups + g] = 0;
                a.gsz[2 * n_groups + g] = 0;
            }
            continue;
        }
        // per part: exclusive prefixes of its keys / ids / pairs over the group
        const bool pl = l < np;
        const uint32_t nk_l = pl ? info[l].nk : 0u, ni_l = pl ? info[l].ni : 0u;
        const uint32_t pr_l = pl ? info[l].no - info[l].nk : 0u;
        const uint32_t ki = wave_incl_scan(nk_l), ii = wave_incl_scan(ni_l), pi = wave_incl_scan(pr_l);
        const uint32_t KT = uniform(__shfl(ki, (int)np - 1, 64)), T = uniform(__shfl(ii, (int)np - 1, 64));
        const uint32_t PT = uniform(__shfl(pi, (int)np - 1, 64));
        if (KT <= UN_KCAP && T <= UN_ECAP && PT <= UN_ECAP)
        {
            // ---- fast path: the group's lists staged in wave-private LDS, ranked there
            UnionLds& L = s_un[threadIdx.x >> 6];
            if (pl)
            {
                L.kst[l] = ki - nk_l;
                L.ist[l] = ii - ni_l;
                L.pst[l] = pi - pr_l;
            }
            wave_lds_sync();
            auto part_of = [&](const uint32_t* st, uint32_t e) -> uint32_t {
                uint32_t q = 0;
                for (uint32_t r = 1; r < np; ++r)
                    if (st[r] <= e) q = r;
                return q;
            };
            for (uint32_t e = l; e < KT; e += 64)
            {
                const uint32_t q = part_of(L.kst, e), i = e - L.kst[q];
                const uint64_t o = info[q].kbase + (uint64_t)w * i;
                L.kv[e] = KeyV{a.keys[o], w == 2 ? a.keys[o + 1] : 0};
                L.head[e] = (uint32_t)a.k2t[info[q].obase + i];
            }
            for (uint32_t e = l; e < T; e += 64)
            {
                const uint32_t q = part_of(L.ist, e);
                L.iv[e] = ids[info[q].ibase + (e - L.ist[q])];
            }
            for (uint32_t e = l; e < PT; e += 64)
            {
                const uint32_t q = part_of(L.pst, e);
                L.pidx[e] = (uint32_t)a.k2t[info[q].obase + info[q].nk + (e - L.pst[q])];
            }
            wave_lds_sync();
            auto kval = [&](uint32_t q, uint32_t i) -> KeyV { return L.kv[L.kst[q] + i]; };
            auto klen = [&](uint32_t q) -> uint32_t { return info[q].nk; };
            auto kslot = [&](uint32_t q, uint32_t i) -> uint32_t { return L.kst[q] + i; };
            const uint32_t KU = union_rank_all<KeyV>(make_lists<KeyV>(np, kval, klen, kslot), L.kdp, L.kuk, a.error);
            auto ival = [&](uint32_t q, uint32_t i) -> uint64_t { return L.iv[L.ist[q] + i]; };
            auto ilen = [&](uint32_t q) -> uint32_t { return info[q].ni; };
            auto islot = [&](uint32_t q, uint32_t i) -> uint32_t { return L.ist[q] + i; };
            const uint32_t U = union_rank_all<uint64_t>(make_lists<uint64_t>(np, ival, ilen, islot), L.idp, L.iu, a.error);
            // pair values (key union index, id union index); the key is the first whose head is above nk + i
            for (uint32_t e = l; e < PT; e += 64)
            {
                const uint32_t q = part_of(L.pst, e), i = e - L.pst[q];
                const uint32_t nk = info[q].nk, k0 = L.kst[q];
                uint32_t key = 0;
                while (key + 1 < nk && L.head[k0 + key] <= nk + i) ++key;
                const uint32_t idx = L.pidx[e];
                if (idx >= info[q].ni) atomicOr(a.error, 8u);
                const uint32_t ui = idx < info[q].ni ? L.iu[L.ist[q] + idx] & ~DUP_BIT : 0xFFFFFFFFu;
                L.pv[e] = ((uint64_t)(L.kuk[k0 + key] & ~DUP_BIT) << 32) | ui;
            }
            wave_lds_sync();
            auto pval = [&](uint32_t q, uint32_t i) -> uint64_t { return L.pv[L.pst[q] + i]; };
            auto plen = [&](uint32_t q) -> uint32_t { return info[q].no - info[q].nk; };
            auto pslot = [&](uint32_t q, uint32_t i) -> uint32_t { return L.pst[q] + i; };
            const auto PL = make_lists<uint64_t>(np, pval, plen, pslot);
            const uint32_t PU = union_rank_all<uint64_t>(PL, L.pdp, L.ppos, a.error);
            // results to the per-element arrays of pass 2, heads of the distinct keys
            for (uint32_t e = l; e < KT; e += 64)
            {
                const uint32_t q = part_of(L.kst, e);
                const uint64_t s = info[q].kbase + (uint64_t)w * (e - L.kst[q]);
                const uint32_t r = L.kuk[e];
                a.kuk[s] = r;
                if (!(r & DUP_BIT)) a.khead[s] = KU + PL.rank_of((uint64_t)((r & ~DUP_BIT) + 1) << 32, L.pdp);
            }
            for (uint32_t e = l; e < T; e += 64)
            {
                const uint32_t q = part_of(L.ist, e);
                a.u[info[q].ibase + (e - L.ist[q])] = L.iu[e];
            }
            for (uint32_t e = l; e < PT; e += 64)
            {
                const uint32_t q = part_of(L.pst, e);
                a.ppos[info[q].obase + info[q].nk + (e - L.pst[q])] = L.ppos[e];
            }
            if (l == 0)
            {
                a.gsz[0 * n_groups + g] = KU * w;
                a.gsz[1 * n_groups + g] = U;
                a.gsz[2 * n_groups + g] = KU + PU;
            }
            continue;
        }
        // ---- general path: the same ranks over the receive buffers
        // keys
        auto kval = [&](uint32_t q, uint32_t i) -> KeyV {
            const uint64_t o = info[q].kbase + (uint64_t)w * i;
            return KeyV{a.keys[o], w == 2 ? a.keys[o + 1] : 0};
        };
        auto klen = [&](uint32_t q) -> uint32_t { return info[q].nk; };
        auto kslot = [&](uint32_t q, uint32_t i) -> uint32_t { return (uint32_t)(info[q].kbase + (uint64_t)w * i); };
        const auto KL = make_lists<KeyV>(np, kval, klen, kslot);
        const uint32_t KU = union_rank_all<KeyV>(KL, a.kdp, a.kuk, a.error);
        // ids
        auto ival = [&](uint32_t q, uint32_t i) -> uint64_t { return ids[info[q].ibase + i]; };
        auto ilen = [&](uint32_t q) -> uint32_t { return info[q].ni; };
        auto islot = [&](uint32_t q, uint32_t i) -> uint32_t { return (uint32_t)(info[q].ibase + i); };
        const auto IL = make_lists<uint64_t>(np, ival, ilen, islot);
        const uint32_t U = union_rank_all<uint64_t>(IL, a.dup, a.u, a.error);
        // pairs: body entry i of part q belongs to the key whose head (absolute end offset) is the
        // first above nk + i; value = (key union index, id union index)
        auto pval = [&](uint32_t q, uint32_t i) -> uint64_t {
            const PartInfo& pi = info[q];
            uint32_t lo = 0, hi = pi.nk;
            while (lo < hi)
            {
                const uint32_t mid = (lo + hi) >> 1;
                if ((uint32_t)a.k2t[pi.obase + mid] <= pi.nk + i) lo = mid + 1;
                else hi = mid;
            }
            const uint32_t key = lo < pi.nk ? lo : pi.nk - 1;
            const uint32_t idx = (uint32_t)a.k2t[pi.obase + pi.nk + i];
            const uint32_t uk = a.kuk[pi.kbase + (uint64_t)w * key] & ~DUP_BIT;
            const uint32_t ui = idx < pi.ni ? a.u[pi.ibase + idx] & ~DUP_BIT : 0xFFFFFFFFu;
            return ((uint64_t)uk << 32) | ui;
        };
        auto plen = [&](uint32_t q) -> uint32_t { return info[q].no - info[q].nk; };
        auto pslot = [&](uint32_t q, uint32_t i) -> uint32_t { return (uint32_t)(info[q].obase + info[q].nk + i); };
        const auto PL = make_lists<uint64_t>(np, pval, plen, pslot);
        const uint32_t PU = union_rank_all<uint64_t>(PL, a.pdp, a.ppos, a.error);
        // heads: union keys + distinct pairs whose key index is <= the key's
        for (uint32_t q = 0; q < np; ++q)
            for (uint32_t i = l; i < info[q].nk; i += 64)
            {
                const uint32_t s = kslot(q, i);
                const uint32_t r = a.kuk[s];
                if (r & DUP_BIT) continue;
                a.khead[s] = KU + PL.rank_of((uint64_t)((r & ~DUP_BIT) + 1) << 32, a.pdp);
            }
        if (l == 0)
        {
            a.gsz[0 * n_groups + g] = KU * w;
            a.gsz[1 * n_groups + g] = U;
            a.gsz[2 * n_groups + g] = KU + PU;
        }
    }
}

__global__ void k_union_emit(MergeArgs a)
{
    const uint64_t p = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / EMIT_LANES;
    const uint32_t j8 = threadIdx.x % EMIT_LANES;
    if (p >= a.n_parts) return;
    const uint64_t n_groups = 3 * a.n_owned, G1 = n_groups + 1, P1 = a.n_parts + 1;
    const int64_t h0 = a.hdr[4 * p];
    const int m = (int)(h0 & 3);
    const uint64_t g = (uint64_t)m * a.n_owned + (uint64_t)((h0 >> 2) - (int64_t)a.txn_base);
    const uint32_t w = m == AD_MAP_RANGE ? 2u : 1u;
    const uint32_t nk = (uint32_t)a.hdr[4 * p + 1], ni = (uint32_t)a.hdr[4 * p + 2], no = (uint32_t)a.hdr[4 * p + 3];
    const uint64_t kbase = a.poff[0 * P1 + p], ibase = a.poff[1 * P1 + p], obase = a.poff[2 * P1 + p];
    const uint64_t KW = a.goff[0 * G1 + g], ID = a.goff[1 * G1 + g], KO = a.goff[2 * G1 + g];
    const uint32_t KU = a.gsz[0 * n_groups + g] / w;
    for (uint32_t i = j8; i < nk; i += EMIT_LANES)
    {
        const uint64_t s = kbase + (uint64_t)w * i;
        const uint32_t r = a.kuk[s];
        if (r & DUP_BIT) continue;
        a.o_keys[KW + (uint64_t)w * r] = a.keys[s];
        if (w == 2) a.o_keys[KW + 2 * (uint64_t)r + 1] = a.keys[s + 1];
        a.o_k2t[KO + r] = (int32_t)a.khead[s];
    }
    const uint32_t* ids = reinterpret_cast<const uint32_t*>(a.ids);
    for (uint32_t e = j8; e < ni; e += EMIT_LANES)
    {
        const uint32_t uu = a.u[ibase + e];
        if (uu & DUP_BIT) continue;
        reinterpret_cast<uint32_t*>(a.o_ids)[ID + uu] = ids[ibase + e];
    }
    for (uint32_t v = j8; v < no - nk; v += EMIT_LANES)
    {
        const uint32_t pp = a.ppos[obase + nk + v];
        if (pp & DUP_BIT) continue;
        const uint32_t idx = (uint32_t)a.k2t[obase + nk + v];
        if (idx >= ni)
        {
            atomicOr(a.error, 8u);
            continue;
        }
        a.o_k2t[KO + KU + pp] = (int32_t)(a.u[ibase + idx] & ~DUP_BIT);
    }
}

hipError_t launch_union_rank(const MergeArgs& a, unsigned blocks, hipStream_t st)
{
    k_union_rank<<<blocks, 64 * XWAVES, 0, st>>>(a);
    return hipGetLastError();
}

hipError_t launch_union_emit(const MergeArgs& a, hipStream_t st)
{
    const uint64_t threads = a.n_parts * EMIT_LANES;
    if (a.n_parts) k_union_emit<<<(unsigned)((threads + 255) / 256), 256, 0, st>>>(a);
    return hipGetLastError();
}

// per map and owned request: offsets of the merged CSR (relative to the map's first group)
__global__ void k_merge_out_offsets(MergeArgs a)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t N1 = a.n_owned + 1;
    if (i >= 3 * N1) return;
    const int m = (int)(i / N1);
    const uint64_t r = i - (uint64_t)m * N1;
    const uint64_t G1 = 3 * a.n_owned + 1, g = (uint64_t)m * a.n_owned + r, mb = (uint64_t)m * a.n_owned;
    const uint64_t w = m == AD_MAP_RANGE ? 2 : 1;
    a.o_keys_off[i] = (a.goff[0 * G1 + g] - a.goff[0 * G1 + mb]) / w;
    a.o_txn_off[i] = a.goff[1 * G1 + g] - a.goff[1 * G1 + mb];
    a.o_k2t_off[i] = a.goff[2 * G1 + g] - a.goff[2 * G1 + mb];
}

__global__ void k_merge_bases(MergeArgs a, uint64_t* out)
{
    // out[3*m + k] = goff[k][m * n_owned] for m = 0..3 (m = 3: totals)
    const int i = threadIdx.x;
    if (i >= 12) return;
    const int m = i / 3, k = i % 3;
    out[i] = a.goff[k * (3 * a.n_owned + 1) + (uint64_t)m * a.n_owned];
}

}  // namespace

hipError_t run_export_sizes(const ExportArgs& a, hipStream_t st)
{
    if (!a.n) return hipSuccess;
    k_export_sizes<<<(unsigned)((a.n + 255) / 256), 256, 0, st>>>(a);
    return hipGetLastError();
}

hipError_t run_export_emit(const ExportArgs& a, hipStream_t st)
{
    if (!a.n) return hipSuccess;
    // lanes per request by the batch's ids per request (a.ids_per_req: from the resolve's stats). Measured
    // (scripts/export_ab.sh, AD_EXPORT_TRACE): at 2 ids per request (config-3 W = 8 stores) 2 lanes take
    // 0.77 ms for the node's eight exports against 0.95 with 4, 1.42 with 8 and 1.11 for the block tiles;
    // at 9 (config-3 N = 1) 4 lanes take 0.245 ms against 0.355 with 2, 0.29 with 8 and 0.38 for tiles
    const int gsel = getenv("AD_EXPORT_G") ? atoi(getenv("AD_EXPORT_G")) : 0;
    const uint32_t G = (gsel == 2 || gsel == 4 || gsel == 8 || gsel == 16 || gsel == 32) ? (uint32_t)gsel : a.ids_per_req <= 4 ? 2u : a.ids_per_req <= 32 ? 4u : a.ids_per_req <= 128 ? 8u : (a.ids_per_req <= 512 ? 16u : 32u);
    const uint64_t blocks = (a.n * G + 255) / 256;
    if (getenv("AD_EXPORT_TRACE")) fprintf(stderr, "export: %llu requests, %llu ids per request, %u lanes each\n",
                                           (unsigned long long)a.n, (unsigned long long)a.ids_per_req, G);
    if (G == 2) k_export_groups<2><<<(unsigned)blocks, 256, 0, st>>>(a);
    else if (G == 4) k_export_groups<4><<<(unsigned)blocks, 256, 0, st>>>(a);
    else if (G == 8) k_export_groups<8><<<(unsigned)blocks, 256, 0, st>>>(a);
    else if (G == 16) k_export_groups<16><<<(unsigned)blocks, 256, 0, st>>>(a);
    else k_export_groups<32><<<(unsigned)blocks, 256, 0, st>>>(a);
    return hipGetLastError();
}

hipError_t run_export_bounds(const ExportArgs& a, const uint64_t* dest_first, uint32_t n_dest, uint64_t* counts,
                             hipStream_t st)
{
    k_export_bounds<<<(n_dest + 1 + 63) / 64, 64, 0, st>>>(a, dest_first, n_dest, counts);
    return hipGetLastError();
}

hipError_t run_x_row(const uint64_t* counts, uint32_t n_dest, const XRowHdr& h, uint64_t* row, hipStream_t st)
{
    const uint32_t n = 4 * n_dest + XROW_HDR;
    k_x_row<<<(n + 63) / 64, 64, 0, st>>>(counts, n_dest, h, row);
    return hipGetLastError();
}

hipError_t run_merge_prepare(const MergeArgs& a, hipStream_t st)
{
    if (!a.n_parts) return hipSuccess;
    const unsigned b = (unsigned)((a.n_parts + 255) / 256);
    k_merge_part_sizes<<<b, 256, 0, st>>>(a);
    return hipGetLastError();
}

hipError_t run_merge_slots(const MergeArgs& a, hipStream_t st)
{
    if (!a.n_parts) return hipSuccess;
    k_merge_slots<<<(unsigned)((a.n_parts + 255) / 256), 256, 0, st>>>(a);
    return hipGetLastError();
}

static unsigned merge_blocks(uint64_t n_groups)
{
    const uint64_t want = (n_groups + XWAVES - 1) / XWAVES;
    const uint64_t cap = (uint64_t)device_cu_count() * 32;
    return (unsigned)std::max<uint64_t>(1, std::min(want, cap));
}

hipError_t run_merge_count(const MergeArgs& a, hipStream_t st)
{
    if (!a.n_owned) return hipSuccess;
    k_merge_count<<<merge_blocks(3 * a.n_owned), 64 * XWAVES, 0, st>>>(a);
    return hipGetLastError();
}

hipError_t run_merge_emit(const MergeArgs& a, hipStream_t st)
{
    if (!a.n_owned) return hipSuccess;
    k_merge_emit<<<merge_blocks(3 * a.n_owned), 64 * XWAVES, 0, st>>>(a);
    return hipGetLastError();
}

hipError_t run_merge_rank(const MergeArgs& a, hipStream_t st)
{
    if (!a.n_owned) return hipSuccess;
    k_merge_rank<<<merge_blocks(a.n_owned), 64 * XWAVES, 0, st>>>(a);
    return hipGetLastError();
}

hipError_t run_merge_emit_rank(const MergeArgs& a, hipStream_t st)
{
    const uint64_t n_off = 3 * (a.n_owned + 1);
    k_merge_out_offsets<<<(unsigned)((n_off + 255) / 256), 256, 0, st>>>(a);
    const uint64_t threads = a.n_parts * EMIT_LANES;
    if (a.n_parts) k_merge_emit_rank<<<(unsigned)((threads + 255) / 256), 256, 0, st>>>(a);
    return hipGetLastError();
}

hipError_t run_rmerge_slots(const MergeArgs& a, hipStream_t st)
{
    if (!a.n_parts) return hipSuccess;
    k_rmerge_slots<<<(unsigned)((a.n_parts + 255) / 256), 256, 0, st>>>(a);
    return hipGetLastError();
}

template <template <uint32_t> class K>
static hipError_t rm_launch(const MergeArgs& a, hipStream_t st)
{
    if (a.n_src > RM_MAX_SRC) return hipErrorInvalidValue;
    if (!a.n_owned) return hipSuccess;
    const uint32_t G = a.n_src <= 8 ? 8u : 16u;
    const uint64_t threads = a.n_owned * G;
    const unsigned blocks = (unsigned)((threads + 64 * RM_WAVES - 1) / (64 * RM_WAVES));
    if (G == 8) K<8>::launch(blocks, a, st);
    else K<16>::launch(blocks, a, st);
    return hipGetLastError();
}

template <uint32_t G>
struct RmSize {
    static void launch(unsigned blocks, const MergeArgs& a, hipStream_t st) { k_rmerge_size<G><<<blocks, 64 * RM_WAVES, 0, st>>>(a); }
};

hipError_t run_rmerge_size(const MergeArgs& a, hipStream_t st)
{
    hipError_t e = hipMemsetAsync(a.n_heavy, 0, sizeof(uint32_t), st);
    if (e != hipSuccess) return e;
    if ((e = rm_launch<RmSize>(a, st)) != hipSuccess) return e;
    if (a.n_owned) k_rmerge_heavy<<<(unsigned)device_cu_count() * 2, 64 * RM_WAVES, 0, st>>>(a);
    return hipGetLastError();
}

hipError_t run_rmerge_copy(const MergeArgs& a, const uint64_t* bases, hipStream_t st)
{
    k_rmerge_bases<<<1, 64, 0, st>>>(a, const_cast<uint64_t*>(bases));
    if (!a.n_parts) return hipGetLastError();
    // load-balanced over blocks of 256 parts (G lanes per part instead -- a copy like the export's -- measured
    // slower: 0.155 against 0.123 ms per owner at W = 8, 0.23 against 0.206 ms at N = 1; deleted in round 6)
    k_rmerge_copy<<<(unsigned)((a.n_parts + RC_PARTS - 1) / RC_PARTS), RC_PARTS, 0, st>>>(a, bases);
    return hipGetLastError();
}

hipError_t run_union_rank(const MergeArgs& a, hipStream_t st)
{
    if (!a.n_owned) return hipSuccess;
    return launch_union_rank(a, merge_blocks(3 * a.n_owned), st);
}

hipError_t run_union_emit(const MergeArgs& a, hipStream_t st)
{
    const uint64_t n_off = 3 * (a.n_owned + 1);
    k_merge_out_offsets<<<(unsigned)((n_off + 255) / 256), 256, 0, st>>>(a);
    return launch_union_emit(a, st);
}

hipError_t run_merge_bases(const MergeArgs& a, uint64_t* out, hipStream_t st)
{
    k_merge_bases<<<1, 64, 0, st>>>(a, out);
    return hipGetLastError();
}

}  // namespace adx
