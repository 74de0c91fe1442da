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

// one 8-lane group per request, its three maps in turn
__global__ void __launch_bounds__(64 * XWAVES) k_export_emit(ExportArgs a)
{
    const uint32_t g8 = threadIdx.x & 7;
    const uint64_t r = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 3;
    if (r >= a.n) return;
    PartBase pb = part_base(a, r);
    for (int m = 0; m < 3; ++m)
    {
        const uint64_t k0 = a.keys_off[m][r], nk = a.keys_off[m][r + 1] - k0;
        if (nk == 0) continue;
        const uint64_t t0 = a.txn_off[m][r], nt = a.txn_off[m][r + 1] - t0;
        const uint64_t o0 = a.k2t_off[m][r], no = a.k2t_off[m][r + 1] - o0;
        const uint64_t P = pb.P, KW = pb.KW, ID = pb.ID, KO = pb.KO;
        // the request's map: packed arrays, or its region (keys, txnIds, keysToTxnIds back to back)
        const int64_t* ikeys;
        const uint32_t* itx;
        const int32_t* ik2t;
        if (a.reg)
        {
            ikeys = reinterpret_cast<const int64_t*>(a.reg + a.t_reg[(uint64_t)m * a.n + r]);
            itx = reinterpret_cast<const uint32_t*>(ikeys + nk);
            ik2t = reinterpret_cast<const int32_t*>(itx + nt);
        }
        else
        {
            ikeys = a.keys[m] + k0;
            itx = a.txns[m] + t0;
            ik2t = a.k2t[m] + o0;
        }
        if (g8 == 0)
        {
            int64_t* h = a.hdr + 4 * P;
            h[0] = (a.txn_index[r] << 2) | m;
            h[1] = (int64_t)nk;
            h[2] = (int64_t)nt;
            h[3] = (int64_t)no;
        }
        if (m == AD_MAP_RANGE)
        {
            for (uint64_t j = g8; j < nk; j += 8)
            {
                const int64_t rid = ikeys[j];
                a.okeys[KW + 2 * j] = a.rt_start[rid];
                a.okeys[KW + 2 * j + 1] = a.rt_end[rid];
            }
        }
        else
        {
            for (uint64_t j = g8; j < nk; j += 8) a.okeys[KW + j] = ikeys[j];
        }
        if (a.gmap)
        {
            uint32_t* o = reinterpret_cast<uint32_t*>(a.oids) + ID;
            for (uint64_t j = g8; j < nt; j += 8) o[j] = a.gmap[itx[j]];
        }
        else
            for (uint64_t j = g8; j < nt; j += 8)
            {
                const uint32_t d = itx[j];
                int64_t* o = a.oids + 3 * (ID + j);
                o[0] = (int64_t)a.dict_msb[d];
                o[1] = (int64_t)a.dict_lsb[d];
                o[2] = (int64_t)a.dict_node[d];
            }
        for (uint64_t j = g8; j < no; j += 8) a.ok2t[KO + j] = ik2t[j];
        pb.P += 1;
        pb.KW += (m == AD_MAP_RANGE ? 2 : 1) * nk;
        pb.ID += nt;
        pb.KO += no;
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
// AD_IDS_RANK: parts carry uint32 ranks of one global dictionary, so the union of a group's id
// lists is integer work. Pass 1 (wave per group): the union index u of every received id -- the
// number of distinct ranks below it in the group -- and whether an earlier part already holds it
// (Timestamp.equals), plus per part the key words and pairs of the earlier parts of its group.
// Pass 2 (thread per part): keys concatenated in source order, union ids materialised from the
// global dictionary at u, keysToTxnIds remapped through u (RelationMultiMap.linearUnion restated,
// RelationMultiMap.java:561-816).
// ---------------------------------------------------------------------------------------
__global__ void k_global_map(const uint64_t* l_msb, const uint64_t* l_lo, const int32_t* l_node, uint64_t n_local,
                             const uint64_t* g_msb, const uint64_t* g_lsb, const int32_t* g_node, uint64_t n_global,
                             uint32_t* map, uint32_t* err)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_local) return;
    const NormTid x{l_msb[i], l_lo[i], l_node[i]};
    uint64_t lo = 0, hi = n_global;
    while (lo < hi)
    {
        const uint64_t mid = (lo + hi) >> 1;
        if (norm_cmp(norm_tid(g_msb[mid], g_lsb[mid], g_node[mid]), x) < 0) lo = mid + 1;
        else hi = mid;
    }
    const bool found = lo < n_global && norm_cmp(norm_tid(g_msb[lo], g_lsb[lo], g_node[lo]), x) == 0;
    if (!found) atomicOr(err, 1u);
    map[i] = found ? (uint32_t)lo : 0u;
}

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
    const uint64_t threads = a.n * 8;
    k_export_emit<<<(unsigned)((threads + 64 * XWAVES - 1) / (64 * XWAVES)), 64 * XWAVES, 0, st>>>(a);
    return hipGetLastError();
}

hipError_t run_export_bounds(const ExportArgs& a, const uint64_t* dest_first, uint32_t n_dest, uint64_t* counts,
                             hipStream_t st)
{
    k_export_bounds<<<(n_dest + 1 + 63) / 64, 64, 0, st>>>(a, dest_first, n_dest, counts);
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

hipError_t run_global_map(const uint64_t* l_msb, const uint64_t* l_lo_norm, const int32_t* l_node, uint64_t n_local,
                          const uint64_t* g_msb, const uint64_t* g_lsb, const int32_t* g_node, uint64_t n_global,
                          uint32_t* map, uint32_t* err, hipStream_t st)
{
    if (!n_local) return hipSuccess;
    k_global_map<<<(unsigned)((n_local + 255) / 256), 256, 0, st>>>(l_msb, l_lo_norm, l_node, n_local, g_msb, g_lsb,
                                                                   g_node, n_global, map, err);
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
