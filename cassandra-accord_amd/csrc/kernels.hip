// kernels.hip — hand-written gfx950 (CDNA4, wave64) kernels of the dependency-resolution path.
//
//   K0  k_encode_txn / k_probe_keys   request -> ranks; (request, key) -> CommandsForKey index
//   K1  k_scan                         CommandsForKey.mapReduceActive (CommandsForKey.java:910-968)
//   K4  k_range                        InMemoryCommandStore.mapReduceRangesInternal (:884-1017)
//                                      + RedundantBefore.collectDeps (RedundantBefore.java:183-192)
//   K2  k_build<EMIT>                  Deps.AbstractBuilder.add + RelationMultiMap.AbstractBuilder.build
//                                      (Deps.java:80-106, RelationMultiMap.java:147-260) and
//                                      PartialDeps.with (PartialDeps.java:73-81, linearUnion
//                                      RelationMultiMap.java:561-816) as a multi-list union
//   trees / scans                      index build and exclusive scans
//
// All integer work; no MFMA. Memory-/latency-bound: coalesced 64-lane loads, ballot/mbcnt
// compaction, LDS staging, wave-uniform control.
#include <hip/hip_runtime.h>

#include "common.hpp"
#include "kernels.hpp"
#include "wave.hpp"

namespace adx {


__device__ __forceinline__ void set_error(BatchCtl* ctl, unsigned code) { atomicCAS(&ctl->error, 0u, code); }

// ---------------------------------------------------------------------------------------
// Index build: per witness class, 64-ary max trees over tau (CFK) and over range ends.
// ---------------------------------------------------------------------------------------
__global__ void k_tree_leaf_cfk(const uint2* __restrict__ ent, uint64_t n, uint32_t* __restrict__ out0,
                                uint32_t* __restrict__ out1, uint32_t* __restrict__ out2, uint64_t n_out)
{
    // one wave per level-1 node: 64 coalesced leaves, wave max per class
    const uint64_t node = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (node >= n_out) return;
    const uint64_t i = node * 64 + lane_id();
    uint32_t v[NCLASS] = {0, 0, 0};
    if (i < n)
    {
        const uint2 e = ent[i];
        const uint32_t kd = e.y >> RANK_BITS;
#pragma unroll
        for (int c = 0; c < NCLASS; ++c) v[c] = ((CLASS_KINDS[c] >> kd) & 1) ? e.x : 0u;
    }
#pragma unroll
    for (int c = 0; c < NCLASS; ++c)
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) v[c] = max(v[c], (uint32_t)__shfl_xor(v[c], d, 64));
    if (lane_id() == 0) { out0[node] = v[0]; out1[node] = v[1]; out2[node] = v[2]; }
}

template <class T>
__global__ void k_tree_up(const T* __restrict__ in, uint64_t n, T* __restrict__ out, uint64_t n_out, T neutral)
{
    const uint64_t node = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (node >= n_out) return;
    const uint64_t i = node * 64 + lane_id();
    T v = i < n ? in[i] : neutral;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1)
    {
        T o = __shfl_xor(v, d, 64);
        v = o > v ? o : v;
    }
    if (lane_id() == 0) out[node] = v;
}

__global__ void k_tree_leaf_range(const int64_t* __restrict__ r_end, const uint32_t* __restrict__ r_txw, uint64_t n,
                                  int64_t* __restrict__ out0, int64_t* __restrict__ out1, int64_t* __restrict__ out2,
                                  uint64_t n_out)
{
    const uint64_t node = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (node >= n_out) return;
    const uint64_t i = node * 64 + lane_id();
    int64_t v[NCLASS] = {INT64_MIN, INT64_MIN, INT64_MIN};
    if (i < n)
    {
        const int64_t e = r_end[i];
        const uint32_t kd = r_txw[i] >> RANK_BITS;
#pragma unroll
        for (int c = 0; c < NCLASS; ++c) v[c] = ((CLASS_KINDS[c] >> kd) & 1) ? e : INT64_MIN;
    }
#pragma unroll
    for (int c = 0; c < NCLASS; ++c)
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1)
        {
            int64_t o = __shfl_xor(v[c], d, 64);
            v[c] = o > v[c] ? o : v[c];
        }
    if (lane_id() == 0) { out0[node] = v[0]; out1[node] = v[1]; out2[node] = v[2]; }
}

static inline unsigned grid_for_waves(uint64_t waves, unsigned waves_per_block)
{
    uint64_t g = (waves + waves_per_block - 1) / waves_per_block;
    return (unsigned)(g ? g : 1);
}

hipError_t build_cfk_trees(const DevSnapshot& s, hipStream_t st)
{
    if (s.n_levels <= 1) return hipSuccess;
    k_tree_leaf_cfk<<<grid_for_waves(s.lvl_n[1], 4), 256, 0, st>>>(
        s.ent, s.n_ent, const_cast<uint32_t*>(s.lvl[0][1]), const_cast<uint32_t*>(s.lvl[1][1]),
        const_cast<uint32_t*>(s.lvl[2][1]), s.lvl_n[1]);
    for (int l = 2; l < s.n_levels; ++l)
        for (int c = 0; c < NCLASS; ++c)
            k_tree_up<uint32_t><<<grid_for_waves(s.lvl_n[l], 4), 256, 0, st>>>(
                s.lvl[c][l - 1], s.lvl_n[l - 1], const_cast<uint32_t*>(s.lvl[c][l]), s.lvl_n[l], 0u);
    return hipGetLastError();
}

hipError_t build_range_trees(const DevSnapshot& s, hipStream_t st)
{
    if (s.n_rlevels <= 1) return hipSuccess;
    k_tree_leaf_range<<<grid_for_waves(s.rlvl_n[1], 4), 256, 0, st>>>(
        s.r_end, s.r_txw, s.n_rent, const_cast<int64_t*>(s.rlvl[0][1]), const_cast<int64_t*>(s.rlvl[1][1]),
        const_cast<int64_t*>(s.rlvl[2][1]), s.rlvl_n[1]);
    for (int l = 2; l < s.n_rlevels; ++l)
        for (int c = 0; c < NCLASS; ++c)
            k_tree_up<int64_t><<<grid_for_waves(s.rlvl_n[l], 4), 256, 0, st>>>(
                s.rlvl[c][l - 1], s.rlvl_n[l - 1], const_cast<int64_t*>(s.rlvl[c][l]), s.rlvl_n[l], INT64_MIN);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// K0: encode requests
// ---------------------------------------------------------------------------------------
// rank of an arbitrary id against the dictionary: member i -> 2i+1, else 2*lower_bound
// (the sampled search: the cache-resident sample, then one DICT_SAMP-id window of the dictionary)
__device__ __forceinline__ uint32_t encode_rank(const DevSnapshot& s, uint64_t msb, uint64_t lsb, int32_t node)
{
    if (!s.ds_hi || !s.n_samp)
    {
        const NormTid x = norm_tid(msb, lsb, node);
        uint64_t lo = 0, hi = s.n_dict;
        while (lo < hi)
        {
            const uint64_t mid = (lo + hi) >> 1;
            const NormTid m = {s.dict_hi[mid], s.dict_lo[mid], s.dict_node[mid]};
            if (norm_cmp(m, x) < 0) lo = mid + 1;
            else hi = mid;
        }
        if (lo < s.n_dict)
        {
            const NormTid m = {s.dict_hi[lo], s.dict_lo[lo], s.dict_node[lo]};
            if (norm_cmp(m, x) == 0) return (uint32_t)(2 * lo + 1);
        }
        return (uint32_t)(2 * lo);
    }
    return dict_rank_sampled(s, norm_tid(msb, lsb, node));
}

__global__ void k_encode_txn(DevSnapshot s, BatchBufs b)
{
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= b.n_txns) return;
    if (b.q_slice_set && b.q_slice_set[t] != SLICE_STORE && b.q_slice_set[t] >= s.n_ssets) set_error(b.ctl, ERR_SLICE);
    const uint64_t tm = b.q_txn_msb[t], tl = b.q_txn_lsb[t];
    const int32_t tn = b.q_txn_node[t];
    const uint64_t em = b.q_exec_msb[t], el = b.q_exec_lsb[t];
    const int32_t en = b.q_exec_node[t];
    const uint32_t kinds = kind_witnesses((uint32_t)((tl >> 1) & 7));   // txnId.kind().witnesses()
    if (kinds == 0) set_error(b.ctl, ERR_INVAL);
    // p1 = executeAt.equals(txnId) ? null : txnId   (PreAccept.java:261)
    const bool same = em == tm && ((el ^ tl) & 0xFFFFFFFFFFFF001EULL) == 0 && en == tn;
    b.t_S[t] = encode_rank(s, em, el, en);
    b.t_self[t] = same ? 0u : encode_rank(s, tm, tl, tn);
    b.t_kinds[t] = kinds | ((uint32_t)kinds_class(kinds) << 8);
    b.t_epoch[t] = (int64_t)(em >> 15);
    for (uint64_t p = b.q_key_off[t]; p < b.q_key_off[t + 1]; ++p) b.p_txn[p] = (uint32_t)t;
}

__global__ void k_probe_keys(DevSnapshot s, BatchBufs b)
{
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= b.n_probes) return;
    const int64_t key = b.q_keys[p];
    const uint32_t t = b.p_txn[p];
    const uint32_t pk = b.p_kind ? b.p_kind[p] : PK_KEY;
    if (pk >= PK_RANGE)
    {
        // a range of a Range-domain request: no CommandsForKey (K1 visits nothing); K4 probes the range
        // commands (sliced range, "in slice") or the redundant-before entries (unsliced range)
        b.p_rec[p] = make_uint4(NO_KEY, b.t_S[t], b.t_self[t], b.t_kinds[t] | (pk == PK_RANGE ? (1u << 12) : 0u) | (pk << 13));
        return;
    }
    const bool in_slice = slice_has(s.start_inclusive, request_slice(s, b.q_slice_set, t), key);
    uint32_t ki = NO_KEY;
    if (in_slice)
    {
        uint64_t lo = 0, hi = s.n_keys;
        while (lo < hi)
        {
            const uint64_t mid = (lo + hi) >> 1;
            if (s.keys[mid] < key) lo = mid + 1;
            else hi = mid;
        }
        if (lo < s.n_keys && s.keys[lo] == key) ki = (uint32_t)lo;   // ifLoadedAndInitialised(key) != null
    }
    b.p_rec[p] = make_uint4(ki, b.t_S[t], b.t_self[t], b.t_kinds[t] | (in_slice ? (1u << 12) : 0u) | (pk << 13));
}

hipError_t run_encode(const DevSnapshot& s, const BatchBufs& b, hipStream_t st)
{
    if (b.n_txns)
        k_encode_txn<<<(unsigned)((b.n_txns + 255) / 256), 256, 0, st>>>(s, b);
    if (b.n_probes)
        k_probe_keys<<<(unsigned)((b.n_probes + 255) / 256), 256, 0, st>>>(s, b);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// Range-domain requests (SafeCommandStore.mapReduceActive over Ranges, SafeCommandStore.java:292):
// every request becomes probes. A key-domain request keeps its keys (PK_KEY). A Range-domain request
// gets, per range sliced to the store (Ranges.slice(slice, Minimal): each non-empty intersection with a
// slice range, ascending), the CommandsForKey keys inside it (PK_RANGE_KEY: commandsForKey.subMap(start,
// startInclusive, end, endInclusive), InMemoryCommandStore.java:289-304) followed by the range itself
// (PK_RANGE, when the store has range commands: mapReduceRangesInternal's intersects/foldl,
// :951-960), and at the end its unsliced ranges (PK_RANGE_RB, when the store has redundant-before
// entries: RedundantBefore.collectDeps over the request's Seekables, RedundantBefore.java:420-423).
// The keys come out ascending (sliced ranges ascending and disjoint), which is all K2 needs: range
// probes contribute no keyDeps keys.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ bool slice_part(const SliceView& v, int64_t a, int64_t b, uint64_t sl, int64_t* lo, int64_t* hi)
{
    if (v.all)
    {
        *lo = a;
        *hi = b;
        return a < b;
    }
    *lo = a > v.st[sl] ? a : v.st[sl];
    *hi = b < v.en[sl] ? b : v.en[sl];
    return *lo < *hi;
}
// parts of one range against the slice: one per slice range (every key: the range itself)
__device__ __forceinline__ uint64_t slice_parts(const SliceView& v) { return v.all ? 1 : v.n; }

__global__ __launch_bounds__(256) void k_range_count(DevSnapshot s, uint64_t n, const uint64_t* __restrict__ key_off,
                                                     const uint64_t* __restrict__ range_off,
                                                     const int64_t* __restrict__ range_start,
                                                     const int64_t* __restrict__ range_end, uint32_t* __restrict__ cnt,
                                                     uint32_t* err, uint32_t* __restrict__ list, bool with_rb)
{
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool on = t < n;
    const uint64_t r0 = on ? range_off[t] : 0, r1 = on ? range_off[t + 1] : 0;
    const uint64_t nk = on ? key_off[t + 1] - key_off[t] : 0;
    // a Range-domain request: validated here, listed (one atomic per wave), its probe count written by
    // k_range_count_r
    bool bad = r1 != r0 && nk != 0;
    for (uint64_t j = r0; j < r1; ++j)
    {
        const int64_t a = range_start[j], e = range_end[j];
        if (a >= e || (j > r0 && range_end[j - 1] > a)) bad = true;
    }
    if (bad) atomicOr(err, 1u);
    if (on) cnt[t] = r1 == r0 ? (uint32_t)nk : 0u;
    const bool listed = on && r1 != r0 && !bad;
    const uint64_t lm = ballot(listed);
    if (!lm) return;
    uint32_t base = 0;
    if (lane_id() == (uint32_t)(__ffsll((unsigned long long)lm) - 1)) base = atomicAdd(&err[1], (uint32_t)__popcll(lm));
    base = (uint32_t)__shfl((int)base, __ffsll((unsigned long long)lm) - 1, 64);
    if (listed) list[base + __popcll(lm & ((1ull << lane_id()) - 1))] = (uint32_t)t;
}

// the snapshot keys inside [lo, hi) by one wave: two 64-ary searches (k0 = first key inside, k1 = first beyond)
__device__ __forceinline__ void wave_key_span(const DevSnapshot& s, int64_t lo, int64_t hi, bool incl, uint64_t& k0, uint64_t& k1)
{
    // EndInclusive (s, e]: keys > lo and <= hi; StartInclusive [s, e): keys >= lo and < hi
    k0 = wave_lower_bound(0, s.n_keys, [&](uint64_t i) { return s.keys[i]; }, [&](int64_t v) { return incl ? v < lo : v <= lo; });
    k1 = wave_lower_bound(k0, s.n_keys, [&](uint64_t i) { return s.keys[i]; }, [&](int64_t v) { return incl ? v < hi : v <= hi; });
}

// one wave per listed Range-domain request: its probe count (keys inside each sliced part, + the part itself with
// range commands, + its unsliced ranges with RedundantBefore entries)
__global__ __launch_bounds__(256) void k_range_count_r(DevSnapshot s, const uint32_t* __restrict__ list,
                                                       const uint32_t* __restrict__ n_list,
                                                       const uint64_t* __restrict__ range_off,
                                                       const int64_t* __restrict__ range_start,
                                                       const int64_t* __restrict__ range_end, const uint32_t* __restrict__ sset,
                                                       uint32_t* __restrict__ cnt, bool with_rb)
{
    const uint64_t li = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (li >= *n_list) return;
    const uint64_t t = list[li];
    const uint64_t r0 = range_off[t], r1 = range_off[t + 1];
    const bool incl = s.start_inclusive != 0;
    const SliceView sv = request_slice(s, sset, t);
    const uint64_t n_sl = slice_parts(sv);
    uint64_t c = 0;
    for (uint64_t j = r0; j < r1; ++j)
    {
        const int64_t a = range_start[j], e = range_end[j];
        for (uint64_t sl = 0; sl < n_sl; ++sl)
        {
            int64_t lo, hi;
            if (!slice_part(sv, a, e, sl, &lo, &hi)) continue;
            uint64_t k0, k1;
            wave_key_span(s, lo, hi, incl, k0, k1);
            c += k1 - k0;
            if (s.n_rent) ++c;
        }
    }
    if (s.n_rb && with_rb) c += r1 - r0;
    if (lane_id() == 0) cnt[t] = (uint32_t)min<uint64_t>(c, 0xFFFFFFFFull);
}

// a key-domain request's keys, 8 lanes per request (a wave copies 8 consecutive requests' keys, coalesced at both
// ends); its range end is never read (PK_KEY)
__global__ __launch_bounds__(256) void k_range_fill_keys(uint64_t n, const uint64_t* __restrict__ key_off,
                                                         const int64_t* __restrict__ keys,
                                                         const uint64_t* __restrict__ range_off,
                                                         const uint64_t* __restrict__ off, int64_t* __restrict__ pkeys,
                                                         uint8_t* __restrict__ pkind)
{
    const uint64_t t = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 3;
    const uint32_t j = threadIdx.x & 7u;
    if (t >= n || range_off[t + 1] != range_off[t]) return;
    const uint64_t k0 = key_off[t], nk = key_off[t + 1] - k0, o = off[t];
    for (uint64_t i = j; i < nk; i += 8)
    {
        pkeys[o + i] = keys[k0 + i];
        pkind[o + i] = PK_KEY;
    }
}

// one wave per Range-domain request (list): the sliced ranges in order, their keys written lane-strided
__global__ __launch_bounds__(256) void k_range_fill(DevSnapshot s, const uint32_t* __restrict__ list, uint32_t n_list,
                                                    const uint64_t* __restrict__ range_off,
                                                    const int64_t* __restrict__ range_start,
                                                    const int64_t* __restrict__ range_end, const uint32_t* __restrict__ sset,
                                                    const uint64_t* __restrict__ off, int64_t* __restrict__ pkeys,
                                                    int64_t* __restrict__ pkeys_hi, uint8_t* __restrict__ pkind, bool with_rb)
{
    const uint64_t li = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (li >= n_list) return;
    const uint64_t t = list[li];
    const uint32_t lane = lane_id();
    const uint64_t r0 = range_off[t], r1 = range_off[t + 1];
    uint64_t o = off[t];
    const uint64_t o_end = off[t + 1];
    if (o_end == o) return;                      // rejected (k_range_count) or nothing to visit
    const bool incl = s.start_inclusive != 0;
    const SliceView sv = request_slice(s, sset, t);
    const uint64_t n_sl = slice_parts(sv);
    for (uint64_t j = r0; j < r1; ++j)
    {
        const int64_t a = range_start[j], e = range_end[j];
        for (uint64_t sl = 0; sl < n_sl; ++sl)
        {
            int64_t lo, hi;
            if (!slice_part(sv, a, e, sl, &lo, &hi)) continue;
            uint64_t k0, k1;
            wave_key_span(s, lo, hi, incl, k0, k1);
            for (uint64_t i = lane; i < k1 - k0; i += 64)
            {
                pkeys[o + i] = s.keys[k0 + i];
                pkeys_hi[o + i] = 0;
                pkind[o + i] = PK_RANGE_KEY;
            }
            o += k1 - k0;
            if (s.n_rent)
            {
                if (lane == 0)
                {
                    pkeys[o] = lo;
                    pkeys_hi[o] = hi;
                    pkind[o] = PK_RANGE;
                }
                ++o;
            }
        }
    }
    if (s.n_rb && with_rb)
        for (uint64_t j = r0 + lane; j < r1; j += 64)
        {
            pkeys[o + (j - r0)] = range_start[j];
            pkeys_hi[o + (j - r0)] = range_end[j];
            pkind[o + (j - r0)] = PK_RANGE_RB;
        }
}

hipError_t run_range_count(const DevSnapshot& s, uint64_t n, const uint64_t* key_off, const uint64_t* range_off,
                           const int64_t* range_start, const int64_t* range_end, const uint32_t* sset, uint32_t* cnt,
                           uint32_t* err, uint32_t* list, uint64_t max_list, bool with_rb, hipStream_t st)
{
    if (!n) return hipSuccess;
    k_range_count<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(s, n, key_off, range_off, range_start, range_end, cnt, err,
                                                               list, with_rb);
    // the listed requests' counts: a wave each, the grid sized for every range of the batch (the list is shorter)
    const uint64_t m = std::min<uint64_t>(max_list, n);
    if (m)
        k_range_count_r<<<(unsigned)((m + 3) / 4), 256, 0, st>>>(s, list, err + 1, range_off, range_start, range_end, sset,
                                                                 cnt, with_rb);
    return hipGetLastError();
}

hipError_t run_range_fill(const DevSnapshot& s, uint64_t n, const uint64_t* key_off, const int64_t* keys,
                          const uint64_t* range_off, const int64_t* range_start, const int64_t* range_end,
                          const uint32_t* sset, const uint64_t* off, int64_t* pkeys, int64_t* pkeys_hi, uint8_t* pkind,
                          const uint32_t* list, uint32_t n_list, bool with_rb, hipStream_t st)
{
    if (n) k_range_fill_keys<<<(unsigned)((8 * n + 255) / 256), 256, 0, st>>>(n, key_off, keys, range_off, off, pkeys, pkind);
    if (n_list)
        k_range_fill<<<(unsigned)((n_list + 3) / 4), 256, 0, st>>>(s, list, n_list, range_off, range_start, range_end, sset, off,
                                                                   pkeys, pkeys_hi, pkind, with_rb);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// K1: CommandsForKey.mapReduceActive, one wave per (request, key) probe
// ---------------------------------------------------------------------------------------
constexpr int K1_WAVES = 4;
constexpr int K1_CAP = 1024;        // LDS staging per wave (u32; k_recover, k_scan's default)
constexpr uint32_t K1_CHUNK = 4096; // arena chunk per wave refill

struct ChunkAlloc {
    uint64_t cur = 0, end = 0;
    // wave-uniform allocation of n elements, contiguous
    __device__ __forceinline__ uint64_t take(unsigned long long* top, unsigned long long cap, unsigned* overflow,
                                             unsigned ovf_bit, uint64_t n, uint64_t chunk)
    {
        if (n > end - cur)
        {
            const uint64_t sz = n > chunk ? n : chunk;
            unsigned long long base = 0;
            if (lane_id() == 0) base = atomicAdd(top, (unsigned long long)sz);
            base = uniform64(base);
            if (base + sz > cap && lane_id() == 0) atomicOr(overflow, ovf_bit);
            cur = base;
            end = base + sz;
        }
        const uint64_t r = cur;
        cur += n;
        return r;
    }
};

// CAP: LDS staging per wave (u32); a probe emitting more replays its descent straight into the arena
template <int CAP>
__global__ __launch_bounds__(256) void k_scan(DevSnapshot s, BatchBufs b)
{
    __shared__ uint32_t stage[K1_WAVES][CAP];
    __shared__ uint64_t stk[K1_WAVES][2 * MAX_LEVELS];
    const int wv = threadIdx.x >> 6;
    const uint32_t lane = lane_id();
    const uint64_t nw = (uint64_t)gridDim.x * K1_WAVES;
    ChunkAlloc alloc;
    const unsigned long long cap = b.ctl->key_cap;

    for (uint64_t p = (uint64_t)blockIdx.x * K1_WAVES + wv; p < b.n_probes; p += nw)
    {
        const uint4 pr = b.p_rec[p];
        const uint32_t ki = pr.x;
        if (ki == NO_KEY)
        {
            if (lane == 0) { b.p_off[p] = 0; b.p_c0[p] = 0; b.p_c1[p] = 0; }
            continue;
        }
        const uint32_t S = pr.y, self = pr.z;
        const uint32_t kinds = pr.w & 0xFF;
        const int cls = (pr.w >> 8) & 3;
        const KeyRec kr = s.krec[ki];
        const uint64_t lo = kr.seg_lo, hi = kr.seg_hi;

        // end = insertPos(startedBefore)  (CommandsForKey.java:912, :1358-1363); tail fast path
        const uint64_t end = (hi == lo || kr.last_txn < S)
                                 ? hi
                                 : wave_lower_bound(lo, hi, [&](uint64_t i) { return s.ent[i].y & RANK_MASK; },
                                                    [&](uint32_t v) { return v < S; });

        // maxCommittedWriteBefore (:913-928): executeAt of the last committed Write before S
        const uint64_t wlo = kr.w_lo, whi = kr.w_hi;
        uint64_t wpos = wlo;
        uint32_t wprev = 0;
        if (whi > wlo)
        {
            if (kr.last_wexec < S)
            {
                wpos = whi;
                wprev = kr.last_wexec;
            }
            else
            {
                wpos = wave_lower_bound(wlo, whi, [&](uint64_t i) { return s.w[i].x; }, [&](uint32_t v) { return v < S; });
                if (wpos > wlo) wprev = s.w[wpos - 1].x;
            }
        }
        const uint32_t M = (s.elide && wpos > wlo) ? wprev : 1u;   // 1: "none", every live entry passes

        // prunedBefore substitute (:952-965): first Write at/after S, clamped to maxAppliedWrite
        uint32_t extra = 0;
        if (kr.pruned != 0 && S <= kr.pruned)
        {
            // no applied Write: binarySearch(committedByExecuteAt, 0, -1, S) = -1, the walk starts
            // at the first committed entry (:955-962); no committed Write at all throws
            if (kr.maw < 0 && whi == wlo) { if (lane == 0) set_error(b.ctl, ERR_STATE); }
            else
            {
                const uint64_t idx = kr.maw < 0 ? wlo : (wpos <= (uint64_t)kr.maw ? wpos : (uint64_t)kr.maw);
                extra = s.w[idx].y;
                if (extra == self) extra = 0;                      // map lambda, PreAccept.java:258
            }
        }

        uint32_t cursor = 0, c0 = 0, c1 = 0, nlt = 0;
        bool overflow = false, dup = false;
        auto node_want = [&](int lv, uint64_t node) { return s.lvl[cls][lv][node] >= M; };
        auto want_of = [&](uint64_t i, bool inr, uint32_t& r, bool& is1) -> bool {
            const uint2 e = inr ? s.ent[i] : make_uint2(0u, 0u);
            r = e.y & RANK_MASK;
            const uint32_t kd = e.y >> RANK_BITS;
            is1 = ((KINDS_RS_OR_WS >> kd) & 1) == 0;           // !managesExecution -> directKeyDeps
            // testKind.test(kind); status/elision via tau >= M; self exclusion (PreAccept.java:258)
            return inr && e.x >= M && ((kinds >> kd) & 1) && r != self;
        };
        auto leaf_stage = [&](uint64_t base, bool inr) {
            uint32_t r;
            bool is1;
            const bool want = want_of(base + lane, inr, r, is1);
            const uint64_t wm = ballot(want), w1 = ballot(want && is1);
            c0 += __popcll(wm & ~w1);
            c1 += __popcll(w1);
            if (extra)
            {
                nlt += __popcll(ballot(want && !is1 && r < extra));
                dup |= ballot(want && r == extra) != 0;
            }
            const uint32_t n = __popcll(wm);
            if (!overflow && cursor + n <= CAP)
            {
                if (want) stage[wv][cursor + mbcnt(wm)] = r | (is1 ? CLASS_DIRECT_BIT : 0u);
                cursor += n;
            }
            else overflow = true;
        };
        wave_descent(lo, end, s.n_levels, node_want, leaf_stage, stk[wv]);

        wave_lds_sync();
        const bool has_extra = extra != 0 && !dup;
        const uint32_t tot0 = c0 + (has_extra ? 1u : 0u), tot = tot0 + c1;
        const uint64_t off = alloc.take(&b.ctl->key_top, cap, &b.ctl->overflow, 1u, tot, K1_CHUNK);
        const bool fits = off + tot <= cap;
        if (fits)
        {
            if (!overflow)
            {
                uint32_t run0 = 0, run1 = 0;
                for (uint32_t i0 = 0; i0 < cursor; i0 += 64)
                {
                    const uint32_t i = i0 + lane;
                    const bool v = i < cursor;
                    const uint32_t x = v ? stage[wv][i] : 0u;
                    const bool is1 = v && (x & CLASS_DIRECT_BIT);
                    const bool is0 = v && !is1;
                    const uint32_t r = x & ~CLASS_DIRECT_BIT;
                    const uint64_t m0 = ballot(is0), m1 = ballot(is1);
                    if (is0) b.arena[off + run0 + mbcnt(m0) + ((has_extra && r > extra) ? 1 : 0)] = r;
                    if (is1) b.arena[off + tot0 + run1 + mbcnt(m1)] = r;
                    run0 += __popcll(m0);
                    run1 += __popcll(m1);
                }
            }
            else
            {
                // staging overflowed: replay the descent writing straight to the exact allocation
                uint32_t run0 = 0, run1 = 0;
                auto leaf_direct = [&](uint64_t base, bool inr) {
                    uint32_t r;
                    bool is1;
                    const bool want = want_of(base + lane, inr, r, is1);
                    const uint64_t w1 = ballot(want && is1), w0 = ballot(want && !is1);
                    if (want && !is1) b.arena[off + run0 + mbcnt(w0) + ((has_extra && r > extra) ? 1 : 0)] = r;
                    if (want && is1) b.arena[off + tot0 + run1 + mbcnt(w1)] = r;
                    run0 += __popcll(w0);
                    run1 += __popcll(w1);
                };
                wave_descent(lo, end, s.n_levels, node_want, leaf_direct, stk[wv]);
            }
            if (has_extra && lane == 0) b.arena[off + nlt] = extra;
        }
        if (lane == 0)
        {
            // on arena overflow record an empty list (the host grows the arena and reruns)
            b.p_off[p] = fits ? (uint32_t)off : 0u;
            b.p_c0[p] = fits ? tot0 : 0u;
            b.p_c1[p] = fits ? c1 : 0u;
        }
    }
}

hipError_t run_scan(const DevSnapshot& s, const BatchBufs& b, hipStream_t st)
{
    if (!b.n_probes) return hipSuccess;
    const uint64_t blocks_needed = (b.n_probes + K1_WAVES - 1) / K1_WAVES;
    // 1024 staged ids per wave (2048 / 4096 -- fewer replayed descents for hot keys at fewer waves per CU --
    // measured slower on the steady state: resolve 3.76 -> 3.93 / 4.06 ms; the selection was deleted in round 6)
    const unsigned grid = (unsigned)std::min<uint64_t>(blocks_needed, (uint64_t)device_cu_count() * 8);
    k_scan<K1_CAP><<<grid, 256, 0, st>>>(s, b);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// K4: range commands + redundant-before, one wave per probe
// ---------------------------------------------------------------------------------------
constexpr int K4_WAVES = 4;
constexpr int K4_CAP = 512;          // LDS staging per wave (u64)
constexpr uint32_t K4_CHUNK = 2048;

__global__ __launch_bounds__(256) void k_range(DevSnapshot s, BatchBufs b)
{
    __shared__ uint64_t stage[K4_WAVES][K4_CAP];
    __shared__ uint64_t stk[K4_WAVES][2 * MAX_LEVELS];
    const int wv = threadIdx.x >> 6;
    const uint32_t lane = lane_id();
    const uint64_t nw = (uint64_t)gridDim.x * K4_WAVES;
    ChunkAlloc alloc;
    const unsigned long long cap = b.ctl->rng_cap;
    const bool incl = s.start_inclusive != 0;

    for (uint64_t p = (uint64_t)blockIdx.x * K4_WAVES + wv; p < b.n_probes; p += nw)
    {
        const int64_t x = b.q_keys[p];
        const uint4 pr = b.p_rec[p];
        const uint32_t pk = (pr.w >> 13) & 3;
        // a range [x, xe) of a Range-domain request (PK_RANGE sliced, PK_RANGE_RB unsliced)
        const int64_t xe = pk >= PK_RANGE ? b.q_keys_hi[p] : 0;
        if (pk == PK_RANGE_RB)
        {
            // RedundantBefore.collectDeps over the request's ranges (RedundantBefore.java:420-423): every
            // entry intersecting [x, xe) (Range.compareIntersecting, Range.java:296-305) -- the entries are
            // disjoint and ascending, so they form one run -- in epoch bounds (:262-265) with a watermark
            // above NONE (:188); values (rid << 32 | rank) ascending with the entries
            const uint64_t e0 = wave_lower_bound(0, s.n_rb, [&](uint64_t i) { return s.rb_end[i]; },
                                                 [&](int64_t v) { return v <= x; });
            const uint64_t e1 = wave_lower_bound(0, s.n_rb, [&](uint64_t i) { return s.rb_start[i]; },
                                                 [&](int64_t v) { return v < xe; });
            const uint32_t t = b.p_txn[p];
            const int64_t ep = b.t_epoch[t];
            const int64_t mine = b.q_min_epoch ? b.q_min_epoch[t] : 0;
            auto ok = [&](uint64_t e) { return !(ep < s.rb_e0[e] || mine >= s.rb_e1[e]) && s.rb_wm[e] != 0; };
            uint32_t cnt = 0;
            for (uint64_t e0r = e0; e0r < e1; e0r += 64)
            {
                const uint64_t e = e0r + lane;
                cnt += __popcll(ballot(e < e1 && ok(e)));
            }
            uint64_t off = cnt ? alloc.take(&b.ctl->rng_top, cap, &b.ctl->overflow, 2u, cnt, K4_CHUNK) : 0;
            if (off + cnt > cap)
            {
                off = 0;
                cnt = 0;                 // overflow: the host grows the arena and reruns
            }
            else if (cnt)
            {
                uint32_t run = 0;
                for (uint64_t e0r = e0; e0r < e1; e0r += 64)
                {
                    const uint64_t e = e0r + lane;
                    const bool want = e < e1 && ok(e);
                    const uint64_t wm = ballot(want);
                    if (want) b.rarena[off + run + mbcnt(wm)] = ((uint64_t)s.rb_rid[e] << 32) | s.rb_wm[e];
                    run += __popcll(wm);
                }
            }
            if (lane == 0)
            {
                b.p_roff[p] = (uint32_t)off;
                b.p_rcnt[p] = cnt;
                b.p_rb[p] = NO_RB;
            }
            continue;
        }
        // RedundantBefore.collectDeps over the request's keys (not sliced), RedundantBefore.java:420-423
        uint64_t rbv = NO_RB;
        if (s.n_rb && pk == PK_KEY)
        {
            const uint64_t c = wave_lower_bound(0, s.n_rb, [&](uint64_t i) { return s.rb_start[i]; },
                                                [&](int64_t v) { return incl ? v <= x : v < x; });
            if (c > 0)
            {
                const uint64_t e = c - 1;
                if (range_contains(s.start_inclusive, s.rb_start[e], s.rb_end[e], x))
                {
                    // Entry.outOfBounds(minEpoch, executeAt) :262-265; watermark > NONE :188
                    const uint32_t t = b.p_txn[p];
                    const int64_t ep = b.t_epoch[t];
                    const int64_t mine = b.q_min_epoch ? b.q_min_epoch[t] : 0;
                    const uint32_t wm = s.rb_wm[e];
                    if (!(ep < s.rb_e0[e] || mine >= s.rb_e1[e]) && wm != 0)
                        rbv = ((uint64_t)s.rb_rid[e] << 32) | wm;
                }
            }
        }

        uint32_t cnt = 0;
        uint64_t off = 0;
        if (((pr.w >> 12) & 1) && s.n_rent && pk != PK_RANGE_KEY)
        {
            const uint32_t S = pr.y, self = pr.z;
            const uint32_t kinds = pr.w & 0xFF;
            const int cls = (pr.w >> 8) & 3;
            // candidate commands: range start before the key (Range.compareTo, Range.java:40-100), or for
            // a sliced range [x, xe) of a Range-domain request, start before its end and end after its start
            // (Range.compareIntersecting, Range.java:296-305): the same prefix + max-end threshold
            const bool rq = pk == PK_RANGE;
            const uint64_t hi = wave_lower_bound(0, s.n_rent, [&](uint64_t i) { return s.r_start[i]; },
                                                 [&](int64_t v) { return rq ? v < xe : (incl ? v <= x : v < x); });
            auto end_ok = [&](int64_t e) { return rq ? e > x : (incl ? e > x : e >= x); };
            auto node_want = [&](int lv, uint64_t node) { return end_ok(s.rlvl[cls][lv][node]); };
            uint32_t cursor = 0;
            bool overflow = false;
            auto want_of = [&](uint64_t i, bool inr, uint64_t& val) -> bool {
                bool want = false;
                val = 0;
                if (inr)
                {
                    const uint32_t txw = s.r_txw[i];
                    const uint32_t r = txw & RANK_MASK, kd = txw >> RANK_BITS;
                    // STARTED_BEFORE (:906-908), testKind (:933), contains key (:948-956), self (PreAccept.java:258)
                    want = end_ok(s.r_end[i]) && r < S && ((kinds >> kd) & 1) && r != self;
                    val = ((uint64_t)s.r_rid[i] << 32) | r;
                }
                return want;
            };
            auto leaf_stage = [&](uint64_t base, bool inr) {
                uint64_t v;
                const bool want = want_of(base + lane, inr, v);
                const uint64_t wm = ballot(want);
                const uint32_t n = __popcll(wm);
                if (!overflow && cursor + n <= K4_CAP)
                {
                    if (want) stage[wv][cursor + mbcnt(wm)] = v;
                }
                else overflow = true;
                cursor += n;
            };
            wave_descent(0, hi, s.n_rlevels, node_want, leaf_stage, stk[wv]);
            wave_lds_sync();
            cnt = cursor;
            off = alloc.take(&b.ctl->rng_top, cap, &b.ctl->overflow, 2u, cnt, K4_CHUNK);
            if (off + cnt > cap)
            {
                off = 0;
                cnt = 0;                 // overflow: the host grows the arena and reruns
            }
            else
            {
                if (!overflow)
                {
                    for (uint32_t i = lane; i < cnt; i += 64) b.rarena[off + i] = stage[wv][i];
                }
                else
                {
                    uint32_t run = 0;
                    auto leaf_direct = [&](uint64_t base, bool inr) {
                        uint64_t v;
                        const bool want = want_of(base + lane, inr, v);
                        const uint64_t wm = ballot(want);
                        if (want) b.rarena[off + run + mbcnt(wm)] = v;
                        run += __popcll(wm);
                    };
                    wave_descent(0, hi, s.n_rlevels, node_want, leaf_direct, stk[wv]);
                }
            }
        }
        if (lane == 0)
        {
            b.p_roff[p] = (uint32_t)off;
            b.p_rcnt[p] = cnt;
            b.p_rb[p] = rbv;
        }
    }
}

hipError_t run_range(const DevSnapshot& s, const BatchBufs& b, hipStream_t st)
{
    if (!b.n_probes) return hipSuccess;
    if (s.n_rent == 0 && s.n_rb == 0)
    {
        // no range commands and no redundant-before entries: every probe's range list is empty
        hipError_t e = hipMemsetAsync(b.p_rcnt, 0, sizeof(uint32_t) * b.n_probes, st);
        if (e == hipSuccess) e = hipMemsetAsync(b.p_rb, 0xFF, sizeof(uint64_t) * b.n_probes, st);
        return e;
    }
    const uint64_t blocks_needed = (b.n_probes + K4_WAVES - 1) / K4_WAVES;
    const unsigned grid = (unsigned)std::min<uint64_t>(blocks_needed, (uint64_t)device_cu_count() * 8);
    k_range<<<grid, 256, 0, st>>>(s, b);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// K2: per request, build keyDeps / directKeyDeps / rangeDeps in RelationMultiMap CSR form.
//
// Multi-list union ("rank merge"): lists L_0..L_{n-1}, each sorted and duplicate-free.
//   kept(x in L_a)  = no L_b, b < a, contains x      (first occurrence of each distinct value)
//   P               = exclusive prefix of kept over the concatenation
//   urank(x)        = sum_b (P[lb_b(x)] - P[st_b])     = number of distinct values < x
// so values[urank(x)] = x for kept x, and urank(x) is the keysToTxnIds body entry of x
// (RelationMultiMap.java:245-257). One wave per request, single pass: every list is gathered
// with one cooperative load per 64 elements, merged in LDS (global scratch when too large),
// and the three maps are written to a chunk-allocated region that k_pack later compacts.
// ---------------------------------------------------------------------------------------
constexpr uint32_t K2_MAXP = 64;     // probes per request on the LDS path
constexpr uint32_t K2_CAP = 512;     // elements per list family on the LDS path
constexpr uint32_t K2_REGION_CHUNK = 1u << 14;


struct K2Mem {
    // per-probe metadata
    uint32_t* off; uint32_t* c0; uint32_t* c1; uint32_t* roff; uint32_t* rcnt; uint64_t* rb;
    uint32_t* st0; uint32_t* st1; uint32_t* stR;      // [np+1], [np+1], [2np+1]
    uint64_t* V;       // [cap] elements
    uint32_t* P;       // [cap + 1]
    uint64_t* UP;      // [cap] unique pairs
    uint32_t* gst;     // [cap + 1] rid group starts
    uint32_t* P2;      // [cap + 1]
};

constexpr size_t k2_lds_bytes()
{
    return (size_t)K2_MAXP * (4 * 5 + 8) + (size_t)(2 * (K2_MAXP + 1) + 2 * K2_MAXP + 1) * 4 + 4 /*align*/ +
           (size_t)K2_CAP * 8 * 2 + (size_t)(K2_CAP + 1) * 4 * 3;
}

__device__ __forceinline__ uint64_t k2_scratch_bytes(uint32_t np, uint32_t capn)
{
    uint64_t b = (uint64_t)np * 8 + (uint64_t)np * 4 * 5 + (uint64_t)(2 * (np + 1) + 2 * np + 1) * 4;
    b = (b + 7) & ~7ull;
    b += (uint64_t)capn * 16 + (uint64_t)(capn + 1) * 12;
    return (b + 7) & ~7ull;
}

__device__ __forceinline__ void k2_carve(K2Mem& m, uint8_t* base, uint32_t np, uint32_t capn)
{
    m.rb = reinterpret_cast<uint64_t*>(base);
    m.off = reinterpret_cast<uint32_t*>(m.rb + np);
    m.c0 = m.off + np;
    m.c1 = m.c0 + np;
    m.roff = m.c1 + np;
    m.rcnt = m.roff + np;
    m.st0 = m.rcnt + np;
    m.st1 = m.st0 + (np + 1);
    m.stR = m.st1 + (np + 1);
    uint8_t* q = reinterpret_cast<uint8_t*>(m.stR + (2 * np + 1));
    q = reinterpret_cast<uint8_t*>(((uintptr_t)q + 7) & ~(uintptr_t)7);
    m.V = reinterpret_cast<uint64_t*>(q);
    m.UP = m.V + capn;
    m.P = reinterpret_cast<uint32_t*>(m.UP + capn);
    m.gst = m.P + (capn + 1);
    m.P2 = m.gst + (capn + 1);
}

template <class Get>
__device__ __forceinline__ uint32_t lb_in(Get get, uint32_t lo, uint32_t hi, uint64_t x)
{
    while (lo < hi)
    {
        const uint32_t mid = (lo + hi) >> 1;
        if (get(mid) < x) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// list of element e: the largest a with st[a] <= e (st ascending, st[n] = total)
__device__ __forceinline__ uint32_t list_of(const uint32_t* st, uint32_t n, uint32_t e)
{
    uint32_t lo = 0, hi = n;                 // answer in [0, n)
    while (hi - lo > 1)
    {
        const uint32_t mid = (lo + hi) >> 1;
        if (st[mid] <= e) lo = mid;
        else hi = mid;
    }
    return lo;
}

// exclusive wave scan of cnt(i), i < n, into st[0..n]; returns total
template <class Cnt>
__device__ __forceinline__ uint32_t wave_list_starts(uint32_t n, Cnt cnt, uint32_t* st)
{
    uint32_t carry = 0;
    for (uint32_t i0 = 0; i0 < n; i0 += 64)
    {
        const uint32_t i = i0 + lane_id();
        const uint32_t c = i < n ? cnt(i) : 0u;
        const uint32_t inc = wave_incl_scan(c);
        if (i < n) st[i] = carry + inc - c;
        carry += __shfl(inc, 63, 64);
    }
    if (lane_id() == 0) st[n] = carry;
    return carry;
}

__device__ __forceinline__ void wave_excl_scan_inplace(uint32_t* P, uint32_t n)
{
    uint32_t carry = 0;
    for (uint32_t i0 = 0; i0 < n; i0 += 64)
    {
        const uint32_t i = i0 + lane_id();
        const uint32_t v = i < n ? P[i] : 0u;
        const uint32_t inc = wave_incl_scan(v);
        if (i < n) P[i] = carry + inc - v;
        carry += __shfl(inc, 63, 64);
    }
    if (lane_id() == 0) P[n] = carry;
}

// kept flags + prefix; returns number of distinct values. Get(e) = element e of the concatenation.
template <class Get>
__device__ __forceinline__ uint32_t rank_merge_kept(Get get, const uint32_t* st, uint32_t nl, uint32_t total, uint32_t* P)
{
    for (uint32_t e0 = 0; e0 < total; e0 += 64)
    {
        const uint32_t e = e0 + lane_id();
        if (e < total)
        {
            const uint32_t a = list_of(st, nl, e);
            const uint64_t x = get(e);
            uint32_t kept = 1;
            for (uint32_t bl = 0; bl < a && kept; ++bl)
            {
                const uint32_t s0 = st[bl], s1 = st[bl + 1];
                if (s1 > s0)
                {
                    const uint32_t j = lb_in(get, s0, s1, x);
                    if (j < s1 && get(j) == x) kept = 0;
                }
            }
            P[e] = kept;
        }
    }
    __syncthreads();
    wave_excl_scan_inplace(P, total);
    __syncthreads();
    return uniform(P[total]);
}

// after rank_merge_kept: unique rank of value x
template <class Get>
__device__ __forceinline__ uint32_t rank_merge_urank(Get get, const uint32_t* st, uint32_t nl, const uint32_t* P, uint64_t x)
{
    uint32_t sum = 0;
    for (uint32_t bl = 0; bl < nl; ++bl)
    {
        const uint32_t s0 = st[bl], s1 = st[bl + 1];
        if (s1 > s0) sum += P[lb_in(get, s0, s1, x)] - P[s0];
    }
    return sum;
}

__device__ __forceinline__ uint32_t dict_index(uint32_t rank) { return (rank - 1) >> 1; }

// region of one map of one request: [keys i64 x nk][txns u32 x U][k2t i32 x (nk + pairs)]
__device__ __forceinline__ uint64_t region_bytes(uint32_t nk, uint32_t U, uint32_t pairs)
{
    return ((uint64_t)nk * 8 + (uint64_t)U * 4 + (uint64_t)(nk + pairs) * 4 + 7) & ~7ull;
}

__global__ __launch_bounds__(64) void k_build(DevSnapshot s, BatchBufs b)
{
    extern __shared__ uint64_t lds_raw[];
    const uint32_t lane = lane_id();
    const uint64_t n = b.n_txns;
    ChunkAlloc ralloc;
    for (uint64_t t = blockIdx.x; t < n; t += gridDim.x)
    {
        const uint64_t p0 = b.q_key_off[t];
        const uint32_t np = (uint32_t)(b.q_key_off[t + 1] - p0);

        // one round trip for the request's probe metadata (lane = probe when np <= 64)
        uint32_t r_off = 0, r_c0 = 0, r_c1 = 0, r_roff = 0, r_rcnt = 0;
        uint64_t r_rb = NO_RB;
        uint32_t tot0 = 0, tot1 = 0, totR = 0;
        for (uint32_t i = lane; i < np; i += 64)
        {
            r_off = b.p_off[p0 + i];
            r_c0 = b.p_c0[p0 + i];
            r_c1 = b.p_c1[p0 + i];
            r_roff = b.p_roff[p0 + i];
            r_rcnt = b.p_rcnt[p0 + i];
            r_rb = b.p_rb[p0 + i];
            tot0 += r_c0;
            tot1 += r_c1;
            totR += r_rcnt + (r_rb != NO_RB ? 1u : 0u);
        }
        tot0 = uniform(wave_sum(tot0));
        tot1 = uniform(wave_sum(tot1));
        totR = uniform(wave_sum(totR));
        const uint32_t capn = max(max(tot0, tot1), totR);
        if (capn > b.k2_big)
        {
            // a heavy request (a hot key's in-flight txns): one whole workgroup, k_build_big
            if (lane == 0) b.big[atomicAdd(&b.ctl->n_big, 1ull)] = (uint32_t)t;
            continue;
        }
        const bool big = np > K2_MAXP || capn > K2_CAP;

        K2Mem mem;
        if (!big)
        {
            k2_carve(mem, reinterpret_cast<uint8_t*>(lds_raw), K2_MAXP, K2_CAP);
            if (lane < np)
            {
                mem.off[lane] = r_off; mem.c0[lane] = r_c0; mem.c1[lane] = r_c1;
                mem.roff[lane] = r_roff; mem.rcnt[lane] = r_rcnt; mem.rb[lane] = r_rb;
            }
        }
        else
        {
            const uint64_t bytes = k2_scratch_bytes(np, capn);
            unsigned long long o = 0;
            if (lane == 0) o = atomicAdd(&b.ctl->scr_top, (unsigned long long)bytes);
            const uint64_t so = uniform64(o);
            if (so + bytes > b.ctl->scr_cap)
            {
                if (lane == 0)
                {
                    atomicOr(&b.ctl->overflow, 4u);
                    for (int a = 0; a < 9; ++a) b.sz[a * n + t] = 0;
                }
                continue;
            }
            k2_carve(mem, b.scratch + so, np, capn);
            for (uint32_t i = lane; i < np; i += 64)
            {
                mem.off[i] = b.p_off[p0 + i]; mem.c0[i] = b.p_c0[p0 + i]; mem.c1[i] = b.p_c1[p0 + i];
                mem.roff[i] = b.p_roff[p0 + i]; mem.rcnt[i] = b.p_rcnt[p0 + i]; mem.rb[i] = b.p_rb[p0 + i];
            }
        }
        __syncthreads();
        wave_list_starts(np, [&](uint32_t i) { return mem.c0[i]; }, mem.st0);
        wave_list_starts(np, [&](uint32_t i) { return mem.c1[i]; }, mem.st1);
        wave_list_starts(2 * np, [&](uint32_t i) {
            return (i & 1) ? (mem.rb[i >> 1] != NO_RB ? 1u : 0u) : mem.rcnt[i >> 1];
        }, mem.stR);
        __syncthreads();

        // ---- keyDeps (class 0) and directKeyDeps (class 1)
        for (int c = 0; c < 2; ++c)
        {
            const int m = c == 0 ? 0 : 2;          // AD_MAP_KEY / AD_MAP_DIRECT_KEY
            const uint32_t tot = c == 0 ? tot0 : tot1;
            const uint32_t* st = c == 0 ? mem.st0 : mem.st1;
            if (tot == 0)
            {
                if (lane == 0) { b.sz[(3 * m) * n + t] = 0; b.sz[(3 * m + 1) * n + t] = 0; b.sz[(3 * m + 2) * n + t] = 0; }
                continue;
            }
            // gather: one cooperative load per 64 elements
            for (uint32_t e = lane; e < tot; e += 64)
            {
                const uint32_t a = list_of(st, np, e);
                mem.V[e] = b.arena[(uint64_t)mem.off[a] + (c == 0 ? 0u : mem.c0[a]) + (e - st[a])];
            }
            __syncthreads();
            auto get = [&](uint32_t e) -> uint64_t { return mem.V[e]; };
            const uint32_t U = rank_merge_kept(get, st, np, tot, mem.P);
            uint32_t nk = 0;
            for (uint32_t i0 = 0; i0 < np; i0 += 64)
            {
                const uint32_t i = i0 + lane;
                nk += __popcll(ballot(i < np && st[i + 1] > st[i]));
            }
            const uint64_t rb = region_bytes(nk, U, tot);
            const uint64_t ro = ralloc.take(&b.ctl->reg_top, b.ctl->reg_cap, &b.ctl->overflow, 8u, rb, K2_REGION_CHUNK);
            const bool fits = ro + rb <= b.ctl->reg_cap;
            if (lane == 0)
            {
                b.sz[(3 * m) * n + t] = fits ? nk : 0;
                b.sz[(3 * m + 1) * n + t] = fits ? U : 0;
                b.sz[(3 * m + 2) * n + t] = fits ? nk + tot : 0;
                b.t_reg[(uint64_t)m * n + t] = ro;
            }
            if (fits)
            {
                int64_t* okeys = reinterpret_cast<int64_t*>(b.reg + ro);
                uint32_t* otx = reinterpret_cast<uint32_t*>(okeys + nk);
                int32_t* ok2t = reinterpret_cast<int32_t*>(otx + U);
                // keys + heads (absolute end offsets starting at nKeys)
                uint32_t kr = 0;
                for (uint32_t i0 = 0; i0 < np; i0 += 64)
                {
                    const uint32_t i = i0 + lane;
                    const bool ne = i < np && st[i + 1] > st[i];
                    const uint64_t mk = ballot(ne);
                    if (ne)
                    {
                        const uint32_t k = kr + mbcnt(mk);
                        okeys[k] = b.q_keys[p0 + i];
                        ok2t[k] = (int32_t)(nk + st[i + 1]);
                    }
                    kr += __popcll(mk);
                }
                // values + body
                for (uint32_t e = lane; e < tot; e += 64)
                {
                    const uint64_t x = mem.V[e];
                    const uint32_t ur = rank_merge_urank(get, st, np, mem.P, x);
                    if (mem.P[e + 1] - mem.P[e]) otx[ur] = dict_index((uint32_t)x);
                    ok2t[nk + e] = (int32_t)ur;
                }
            }
            __syncthreads();
        }

        // ---- rangeDeps: lists = per probe [range-command pairs], [redundant pair]
        {
            const uint32_t nl = 2 * np;
            if (totR == 0)
            {
                if (lane == 0) { b.sz[3 * n + t] = 0; b.sz[4 * n + t] = 0; b.sz[5 * n + t] = 0; }
                continue;
            }
            for (uint32_t e = lane; e < totR; e += 64)
            {
                const uint32_t a = list_of(mem.stR, nl, e);
                const uint32_t pi = a >> 1;
                mem.V[e] = (a & 1) ? mem.rb[pi] : b.rarena[(uint64_t)mem.roff[pi] + (e - mem.stR[a])];
            }
            __syncthreads();
            auto get = [&](uint32_t e) -> uint64_t { return mem.V[e]; };
            const uint32_t UPn = rank_merge_kept(get, mem.stR, nl, totR, mem.P);
            // unique pairs, sorted by (rid, rank) = (Range.compare, TxnId.compareTo)
            for (uint32_t e = lane; e < totR; e += 64)
            {
                if (mem.P[e + 1] - mem.P[e])
                {
                    const uint64_t x = mem.V[e];
                    mem.UP[rank_merge_urank(get, mem.stR, nl, mem.P, x)] = x;
                }
            }
            __syncthreads();
            // rid groups
            uint32_t nR = 0;
            for (uint32_t i0 = 0; i0 < UPn; i0 += 64)
            {
                const uint32_t i = i0 + lane;
                const bool first = i < UPn && (i == 0 || (mem.UP[i] >> 32) != (mem.UP[i - 1] >> 32));
                const uint64_t mk = ballot(first);
                if (first) mem.gst[nR + mbcnt(mk)] = i;
                nR += __popcll(mk);
            }
            if (lane == 0) mem.gst[nR] = UPn;
            __syncthreads();
            // distinct txnIds across groups: rank merge over the groups by rank
            auto getr = [&](uint32_t e) -> uint64_t { return mem.UP[e] & 0xFFFFFFFFull; };
            const uint32_t UR = rank_merge_kept(getr, mem.gst, nR, UPn, mem.P2);
            const uint64_t rbytes = region_bytes(nR, UR, UPn);
            const uint64_t ro = ralloc.take(&b.ctl->reg_top, b.ctl->reg_cap, &b.ctl->overflow, 8u, rbytes, K2_REGION_CHUNK);
            const bool fits = ro + rbytes <= b.ctl->reg_cap;
            if (lane == 0)
            {
                b.sz[3 * n + t] = fits ? nR : 0;
                b.sz[4 * n + t] = fits ? UR : 0;
                b.sz[5 * n + t] = fits ? nR + UPn : 0;
                b.t_reg[(uint64_t)1 * n + t] = ro;
            }
            if (fits)
            {
                int64_t* okeys = reinterpret_cast<int64_t*>(b.reg + ro);
                uint32_t* otx = reinterpret_cast<uint32_t*>(okeys + nR);
                int32_t* ok2t = reinterpret_cast<int32_t*>(otx + UR);
                for (uint32_t g = lane; g < nR; g += 64)
                {
                    okeys[g] = (int64_t)(mem.UP[mem.gst[g]] >> 32);
                    ok2t[g] = (int32_t)(nR + mem.gst[g + 1]);
                }
                for (uint32_t e = lane; e < UPn; e += 64)
                {
                    const uint64_t x = getr(e);
                    const uint32_t ur = rank_merge_urank(getr, mem.gst, nR, mem.P2, x);
                    if (mem.P2[e + 1] - mem.P2[e]) otx[ur] = dict_index((uint32_t)x);
                    ok2t[nR + e] = (int32_t)ur;
                }
            }
            __syncthreads();
        }
    }
}

// ---- K2 for heavy requests: the same build with one 1024-thread workgroup per request (a request
// whose lists hold thousands of ids -- a Zipf-hot key's in-flight txns -- would keep one wave busy
// for milliseconds). Every per-element step (gather, rank-merge dedup, unique ranks, writes) is
// spread over the 16 waves; the list starts and the kept-flag prefix are block scans.
constexpr uint32_t KB_THREADS = 1024;
constexpr uint32_t KB_WAVES = KB_THREADS / 64;

struct KbLds {
    uint32_t wsum[KB_WAVES + 1];
    uint32_t red[4];
    unsigned long long so, have, ro;
    uint32_t nk;
};

// exclusive block scan of cnt(i), i < n, into st[0..n] (st may alias the source: each i is read and
// written by one thread); returns the total
template <class Cnt>
__device__ uint32_t block_scan_into(KbLds& L, uint32_t n, Cnt cnt, uint32_t* st)
{
    const uint32_t tid = threadIdx.x, wv = tid >> 6, lane = lane_id();
    uint32_t carry = 0;
    for (uint32_t i0 = 0; i0 < n; i0 += KB_THREADS)
    {
        const uint32_t i = i0 + tid;
        const uint32_t c = i < n ? cnt(i) : 0u;
        const uint32_t inc = wave_incl_scan(c);
        if (lane == 63) L.wsum[wv] = inc;
        __syncthreads();
        if (wv == 0)
        {
            const uint32_t v = lane < KB_WAVES ? L.wsum[lane] : 0u;
            const uint32_t vi = wave_incl_scan(v);
            if (lane < KB_WAVES) L.wsum[lane] = vi - v;
            if (lane == KB_WAVES - 1) L.wsum[KB_WAVES] = vi;
        }
        __syncthreads();
        if (i < n) st[i] = carry + L.wsum[wv] + inc - c;
        carry += L.wsum[KB_WAVES];
        __syncthreads();
    }
    if (tid == 0) st[n] = carry;
    __syncthreads();
    return carry;
}

template <class Get>
__device__ uint32_t block_rank_merge_kept(KbLds& L, Get get, const uint32_t* st, uint32_t nl, uint32_t total, uint32_t* P)
{
    for (uint32_t e = threadIdx.x; e < total; e += KB_THREADS)
    {
        const uint32_t a = list_of(st, nl, e);
        const uint64_t x = get(e);
        uint32_t kept = 1;
        for (uint32_t bl = 0; bl < a && kept; ++bl)
        {
            const uint32_t s0 = st[bl], s1 = st[bl + 1];
            if (s1 > s0)
            {
                const uint32_t j = lb_in(get, s0, s1, x);
                if (j < s1 && get(j) == x) kept = 0;
            }
        }
        P[e] = kept;
    }
    __syncthreads();
    return block_scan_into(L, total, [&](uint32_t i) { return P[i]; }, P);
}

// region of one map: bytes taken exactly (one atomic per request and map); 0 sizes on overflow
__device__ bool kb_region(KbLds& L, const BatchBufs& b, uint64_t bytes, uint64_t* ro)
{
    if (threadIdx.x == 0)
    {
        const unsigned long long o = atomicAdd(&b.ctl->reg_top, (unsigned long long)bytes);
        if (o + bytes > b.ctl->reg_cap) atomicOr(&b.ctl->overflow, 8u);
        L.ro = o;
    }
    __syncthreads();
    *ro = L.ro;
    const bool fits = L.ro + bytes <= b.ctl->reg_cap;
    return fits;
}

// A heavy request's keyDeps / directKeyDeps of at most KB_LDS_CAP elements (over at most KB_LDS_LISTS lists) merge
// in LDS: values, list starts and the kept-flag prefix held there, so the rank merge's binary searches (~8 lists x
// ~12 probes per element, RelationMultiMap's dedup :147-260) read LDS instead of global scratch. (A block bitonic
// sort of (value, element) in LDS measured no better: its ~80 barrier-separated stages cost about what the
// searches through L2 did -- steady-state resolve 8.95 against 9.42 ms.)
constexpr uint32_t KB_LDS_CAP = 16384;
constexpr uint32_t KB_LDS_LISTS = 64;

// The LDS merge as a merge tree (BatchBufs.kb_merge): the np sorted lists of X (starts S) merged pairwise,
// ceil(log2 np) levels ping-ponging between X and Y -- an element's place in the merged run is its place
// in its own run plus its co-rank in the partner run (one binary search per level: strictly-less counts for
// the left run's elements, less-or-equal for the right run's, so equal values keep list order) -- instead
// of the rank merge's searches in every list (~1.5 np searches per element). Then the unique flags of the
// sorted run and their exclusive prefix (Y): an element's unique rank is the prefix at the first occurrence
// of its value. Returns the sorted array (X or Y); *pre the prefix array (the other one), total unique.
__device__ uint32_t block_merge_tree(KbLds& L, uint32_t* X, uint32_t* Y, const uint32_t* S, uint32_t np, uint32_t tot,
                                     uint32_t** sorted, uint32_t** pre)
{
    for (uint32_t l = 0; (1u << l) < np; ++l)
    {
        for (uint32_t e = threadIdx.x; e < tot; e += KB_THREADS)
        {
            const uint32_t a = list_of(S, np, e);
            const uint32_t run = a >> l;
            const uint32_t la = (run & ~1u) << l;
            const uint32_t sA = S[la];
            const uint32_t sB = S[min(la + (1u << l), np)], eB = S[min(la + (2u << l), np)];
            const uint32_t x = X[e];
            uint32_t d;
            if (!(run & 1u))
            {
                uint32_t lo = sB, hi = eB;           // B elements < x
                while (lo < hi)
                {
                    const uint32_t mid = (lo + hi) >> 1;
                    if (X[mid] < x) lo = mid + 1;
                    else hi = mid;
                }
                d = e + (lo - sB);
            }
            else
            {
                uint32_t lo = sA, hi = sB;           // A elements <= x
                while (lo < hi)
                {
                    const uint32_t mid = (lo + hi) >> 1;
                    if (X[mid] <= x) lo = mid + 1;
                    else hi = mid;
                }
                d = sA + (e - sB) + (lo - sA);
            }
            Y[d] = x;
        }
        __syncthreads();
        uint32_t* t = X;
        X = Y;
        Y = t;
    }
    const uint32_t* Xc = X;
    const uint32_t U = block_scan_into(L, tot, [&](uint32_t i) { return (i == 0 || Xc[i] != Xc[i - 1]) ? 1u : 0u; }, Y);
    *sorted = X;
    *pre = Y;
    return U;
}

__global__ __launch_bounds__(KB_THREADS) void k_build_big(DevSnapshot s, BatchBufs b)
{
    __shared__ KbLds L;
    __shared__ uint32_t Vs[KB_LDS_CAP + 1];      // (+1: the merge tree may leave its prefix here)
    __shared__ uint32_t Ps[KB_LDS_CAP + 1];
    __shared__ uint32_t Ss[KB_LDS_LISTS + 1];
    __shared__ uint32_t So[KB_LDS_LISTS];           // the lists' arena offsets for this class (np <= KB_LDS_LISTS)
    const uint32_t tid = threadIdx.x, lane = lane_id(), wv = tid >> 6;
    const uint64_t n = b.n_txns;
    const uint64_t nbig = b.ctl->n_big;
    if (tid == 0) { L.so = 0; L.have = 0; }
    __syncthreads();
    for (uint64_t bi = blockIdx.x; bi < nbig; bi += gridDim.x)
    {
        const uint64_t t = b.big[bi];
        const uint64_t p0 = b.q_key_off[t];
        const uint32_t np = (uint32_t)(b.q_key_off[t + 1] - p0);
        // per-probe metadata and list starts: one wave when the request has at most 64 probes (the usual <= 8 keys:
        // register scans, one barrier, no global round trip), else block-wide reduces and scans
        const bool few = np <= 64;
        if (few)
        {
            if (wv == 0)
            {
                const bool on = lane < np;
                const uint64_t pi = p0 + lane;
                const uint32_t c0 = on ? b.p_c0[pi] : 0u, c1 = on ? b.p_c1[pi] : 0u, rc = on ? b.p_rcnt[pi] : 0u;
                const uint64_t rbv = on ? b.p_rb[pi] : NO_RB;
                const uint32_t of = on ? b.p_off[pi] : 0u, rof = on ? b.p_roff[pi] : 0u;
                const uint32_t rf = rbv != NO_RB ? 1u : 0u;
                const uint32_t i0 = wave_incl_scan(c0), i1 = wave_incl_scan(c1), iR = wave_incl_scan(rc + rf);
                const uint32_t t0 = __shfl(i0, 63, 64), t1 = __shfl(i1, 63, 64), tR = __shfl(iR, 63, 64);
                const uint32_t cp = max(max(t0, t1), tR);
                const uint64_t by = k2_scratch_bytes(np, cp);
                if (lane == 0)
                {
                    L.red[0] = t0;
                    L.red[1] = t1;
                    L.red[2] = tR;
                    if (by > L.have)
                    {
                        const unsigned long long grow = by + by / 2;
                        L.so = atomicAdd(&b.ctl->scr_top, grow);
                        L.have = L.so + grow > b.ctl->scr_cap ? 0ull : grow;
                        if (!L.have) atomicOr(&b.ctl->overflow, 4u);
                    }
                }
                wave_lds_sync();
                if (L.have >= by)
                {
                    K2Mem mm;
                    k2_carve(mm, b.scratch + L.so, np, cp);
                    if (on)
                    {
                        mm.off[lane] = of; mm.c0[lane] = c0; mm.c1[lane] = c1;
                        mm.roff[lane] = rof; mm.rcnt[lane] = rc; mm.rb[lane] = rbv;
                        mm.st0[lane] = i0 - c0;
                        mm.st1[lane] = i1 - c1;
                        mm.stR[2 * lane] = iR - rc - rf;
                        mm.stR[2 * lane + 1] = iR - rf;
                    }
                    if (lane == 0)
                    {
                        mm.st0[np] = t0;
                        mm.st1[np] = t1;
                        mm.stR[2 * np] = tR;
                    }
                }
            }
            __syncthreads();
        }
        else
        {
            if (tid < 3) L.red[tid] = 0;
            __syncthreads();
            uint32_t a0 = 0, a1 = 0, aR = 0;
            for (uint32_t i = tid; i < np; i += KB_THREADS)
            {
                a0 += b.p_c0[p0 + i];
                a1 += b.p_c1[p0 + i];
                aR += b.p_rcnt[p0 + i] + (b.p_rb[p0 + i] != NO_RB ? 1u : 0u);
            }
            a0 = wave_sum(a0);
            a1 = wave_sum(a1);
            aR = wave_sum(aR);
            if (lane == 0)
            {
                if (a0) atomicAdd(&L.red[0], a0);
                if (a1) atomicAdd(&L.red[1], a1);
                if (aR) atomicAdd(&L.red[2], aR);
            }
            __syncthreads();
            const uint32_t cp = max(max(L.red[0], L.red[1]), L.red[2]);
            const uint64_t by = k2_scratch_bytes(np, cp);
            // this workgroup's scratch, reused across its requests (grown when a request needs more)
            if (tid == 0 && by > L.have)
            {
                const unsigned long long grow = by + by / 2;
                L.so = atomicAdd(&b.ctl->scr_top, grow);
                L.have = L.so + grow > b.ctl->scr_cap ? 0ull : grow;
                if (!L.have) atomicOr(&b.ctl->overflow, 4u);
            }
            __syncthreads();
        }
        const uint32_t tot0 = L.red[0], tot1 = L.red[1], totR = L.red[2];
        const uint32_t capn = max(max(tot0, tot1), totR);
        const uint64_t bytes = k2_scratch_bytes(np, capn);
        if (L.have < bytes)
        {
            if (tid < 9) b.sz[tid * n + t] = 0;
            __syncthreads();
            continue;
        }
        K2Mem mem;
        k2_carve(mem, b.scratch + L.so, np, capn);
        if (!few)
        {
            for (uint32_t i = tid; i < np; i += KB_THREADS)
            {
                mem.off[i] = b.p_off[p0 + i]; mem.c0[i] = b.p_c0[p0 + i]; mem.c1[i] = b.p_c1[p0 + i];
                mem.roff[i] = b.p_roff[p0 + i]; mem.rcnt[i] = b.p_rcnt[p0 + i]; mem.rb[i] = b.p_rb[p0 + i];
            }
            __syncthreads();
            block_scan_into(L, np, [&](uint32_t i) { return mem.c0[i]; }, mem.st0);
            block_scan_into(L, np, [&](uint32_t i) { return mem.c1[i]; }, mem.st1);
            block_scan_into(L, 2 * np, [&](uint32_t i) {
                return (i & 1) ? (mem.rb[i >> 1] != NO_RB ? 1u : 0u) : mem.rcnt[i >> 1];
            }, mem.stR);
        }

        // ---- keyDeps (class 0) and directKeyDeps (class 1)
        for (int c = 0; c < 2; ++c)
        {
            const int m = c == 0 ? 0 : 2;
            const uint32_t tot = c == 0 ? tot0 : tot1;
            const uint32_t* st = c == 0 ? mem.st0 : mem.st1;
            if (tot == 0)
            {
                if (tid == 0) { b.sz[(3 * m) * n + t] = 0; b.sz[(3 * m + 1) * n + t] = 0; b.sz[(3 * m + 2) * n + t] = 0; }
                continue;
            }
            const bool lds = tot <= min(KB_LDS_CAP, b.kb_sort) && np <= KB_LDS_LISTS;
            // few lists (the usual <= 8 keys): their starts and arena offsets in LDS, so the gather is one global
            // load per element instead of a search through the scratch starts and two scratch reads
            const bool lst = np <= KB_LDS_LISTS;
            if (lst)
            {
                for (uint32_t i = tid; i <= np; i += KB_THREADS) Ss[i] = st[i];
                for (uint32_t i = tid; i < np; i += KB_THREADS) So[i] = mem.off[i] + (c == 0 ? 0u : mem.c0[i]);
                __syncthreads();
            }
            // (the merge tree in global scratch: the u32 values in V's and UP's room, 2 cap words each)
            const bool tree = b.kb_merge;
            uint32_t* gX = reinterpret_cast<uint32_t*>(mem.V);
            for (uint32_t e = tid; e < tot; e += KB_THREADS)
            {
                uint32_t v;
                if (lst)
                {
                    const uint32_t a = list_of(Ss, np, e);
                    v = b.arena[(uint64_t)So[a] + (e - Ss[a])];
                }
                else
                {
                    const uint32_t a = list_of(st, np, e);
                    v = b.arena[(uint64_t)mem.off[a] + (c == 0 ? 0u : mem.c0[a]) + (e - st[a])];
                }
                if (lds) Vs[e] = v;
                else if (tree) gX[e] = v;
                else mem.V[e] = v;
            }
            __syncthreads();
            auto get = [&](uint32_t e) -> uint64_t { return mem.V[e]; };
            auto getl = [&](uint32_t e) -> uint64_t { return Vs[e]; };
            uint32_t *Xs = Vs, *Xp = Ps;
            const uint32_t U = tree  ? (lds ? block_merge_tree(L, Vs, Ps, Ss, np, tot, &Xs, &Xp)
                                            : block_merge_tree(L, gX, reinterpret_cast<uint32_t*>(mem.UP), st, np, tot, &Xs, &Xp))
                               : lds ? block_rank_merge_kept(L, getl, Ss, np, tot, Ps)
                                     : block_rank_merge_kept(L, get, st, np, tot, mem.P);
            if (wv == 0)
            {
                uint32_t nk = 0;
                for (uint32_t i0 = 0; i0 < np; i0 += 64)
                {
                    const uint32_t i = i0 + lane;
                    nk += __popcll(ballot(i < np && st[i + 1] > st[i]));
                }
                if (lane == 0) L.nk = nk;
            }
            __syncthreads();
            const uint32_t nk = L.nk;
            const uint64_t rb = region_bytes(nk, U, tot);
            uint64_t ro;
            const bool fits = kb_region(L, b, rb, &ro);
            if (tid == 0)
            {
                b.sz[(3 * m) * n + t] = fits ? nk : 0;
                b.sz[(3 * m + 1) * n + t] = fits ? U : 0;
                b.sz[(3 * m + 2) * n + t] = fits ? nk + tot : 0;
                b.t_reg[(uint64_t)m * n + t] = ro;
            }
            if (fits)
            {
                int64_t* okeys = reinterpret_cast<int64_t*>(b.reg + ro);
                uint32_t* otx = reinterpret_cast<uint32_t*>(okeys + nk);
                int32_t* ok2t = reinterpret_cast<int32_t*>(otx + U);
                if (wv == 0)
                {
                    uint32_t kr = 0;
                    for (uint32_t i0 = 0; i0 < np; i0 += 64)
                    {
                        const uint32_t i = i0 + lane;
                        const bool ne = i < np && st[i + 1] > st[i];
                        const uint64_t mk = ballot(ne);
                        if (ne)
                        {
                            const uint32_t k = kr + mbcnt(mk);
                            okeys[k] = b.q_keys[p0 + i];
                            ok2t[k] = (int32_t)(nk + st[i + 1]);
                        }
                        kr += __popcll(mk);
                    }
                }
                if (tree)
                {
                    // the unique values in order, then every element's unique rank: its value (gathered again, in list
                    // order) found in the sorted run, the prefix there
                    for (uint32_t i = tid; i < tot; i += KB_THREADS)
                        if (i == 0 || Xs[i] != Xs[i - 1]) otx[Xp[i]] = dict_index(Xs[i]);
                    for (uint32_t e = tid; e < tot; e += KB_THREADS)
                    {
                        uint32_t x;
                        if (lst)
                        {
                            const uint32_t a = list_of(Ss, np, e);
                            x = b.arena[(uint64_t)So[a] + (e - Ss[a])];
                        }
                        else
                        {
                            const uint32_t a = list_of(st, np, e);
                            x = b.arena[(uint64_t)mem.off[a] + (c == 0 ? 0u : mem.c0[a]) + (e - st[a])];
                        }
                        uint32_t lo = 0, hi = tot;
                        while (lo < hi)
                        {
                            const uint32_t mid = (lo + hi) >> 1;
                            if (Xs[mid] < x) lo = mid + 1;
                            else hi = mid;
                        }
                        ok2t[nk + e] = (int32_t)Xp[lo];
                    }
                }
                else if (lds)
                    for (uint32_t e = tid; e < tot; e += KB_THREADS)
                    {
                        const uint64_t x = Vs[e];
                        const uint32_t ur = rank_merge_urank(getl, Ss, np, Ps, x);
                        if (Ps[e + 1] - Ps[e]) otx[ur] = dict_index((uint32_t)x);
                        ok2t[nk + e] = (int32_t)ur;
                    }
                else
                    for (uint32_t e = tid; e < tot; e += KB_THREADS)
                    {
                        const uint64_t x = mem.V[e];
                        const uint32_t ur = rank_merge_urank(get, st, np, mem.P, x);
                        if (mem.P[e + 1] - mem.P[e]) otx[ur] = dict_index((uint32_t)x);
                        ok2t[nk + e] = (int32_t)ur;
                    }
            }
            __syncthreads();
        }

        // ---- rangeDeps: lists = per probe [range-command pairs], [redundant pair]
        const uint32_t nl = 2 * np;
        if (totR == 0)
        {
            if (tid == 0) { b.sz[3 * n + t] = 0; b.sz[4 * n + t] = 0; b.sz[5 * n + t] = 0; }
            __syncthreads();
            continue;
        }
        for (uint32_t e = tid; e < totR; e += KB_THREADS)
        {
            const uint32_t a = list_of(mem.stR, nl, e);
            const uint32_t pi = a >> 1;
            mem.V[e] = (a & 1) ? mem.rb[pi] : b.rarena[(uint64_t)mem.roff[pi] + (e - mem.stR[a])];
        }
        __syncthreads();
        auto get = [&](uint32_t e) -> uint64_t { return mem.V[e]; };
        const uint32_t UPn = block_rank_merge_kept(L, get, mem.stR, nl, totR, mem.P);
        for (uint32_t e = tid; e < totR; e += KB_THREADS)
            if (mem.P[e + 1] - mem.P[e]) mem.UP[rank_merge_urank(get, mem.stR, nl, mem.P, mem.V[e])] = mem.V[e];
        __syncthreads();
        // rid groups (group starts compacted in order by a block scan of the first-of-group flags)
        const uint32_t nR = block_scan_into(L, UPn, [&](uint32_t i) {
            return (i == 0 || (mem.UP[i] >> 32) != (mem.UP[i - 1] >> 32)) ? 1u : 0u;
        }, mem.P2);
        for (uint32_t i = tid; i < UPn; i += KB_THREADS)
            if (i == 0 || (mem.UP[i] >> 32) != (mem.UP[i - 1] >> 32)) mem.gst[mem.P2[i]] = i;
        if (tid == 0) mem.gst[nR] = UPn;
        __syncthreads();
        auto getr = [&](uint32_t e) -> uint64_t { return mem.UP[e] & 0xFFFFFFFFull; };
        const uint32_t UR = block_rank_merge_kept(L, getr, mem.gst, nR, UPn, mem.P2);
        const uint64_t rbytes = region_bytes(nR, UR, UPn);
        uint64_t ro;
        const bool fits = kb_region(L, b, rbytes, &ro);
        if (tid == 0)
        {
            b.sz[3 * n + t] = fits ? nR : 0;
            b.sz[4 * n + t] = fits ? UR : 0;
            b.sz[5 * n + t] = fits ? nR + UPn : 0;
            b.t_reg[(uint64_t)1 * n + t] = ro;
        }
        if (fits)
        {
            int64_t* okeys = reinterpret_cast<int64_t*>(b.reg + ro);
            uint32_t* otx = reinterpret_cast<uint32_t*>(okeys + nR);
            int32_t* ok2t = reinterpret_cast<int32_t*>(otx + UR);
            for (uint32_t g = tid; g < nR; g += KB_THREADS)
            {
                okeys[g] = (int64_t)(mem.UP[mem.gst[g]] >> 32);
                ok2t[g] = (int32_t)(nR + mem.gst[g + 1]);
            }
            for (uint32_t e = tid; e < UPn; e += KB_THREADS)
            {
                const uint64_t x = getr(e);
                const uint32_t ur = rank_merge_urank(getr, mem.gst, nR, mem.P2, x);
                if (mem.P2[e + 1] - mem.P2[e]) otx[ur] = dict_index((uint32_t)x);
                ok2t[nR + e] = (int32_t)ur;
            }
        }
        __syncthreads();
    }
}

hipError_t run_build(const DevSnapshot& s, const BatchBufs& b, hipStream_t st)
{
    if (!b.n_txns) return hipSuccess;
    hipError_t e = hipMemsetAsync(&b.ctl->n_big, 0, sizeof(unsigned long long), st);
    if (e != hipSuccess) return e;
    const unsigned grid = (unsigned)std::min<uint64_t>(b.n_txns, (uint64_t)device_cu_count() * 16);
    k_build<<<grid, 64, k2_lds_bytes(), st>>>(s, b);
    // heavy requests: the count stays on the device; idle workgroups exit at once
    k_build_big<<<(unsigned)std::min<uint64_t>(b.n_txns, (uint64_t)device_cu_count() * 2), KB_THREADS, 0, st>>>(s, b);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// pack: per-request regions -> contiguous per-map arrays at the scanned offsets
// ---------------------------------------------------------------------------------------
// Pack: one wave per 64 consecutive requests. For each (map, array) the wave's output is one
// contiguous run [off[t0], off[t0 + 64]); lane x of a 64-word chunk copies word x from the region
// of the request whose output range holds it. Writes are fully coalesced; reads are contiguous
// within each request's region. The owning request of every word of a window of 64 x PACK_UNROLL
// words comes from the run starts inside the window: each non-empty request marks its start in a
// per-chunk 64-bit LDS mask and its lane in an owner byte at that position; word x's owner is the
// owner byte at the highest marked position <= x, or the previous chunk's last owner (one LDS
// read and a few bit operations per word instead of a 7-step search of the starts).
constexpr uint32_t PACK_WAVES = 4;
#ifndef PACK_UNROLL_N
#define PACK_UNROLL_N 16
#endif
constexpr uint32_t PACK_UNROLL = PACK_UNROLL_N;

struct PackScratch
{
    uint64_t msk[PACK_UNROLL];
    uint8_t own[64 * PACK_UNROLL];
};

template <typename T>
__device__ __forceinline__ void pack_run(const uint8_t* __restrict__ reg, const uint32_t* st, const uint64_t* src,
                                         uint64_t total, T* __restrict__ out, PackScratch* ps)
{
    const uint32_t lane = lane_id();
    const uint32_t s0 = st[lane], s1 = st[lane + 1];
    const bool ne = s1 > s0;
    const uint64_t upto = lane == 63 ? ~0ull : (2ull << lane) - 1ull;     // positions <= lane
    uint32_t carry = 0;          // owner of the word before the chunk (word 0's run starts at 0)
    for (uint64_t xb = 0; xb < total; xb += 64 * PACK_UNROLL)
    {
        if (lane < PACK_UNROLL) ps->msk[lane] = 0;
        wave_lds_sync();
        if (ne && s0 >= xb && s0 < xb + 64 * PACK_UNROLL)
        {
            const uint32_t q = (uint32_t)(s0 - xb);
            atomicOr(reinterpret_cast<unsigned long long*>(&ps->msk[q >> 6]), 1ull << (q & 63));
            ps->own[q] = (uint8_t)lane;
        }
        wave_lds_sync();
        const T* p[PACK_UNROLL];
        bool ok[PACK_UNROLL];
#pragma unroll
        for (uint32_t u = 0; u < PACK_UNROLL; ++u)
        {
            const uint64_t x = xb + u * 64 + lane;
            ok[u] = x < total;
            const uint64_t m = ps->msk[u] & upto;
            const uint32_t r = m ? (uint32_t)ps->own[u * 64 + 63 - __clzll((long long)m)] : carry;
            carry = (uint32_t)__builtin_amdgcn_readlane((int)r, 63);
            p[u] = ok[u] ? reinterpret_cast<const T*>(reg + src[r]) + ((uint32_t)x - st[r]) : reinterpret_cast<const T*>(reg);
        }
        T v[PACK_UNROLL];
#pragma unroll
        for (uint32_t u = 0; u < PACK_UNROLL; ++u) v[u] = *p[u];
#pragma unroll
        for (uint32_t u = 0; u < PACK_UNROLL; ++u)
            if (ok[u]) out[xb + u * 64 + lane] = v[u];
        wave_lds_sync();
    }
}

__global__ __launch_bounds__(64 * PACK_WAVES) void k_pack(BatchBufs b)
{
    __shared__ uint32_t s_start[PACK_WAVES][65];
    __shared__ uint64_t s_src[PACK_WAVES][64];
    __shared__ PackScratch s_ps[PACK_WAVES];
    const uint32_t w = threadIdx.x >> 6, lane = lane_id();
    const uint64_t n = b.n_txns;
    const uint64_t t0 = ((uint64_t)blockIdx.x * PACK_WAVES + w) * 64;
    if (t0 >= n) return;
    const uint64_t t = t0 + lane, te = t0 + 64 < n ? t0 + 64 : n;
    const bool on = t < n;
    uint32_t* st = s_start[w];
    uint64_t* src = s_src[w];
#pragma unroll 1
    for (int m = 0; m < 3; ++m)
    {
        const uint32_t nk = on ? b.sz[(3 * m) * n + t] : 0u, U = on ? b.sz[(3 * m + 1) * n + t] : 0u;
        const uint64_t rb = on ? b.t_reg[(uint64_t)m * n + t] : 0;
#pragma unroll
        for (int a = 0; a < 3; ++a)
        {
            const uint64_t* off = b.off + (uint64_t)(3 * m + a) * (n + 1);
            const uint64_t o0 = off[t0], total = off[te] - o0;
            if (total == 0) continue;
            wave_lds_sync();
            st[lane] = on ? (uint32_t)(off[t] - o0) : (uint32_t)total;
            if (lane == 0) st[64] = (uint32_t)total;
            src[lane] = rb + (a == 0 ? 0 : (a == 1 ? 8ull * nk : 8ull * nk + 4ull * U));
            wave_lds_sync();
            if (a == 0) pack_run<int64_t>(b.reg, st, src, total, b.o_keys[m] + o0, &s_ps[w]);
            else if (a == 1) pack_run<uint32_t>(b.reg, st, src, total, b.o_txns[m] + o0, &s_ps[w]);
            else pack_run<int32_t>(b.reg, st, src, total, b.o_k2t[m] + o0, &s_ps[w]);
        }
    }
}

hipError_t run_pack(const BatchBufs& b, hipStream_t st)
{
    if (!b.n_txns) return hipSuccess;
    const uint64_t waves = (b.n_txns + 63) / 64;
    k_pack<<<(unsigned)((waves + PACK_WAVES - 1) / PACK_WAVES), 64 * PACK_WAVES, 0, st>>>(b);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// scan + pack without a host round trip: reduce -> scan of tile sums -> pack
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(LB_TILE) void k_tile_sums(BatchBufs b)
{
    constexpr uint32_t NW = LB_TILE / 64;
    __shared__ uint64_t s_w[NW][9];
    const BatchCtl* cc = b.ctl;
    if (cc->n_deferred || cc->error || (cc->overflow & 15u)) return;
    const uint32_t tid = threadIdx.x, w = tid >> 6, lane = lane_id();
    const uint64_t n = b.n_txns, t = (uint64_t)blockIdx.x * LB_TILE + tid;
    uint32_t v[9];
#pragma unroll
    for (int a = 0; a < 9; ++a) v[a] = t < n ? b.sz[(uint64_t)a * n + t] : 0u;     // all in flight together
#pragma unroll
    for (int a = 0; a < 9; ++a)
    {
        const uint64_t x = wave_incl_scan64(v[a]);
        if (lane == 63) s_w[w][a] = x;
    }
    __syncthreads();
    if (tid < 9)
    {
        uint64_t acc = 0;
#pragma unroll
        for (uint32_t ww = 0; ww < NW; ++ww) acc += s_w[ww][tid];
        b.lb_agg[(uint64_t)tid * gridDim.x + blockIdx.x] = acc;      // [9][tiles]
    }
}

// one block of 1024 threads per array a: lb_inc[a][tile] = exclusive prefix of lb_agg[a] over the
// tiles (4 consecutive tiles per thread, chunks of 4096 tiles with a carry), the total into the
// control block and off[a][n].
__global__ __launch_bounds__(1024) void k_tile_scan(BatchBufs b, uint64_t tiles)
{
    __shared__ uint64_t s_w[16];
    const BatchCtl* cc = b.ctl;
    if (cc->n_deferred || cc->error || (cc->overflow & 15u)) return;
    const uint32_t tid = threadIdx.x, w = tid >> 6, lane = lane_id();
    const int a = blockIdx.x;
    const uint64_t* __restrict__ agg = b.lb_agg + (uint64_t)a * tiles;
    uint64_t* __restrict__ inc = b.lb_inc + (uint64_t)a * tiles;
    uint64_t carry = 0;
    for (uint64_t c0 = 0; c0 < tiles; c0 += 4096)
    {
        const uint64_t i0 = c0 + 4ull * tid;
        uint64_t y[4], sum = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k)
        {
            y[k] = i0 + k < tiles ? agg[i0 + k] : 0;
            sum += y[k];
        }
        uint64_t x = sum;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1)
        {
            const uint64_t z = __shfl_up(x, d, 64);
            if ((int)lane >= d) x += z;
        }
        if (lane == 63) s_w[w] = x;
        __syncthreads();
        uint64_t wpre = 0, tot = 0;
#pragma unroll
        for (uint32_t ww = 0; ww < 16; ++ww)
        {
            const uint64_t z = s_w[ww];
            if (ww < w) wpre += z;
            tot += z;
        }
        uint64_t e = carry + wpre + x - sum;
#pragma unroll
        for (int k = 0; k < 4; ++k)
        {
            if (i0 + k < tiles) inc[i0 + k] = e;
            e += y[k];
        }
        carry += tot;
        __syncthreads();
    }
    if (tid == 0)
    {
        b.ctl->tot[a] = carry;
        b.off[(uint64_t)a * (b.n_txns + 1) + b.n_txns] = carry;
    }
}

__global__ __launch_bounds__(LB_TILE) void k_pack_tiles(BatchBufs b, int copy)
{
    constexpr uint32_t NW = LB_TILE / 64;
    __shared__ uint64_t s_ex[9][LB_TILE + 1];    // offsets of the tile's requests (+ the tile end)
    __shared__ uint64_t s_wsum[NW][9], s_wo[NW][9];
    __shared__ uint32_t s_start[NW][65];
    __shared__ uint64_t s_src[NW][64];
    __shared__ PackScratch s_ps[NW];
    const BatchCtl* cc = b.ctl;
    if (cc->n_deferred || cc->error || (cc->overflow & 15u)) return;
    const uint32_t tid = threadIdx.x, w = tid >> 6, lane = lane_id();
    const uint32_t tile = blockIdx.x;
    const uint64_t n = b.n_txns;
    const uint64_t t = (uint64_t)tile * LB_TILE + tid;
    const bool on = t < n;
    uint32_t vv[9];
#pragma unroll
    for (int a = 0; a < 9; ++a) vv[a] = on ? b.sz[(uint64_t)a * n + t] : 0u;     // all in flight together
#pragma unroll
    for (int a = 0; a < 9; ++a)
    {
        const uint32_t v = vv[a];
        const uint64_t x = wave_incl_scan64(v);
        s_ex[a][tid] = x - v;
        if (lane == 63) s_wsum[w][a] = x;
    }
    __syncthreads();
    if (tid < 9)
    {
        uint64_t acc = b.lb_inc[(uint64_t)tid * gridDim.x + tile];
#pragma unroll
        for (uint32_t ww = 0; ww < NW; ++ww)
        {
            s_wo[ww][tid] = acc;
            acc += s_wsum[ww][tid];
        }
        s_ex[tid][LB_TILE] = acc;
    }
    __syncthreads();
#pragma unroll 1
    for (int a = 0; a < 9; ++a)
    {
        const uint64_t e = s_wo[w][a] + s_ex[a][tid];
        s_ex[a][tid] = e;
        if (on) b.off[(uint64_t)a * (n + 1) + t] = e;
    }
    if (!copy) return;
    __syncthreads();
    // pack: wave w copies requests [64 w, 64 w + 64) of the tile; per (map, array) one contiguous run
    uint32_t* st = s_start[w];
    uint64_t* src = s_src[w];
    const uint64_t t0 = (uint64_t)tile * LB_TILE + 64 * w;
    if (t0 >= n) return;
    const uint32_t i0 = 64 * w, i1 = 64 * w + 64;     // s_ex[a][i1]: the next wave's start or the tile end
#pragma unroll 1
    for (int m = 0; m < 3; ++m)
    {
        if (s_ex[3 * m][i1] == s_ex[3 * m][i0] && s_ex[3 * m + 1][i1] == s_ex[3 * m + 1][i0] &&
            s_ex[3 * m + 2][i1] == s_ex[3 * m + 2][i0])
            continue;                                   // the map is empty for the wave's requests
        const uint32_t nk = (uint32_t)(s_ex[3 * m][tid + 1] - s_ex[3 * m][tid]);
        const uint32_t U = (uint32_t)(s_ex[3 * m + 1][tid + 1] - s_ex[3 * m + 1][tid]);
        const uint64_t rb = on ? b.t_reg[(uint64_t)m * n + t] : 0;
#pragma unroll 1
        for (int k = 0; k < 3; ++k)
        {
            const int a = 3 * m + k;
            const uint64_t o0 = s_ex[a][i0];
            const uint64_t total = s_ex[a][i1] - o0;
            if (total == 0) continue;
            if (o0 + total > b.o_cap[a])
            {
                if (lane == 0) atomicOr(&b.ctl->overflow, OVF_PACK);
                continue;
            }
            wave_lds_sync();
            st[lane] = on ? (uint32_t)(s_ex[a][tid] - o0) : (uint32_t)total;
            if (lane == 0) st[64] = (uint32_t)total;
            src[lane] = rb + (k == 0 ? 0 : (k == 1 ? 8ull * nk : 8ull * nk + 4ull * U));
            wave_lds_sync();
            if (k == 0) pack_run<int64_t>(b.reg, st, src, total, b.o_keys[m] + o0, &s_ps[w]);
            else if (k == 1) pack_run<uint32_t>(b.reg, st, src, total, b.o_txns[m] + o0, &s_ps[w]);
            else pack_run<int32_t>(b.reg, st, src, total, b.o_k2t[m] + o0, &s_ps[w]);
        }
    }
}

// ---------------------------------------------------------------------------------------
// The copy of a batch of few, heavy requests (BatchBufs.pack_even): k_pack_tiles's one wave per 64
// requests leaves most of the chip idle when a batch has a few thousand requests of thousands of pairs
// each (the steady state: 16384 requests, 56M pairs, 256 waves). Here the packed output of array a
// (blockIdx.y) is cut into chunks of PE_CHUNK elements, a workgroup per chunk (grid-stride): the
// chunk's requests (found by two binary searches of off[a]) in windows of PE_WIN held in LDS, each
// element's request found in the window by a binary search from the thread's previous one.
// ---------------------------------------------------------------------------------------
constexpr uint32_t PE_THREADS = 256, PE_CHUNK = 8192, PE_WIN = 1024, PE_UNROLL = 4;

__device__ __forceinline__ uint64_t last_le(const uint64_t* __restrict__ off, uint64_t n1, uint64_t p)
{
    // the last r in [0, n1) with off[r] <= p (off ascending, off[0] <= p)
    uint64_t lo = 0, hi = n1;
    while (hi - lo > 1)
    {
        const uint64_t mid = (lo + hi) >> 1;
        if (off[mid] <= p) lo = mid;
        else hi = mid;
    }
    return lo;
}

template <class T>
__device__ __forceinline__ void pack_even_array(const BatchBufs& b, int a, T* __restrict__ out, uint64_t* s_off,
                                                uint64_t* s_src, uint64_t* s_r)
{
    const uint64_t n = b.n_txns;
    const uint32_t tid = threadIdx.x;
    const int m = a / 3, k = a % 3;
    const uint64_t* __restrict__ off = b.off + (uint64_t)a * (n + 1);
    const uint64_t total = off[n];
    if (total == 0) return;
    if (total > b.o_cap[a])
    {
        if (blockIdx.x == 0 && tid == 0) atomicOr(&b.ctl->overflow, OVF_PACK);
        return;
    }
    for (uint64_t p0 = (uint64_t)blockIdx.x * PE_CHUNK; p0 < total; p0 += (uint64_t)gridDim.x * PE_CHUNK)
    {
        const uint64_t p1 = p0 + PE_CHUNK < total ? p0 + PE_CHUNK : total;
        if (tid == 0) s_r[0] = last_le(off, n + 1, p0);
        if (tid == 64) s_r[1] = last_le(off, n + 1, p1 - 1);
        __syncthreads();
        const uint64_t r0 = s_r[0], r1 = s_r[1];
        for (uint64_t ra = r0; ra <= r1; ra += PE_WIN)
        {
            const uint32_t wn = (uint32_t)((r1 - ra + 1) < PE_WIN ? (r1 - ra + 1) : PE_WIN);
            __syncthreads();                        // the previous window (and s_r) read by every thread
            for (uint32_t i = tid; i <= wn; i += PE_THREADS) s_off[i] = off[ra + i];
            for (uint32_t i = tid; i < wn; i += PE_THREADS)
            {
                const uint64_t r = ra + i;
                uint64_t src = b.t_reg[(uint64_t)m * n + r];
                if (k) src += 8ull * b.sz[(uint64_t)(3 * m) * n + r];
                if (k == 2) src += 4ull * b.sz[(uint64_t)(3 * m + 1) * n + r];
                s_src[i] = src;
            }
            __syncthreads();
            const uint64_t q0 = p0 > s_off[0] ? p0 : s_off[0], q1 = p1 < s_off[wn] ? p1 : s_off[wn];
            uint32_t lo = 0;
            for (uint64_t base = q0 + tid; base < q1; base += PE_UNROLL * PE_THREADS)
            {
                T v[PE_UNROLL];
#pragma unroll
                for (uint32_t u = 0; u < PE_UNROLL; ++u)
                {
                    const uint64_t p = base + (uint64_t)u * PE_THREADS;
                    if (p < q1)
                    {
                        uint32_t hi = wn;
                        while (hi - lo > 1)
                        {
                            const uint32_t mid = (lo + hi) >> 1;
                            if (s_off[mid] <= p) lo = mid;
                            else hi = mid;
                        }
                        v[u] = reinterpret_cast<const T*>(b.reg + s_src[lo])[p - s_off[lo]];
                    }
                }
#pragma unroll
                for (uint32_t u = 0; u < PE_UNROLL; ++u)
                {
                    const uint64_t p = base + (uint64_t)u * PE_THREADS;
                    if (p < q1) out[p] = v[u];
                }
            }
        }
        __syncthreads();                            // s_r rewritten by the next chunk
    }
}

__global__ __launch_bounds__(PE_THREADS) void k_pack_even(BatchBufs b)
{
    __shared__ uint64_t s_off[PE_WIN + 1];
    __shared__ uint64_t s_src[PE_WIN];
    __shared__ uint64_t s_r[2];
    const BatchCtl* cc = b.ctl;
    if (cc->n_deferred || cc->error || (cc->overflow & 15u)) return;
    const int a = blockIdx.y, m = a / 3;
    if (a % 3 == 0) pack_even_array<int64_t>(b, a, b.o_keys[m], s_off, s_src, s_r);
    else if (a % 3 == 1) pack_even_array<uint32_t>(b, a, b.o_txns[m], s_off, s_src, s_r);
    else pack_even_array<int32_t>(b, a, b.o_k2t[m], s_off, s_src, s_r);
}

hipError_t run_pack_lb(const BatchBufs& b, bool copy, hipStream_t st)
{
    if (!b.n_txns) return hipMemsetAsync(b.off, 0, sizeof(uint64_t) * 9, st);     // off[a][0] = 0
    const uint64_t tiles = lb_tiles(b.n_txns);
    k_tile_sums<<<(unsigned)tiles, LB_TILE, 0, st>>>(b);
    k_tile_scan<<<9, 1024, 0, st>>>(b, tiles);
    const bool even = copy && b.pack_even;
    k_pack_tiles<<<(unsigned)tiles, LB_TILE, 0, st>>>(b, copy && !even ? 1 : 0);
    if (even) k_pack_even<<<dim3(512, 9), PE_THREADS, 0, st>>>(b);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// exclusive scans of size arrays -> u64 offsets [n_arrays][n+1], reduce-then-scan: block sums of
// the input, a parallel scan of the block sums (one block per array), then every block scans its
// tile again with its offset (the input is read twice, the offsets written once)
// ---------------------------------------------------------------------------------------
constexpr int SCAN_BLOCK = 1024;

// exclusive scan of v over the block (SCAN_BLOCK threads); *total = the block's sum
__device__ __forceinline__ uint64_t block_excl_scan(uint64_t v, uint64_t* wsum /* [SCAN_BLOCK/64 + 1] */, uint64_t* total)
{
    const uint64_t inc = wave_incl_scan64(v);
    const int l = lane_id();
    const int w = threadIdx.x >> 6;
    if (l == 63) wsum[w] = inc;
    __syncthreads();
    if (threadIdx.x < 64)
    {
        const uint64_t x = threadIdx.x < SCAN_BLOCK / 64 ? wsum[threadIdx.x] : 0;
        uint64_t sacc = x;
#pragma unroll
        for (int d = 1; d < SCAN_BLOCK / 64; d <<= 1)
        {
            const uint64_t tt = __shfl_up(sacc, d, 64);
            if (l >= d) sacc += tt;
        }
        if (threadIdx.x < SCAN_BLOCK / 64) wsum[threadIdx.x] = sacc - x;
        if (threadIdx.x == SCAN_BLOCK / 64 - 1) wsum[SCAN_BLOCK / 64] = sacc;
    }
    __syncthreads();
    const uint64_t r = inc - v + wsum[w];
    *total = wsum[SCAN_BLOCK / 64];
    __syncthreads();            // wsum is reused by the caller's next scan
    return r;
}

// A block scans SCAN_BLOCK * SCAN_ITEMS elements: wave w the 512 at [w * 512, +512) as 8 coalesced chunks of 64
// (chunk-major is memory order, so a chunk's lane prefix plus the earlier chunks' totals is the wave prefix).
// (One element per thread, as before round 6, spent the 4-array scan of a 16M-entry derivation mostly on
// block overhead: 64k blocks of 4 KB each.)
constexpr int SCAN_ITEMS = 8;
constexpr uint64_t SCAN_TILE = (uint64_t)SCAN_BLOCK * SCAN_ITEMS;

__global__ __launch_bounds__(SCAN_BLOCK) void k_scan_reduce(const uint32_t* __restrict__ sz, uint64_t n,
                                                            uint64_t* __restrict__ bsum, uint64_t nb)
{
    __shared__ uint64_t part[SCAN_BLOCK / 64];
    const int a = blockIdx.y;
    const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE + (uint64_t)(threadIdx.x >> 6) * (64 * SCAN_ITEMS) + lane_id();
    const uint32_t* __restrict__ in = sz + (uint64_t)a * n;
    uint32_t v[SCAN_ITEMS];
#pragma unroll
    for (int j = 0; j < SCAN_ITEMS; ++j)
    {
        const uint64_t i = base + 64ull * j;
        v[j] = i < n ? in[i] : 0u;
    }
    uint64_t t = 0;
#pragma unroll
    for (int j = 0; j < SCAN_ITEMS; ++j) t += v[j];
    t = wave_incl_scan64(t);
    if (lane_id() == 63) part[threadIdx.x >> 6] = t;
    __syncthreads();
    if (threadIdx.x == 0)
    {
        uint64_t x = 0;
        for (int w = 0; w < SCAN_BLOCK / 64; ++w) x += part[w];
        bsum[(uint64_t)a * nb + blockIdx.x] = x;
    }
}

__global__ __launch_bounds__(SCAN_BLOCK) void k_scan_sums(uint64_t* bsum, uint64_t nb, uint64_t* __restrict__ off, uint64_t n)
{
    // one block per array: exclusive scan of its block sums in place, total -> off[n]
    __shared__ uint64_t wsum[SCAN_BLOCK / 64 + 1];
    const int a = blockIdx.x;
    uint64_t carry = 0;
    for (uint64_t i0 = 0; i0 < nb; i0 += SCAN_BLOCK)
    {
        const uint64_t i = i0 + threadIdx.x;
        const uint64_t v = i < nb ? bsum[(uint64_t)a * nb + i] : 0;
        uint64_t tot;
        const uint64_t ex = block_excl_scan(v, wsum, &tot);
        if (i < nb) bsum[(uint64_t)a * nb + i] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0) off[(uint64_t)a * (n + 1) + n] = carry;
}

__global__ __launch_bounds__(SCAN_BLOCK) void k_scan_tile(const uint32_t* __restrict__ sz, uint64_t n,
                                                          const uint64_t* __restrict__ bsum, uint64_t nb,
                                                          uint64_t* __restrict__ off)
{
    __shared__ uint64_t wpre[SCAN_BLOCK / 64];
    const int a = blockIdx.y;
    const uint32_t w = threadIdx.x >> 6, lane = lane_id();
    const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE + (uint64_t)w * (64 * SCAN_ITEMS) + lane;
    const uint32_t* __restrict__ in = sz + (uint64_t)a * n;
    uint64_t* __restrict__ out = off + (uint64_t)a * (n + 1);
    uint32_t v[SCAN_ITEMS];
#pragma unroll
    for (int j = 0; j < SCAN_ITEMS; ++j)
    {
        const uint64_t i = base + 64ull * j;
        v[j] = i < n ? in[i] : 0u;
    }
    uint64_t ex[SCAN_ITEMS];
    uint64_t run = 0;
#pragma unroll
    for (int j = 0; j < SCAN_ITEMS; ++j)
    {
        const uint64_t inc = wave_incl_scan64(v[j]);
        ex[j] = run + inc - v[j];
        run += __shfl(inc, 63, 64);
    }
    if (lane == 0) wpre[w] = run;          // the wave's total
    __syncthreads();
    uint64_t pre = bsum[(uint64_t)a * nb + blockIdx.x];
    for (uint32_t ww = 0; ww < w; ++ww) pre += wpre[ww];
#pragma unroll
    for (int j = 0; j < SCAN_ITEMS; ++j)
    {
        const uint64_t i = base + 64ull * j;
        if (i < n) out[i] = pre + ex[j];
    }
}

// small arrays (the radix histograms of the update's sorts, per-request counts of small batches): one block per
// array walks it in tiles with a carry -- one launch instead of three (a step of the steady state runs ~30 scans)
constexpr uint64_t SCAN_SMALL = 8 * SCAN_TILE;

__global__ __launch_bounds__(SCAN_BLOCK) void k_scan_small(const uint32_t* __restrict__ sz, uint64_t n, uint64_t* __restrict__ off)
{
    __shared__ uint64_t wtot[SCAN_BLOCK / 64];
    const int a = blockIdx.x;
    const uint32_t w = threadIdx.x >> 6, lane = lane_id();
    const uint32_t* __restrict__ in = sz + (uint64_t)a * n;
    uint64_t* __restrict__ out = off + (uint64_t)a * (n + 1);
    uint64_t carry = 0;
    for (uint64_t t0 = 0; t0 < n; t0 += SCAN_TILE)
    {
        const uint64_t base = t0 + (uint64_t)w * (64 * SCAN_ITEMS) + lane;
        uint32_t v[SCAN_ITEMS];
#pragma unroll
        for (int j = 0; j < SCAN_ITEMS; ++j)
        {
            const uint64_t i = base + 64ull * j;
            v[j] = i < n ? in[i] : 0u;
        }
        uint64_t ex[SCAN_ITEMS];
        uint64_t run = 0;
#pragma unroll
        for (int j = 0; j < SCAN_ITEMS; ++j)
        {
            const uint64_t inc = wave_incl_scan64(v[j]);
            ex[j] = run + inc - v[j];
            run += __shfl(inc, 63, 64);
        }
        if (lane == 0) wtot[w] = run;
        __syncthreads();
        uint64_t pre = carry, tot = 0;
        for (uint32_t ww = 0; ww < SCAN_BLOCK / 64; ++ww)
        {
            const uint64_t x = wtot[ww];
            if (ww < w) pre += x;
            tot += x;
        }
#pragma unroll
        for (int j = 0; j < SCAN_ITEMS; ++j)
        {
            const uint64_t i = base + 64ull * j;
            if (i < n) out[i] = pre + ex[j];
        }
        carry += tot;
        __syncthreads();                    // wtot rewritten by the next tile
    }
    if (threadIdx.x == 0) out[n] = carry;
}

hipError_t run_scan_arrays(const uint32_t* in, uint64_t* out, uint64_t n, int n_arrays, uint64_t* bsum, hipStream_t st)
{
    if (n && n <= SCAN_SMALL)
    {
        k_scan_small<<<n_arrays, SCAN_BLOCK, 0, st>>>(in, n, out);
        return hipGetLastError();
    }
    // out[a][0..n] = exclusive prefix of in[a][0..n), out[a][n] = total, for a < n_arrays
    // (bsum: n_arrays * ceil(n / SCAN_TILE) entries -- callers size it for ceil(n / 1024), more than enough)
    const uint64_t nb = (n + SCAN_TILE - 1) / SCAN_TILE;
    if (n == 0) return hipMemsetAsync(out, 0, sizeof(uint64_t) * n_arrays, st);    // out[a][0], a < n_arrays
    dim3 g((unsigned)nb, (unsigned)n_arrays);
    k_scan_reduce<<<g, SCAN_BLOCK, 0, st>>>(in, n, bsum, nb);
    k_scan_sums<<<n_arrays, SCAN_BLOCK, 0, st>>>(bsum, nb, out, n);
    k_scan_tile<<<g, SCAN_BLOCK, 0, st>>>(in, n, bsum, nb, out);
    return hipGetLastError();
}

hipError_t run_offsets(const BatchBufs& b, hipStream_t st) { return run_scan_arrays(b.sz, b.off, b.n_txns, 9, b.bsum, st); }

// the 9 totals into the control block, so one copy of it tells the host everything
__global__ void k_collect_totals(const uint64_t* __restrict__ off, uint64_t n, BatchCtl* ctl)
{
    if (threadIdx.x < 9) ctl->tot[threadIdx.x] = off[(uint64_t)threadIdx.x * (n + 1) + n];
}

hipError_t run_collect_totals(const BatchBufs& b, hipStream_t st)
{
    k_collect_totals<<<1, 64, 0, st>>>(b.off, b.n_txns, b.ctl);
    return hipGetLastError();
}

// The lean kernels' KeyLine of every key (common.hpp), from the KeyEntry (newest fields, class
// lists) and the emission lists; thread per key, written to the key's slot (empty slots: meta 0).
__device__ __forceinline__ uint32_t n2_inl_off(uint32_t meta) { return (meta >> KL_INL_SHIFT) & 31u; }

__global__ __launch_bounds__(256) void k_build_klines(DevSnapshot s, const uint32_t* __restrict__ kslot,
                                                      const uint32_t* __restrict__ kcell, KeyLine* __restrict__ out,
                                                      LeanQuads* __restrict__ kquad)
{
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= s.n_keys) return;
    const KeyEntry ke = s.kent[k];
    KeyLine L;
    L.key = s.keys[k];
    const uint32_t cell = kcell ? kcell[k] : NO_CELL;
    L.cell_lo = (cell != NO_CELL && s.cell_off) ? s.cell_off[cell] : 0u;
    L.cell_hi = (cell != NO_CELL && s.cell_off) ? s.cell_off[cell + 1] : 0u;
    L.last_txn = ke.last_txn;
    L.last_wexec = ke.last_wexec;
    L.last_w_txn = ke.last_w_txn;
    for (int c = 0; c < NCLASS; ++c) L.cls[c] = KeyClassSpan{ke.cl[c].cand_hi - ke.cl[c].cand_lo, ke.cl[c].cand_lo};
    L.cwr_tail = ke.cl[0].cwr_tail;
    L.pruned = s.krec[k].pruned;
    const uint32_t n_cwr = ke.cl[0].cwr_hi - ke.cl[0].cwr_tail;
    const uint32_t n2 = L.cls[2].n;
    uint32_t meta = KL_USED | (n_cwr & KL_NCWR_MASK);
    if (n_cwr > KL_NCWR_MASK) meta |= KL_NOLEAN;
    for (uint32_t i = 0; i < KL_INL; ++i) L.inl[i] = 0;
    if (n2 + n_cwr <= KL_INL)
    {
        // nested by class: Writes (class 0), then the Reads of class 1, then the (Exclusive)SyncPoints
        // of class 2; then the cwr tail
        uint32_t i = 0;
        for (uint32_t j = 0; j < L.cls[0].n; ++j) L.inl[i++] = s.cand[L.cls[0].base + j];
        for (uint32_t j = 0; j < L.cls[1].n; ++j)
        {
            const uint32_t x = s.cand[L.cls[1].base + j];
            if ((x >> RANK_BITS) == 0u) L.inl[i++] = x;     // Txn.Kind.Read
        }
        for (uint32_t j = 0; j < L.cls[2].n; ++j)
        {
            const uint32_t x = s.cand[L.cls[2].base + j];
            if (((KINDS_ANY_GLOBALLY_VISIBLE & ~KINDS_RS_OR_WS) >> (x >> RANK_BITS)) & 1u) L.inl[i++] = x;
        }
        for (uint32_t j = 0; j < n_cwr; ++j) L.inl[n2 + j] = s.cwr[L.cwr_tail + j];
        meta |= KL_INLINE | (n2 << KL_INL_SHIFT);
    }
    {
        // the stabbing cell's entries after the inline emissions, when they fit (u64-aligned)
        const uint32_t used = (meta & KL_INLINE) ? n2 + n_cwr : 0u;
        const uint32_t co = (used + 1) & ~1u, nc = L.cell_hi - L.cell_lo;
        if (nc > 0 && co + 2 * nc <= KL_INL)
        {
            uint64_t* in64 = reinterpret_cast<uint64_t*>(L.inl);
            for (uint32_t j = 0; j < nc; ++j) in64[co / 2 + j] = s.cell_ent[L.cell_lo + j];
            meta |= KL_CELLINL | ((co / 2) << KL_CELL_SHIFT);
        }
    }
    L.meta = meta;
    out[kslot[k]] = L;
    // the probe quads (LeanQuads): the newest threshold, per class the two emission runs
    LeanQuads Q;
    const bool inl = (meta & KL_INLINE) != 0;
    const uint32_t thr0 = max(L.last_wexec, L.pruned);
    const uint32_t wbase = kslot[k] * (uint32_t)(sizeof(KeyLine) / 4) + (uint32_t)(offsetof(KeyLine, inl) / 4);
    for (int c = 0; c < NCLASS; ++c)
    {
        const uint32_t n1 = L.cls[c].n, n2 = c == 0 ? (L.last_w_txn != 0 ? 1u : 0u) : n_cwr;
        const bool lean = !(meta & KL_NOLEAN) && n1 <= LQ_NMAX && n2 <= LQ_NMAX;
        const uint32_t b1 = inl ? wbase : L.cls[c].base;
        const uint32_t b2 = c == 0 ? (L.last_w_txn | (1u << RANK_BITS)) : (inl ? wbase + n2_inl_off(meta) : L.cwr_tail);
        Q.q[c] = make_uint4(lean ? thr0 : 0xFFFFFFFFu, lean ? (n1 | (n2 << 8) | (inl ? LQ_INLINE : 0u)) : 0u, b1, b2);
    }
    Q.key = L.key;
    Q.used = 1;
    Q.pad = 0;
    kquad[kslot[k]] = Q;
}

__global__ void k_key_slots(const int64_t* __restrict__ keys, uint64_t nk, const uint32_t* __restrict__ disp, uint64_t nb,
                            uint64_t m, uint32_t* __restrict__ kslot)
{
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < nk) kslot[k] = (uint32_t)kl_index(key_hash2(keys[k]), disp[kl_bucket(key_hash(keys[k]), nb)], m);
}

hipError_t run_key_slots(const int64_t* keys, uint64_t nk, const uint32_t* disp, uint64_t nb, uint64_t m, uint32_t* kslot,
                         hipStream_t st)
{
    if (!nk) return hipSuccess;
    k_key_slots<<<(unsigned)((nk + 255) / 256), 256, 0, st>>>(keys, nk, disp, nb, m, kslot);
    return hipGetLastError();
}

hipError_t run_build_klines(const DevSnapshot& s, const uint32_t* kslot, const uint32_t* kcell, KeyLine* table,
                            uint64_t table_slots, hipStream_t st)
{
    // the LeanQuads sit right after the KeyLines (one allocation: kline_table_bytes)
    LeanQuads* quads = reinterpret_cast<LeanQuads*>(table + table_slots);
    hipError_t e = hipMemsetAsync(table, 0, kline_table_bytes(table_slots), st);
    if (e != hipSuccess || !s.n_keys) return e;
    k_build_klines<<<(unsigned)((s.n_keys + 255) / 256), 256, 0, st>>>(s, kslot, kcell, table, quads);
    return hipGetLastError();
}

// both levels: entries [0, n1) every DICT_SAMP-th id, [base2, base2 + n2) every DICT_SAMP2-th
__global__ void k_snap_dict_sample(DevSnapshot s, uint64_t* hi, uint64_t* lo, int32_t* node, uint64_t n1, uint64_t base2,
                                   uint64_t n2)
{
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t i;
    if (j < n1) i = j * DICT_SAMP;
    else if (j >= base2 && j < base2 + n2) i = (j - base2) * DICT_SAMP2;
    else return;
    hi[j] = s.dict_hi[i];
    lo[j] = s.dict_lo[i];
    node[j] = s.dict_node[i];
}

hipError_t run_dict_sample(const DevSnapshot& s, uint64_t* hi, uint64_t* lo, int32_t* node, hipStream_t st)
{
    const uint64_t n1 = dict_samples(s.n_dict), base2 = dict_samp2_base(n1), n2 = dict_samples2(s.n_dict);
    if (n1) k_snap_dict_sample<<<(unsigned)((base2 + n2 + 255) / 256), 256, 0, st>>>(s, hi, lo, node, n1, base2, n2);
    return hipGetLastError();
}

// The bucket index of the first sample level (common.hpp dict_bucket_of), thread per bucket start: start[b] =
// the first sample whose bucket is >= b (a binary search of the samples); thread 0 also writes the header.
__global__ void k_dict_buckets(DevSnapshot s, uint32_t* B, uint32_t lg)
{
    const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t nb = 1ull << lg;
    if (b > nb) return;
    const uint64_t mh = s.ds_hi[0], ml = s.ds_lo[0];
    // span of the dictionary: its last id less the first sample (= its first id)
    const unsigned __int128 span = ((((unsigned __int128)s.dict_last_hi) << 64) | s.dict_last_lo) -
                                   ((((unsigned __int128)mh) << 64) | ml);
    const uint32_t bl = bitlen128((uint64_t)(span >> 64), (uint64_t)span);
    const uint32_t sh = bl > lg ? bl - lg : 0u;
    if (b == 0)
    {
        B[0] = (uint32_t)mh;
        B[1] = (uint32_t)(mh >> 32);
        B[2] = (uint32_t)ml;
        B[3] = (uint32_t)(ml >> 32);
        B[4] = sh;
        B[5] = lg;
        B[6] = (uint32_t)s.n_samp;
        B[7] = 0;
    }
    uint64_t lo = 0, hi = s.n_samp;
    while (lo < hi)
    {
        const uint64_t mid = (lo + hi) >> 1;
        if (dict_bucket_of(mh, ml, sh, lg, s.ds_hi[mid], s.ds_lo[mid]) < b) lo = mid + 1;
        else hi = mid;
    }
    B[DB_HDR + b] = (uint32_t)lo;
}

hipError_t run_dict_buckets(const DevSnapshot& s, uint32_t* B, uint32_t lg, hipStream_t st)
{
    if (!s.n_samp) return hipSuccess;
    const uint64_t n = (1ull << lg) + 1;
    k_dict_buckets<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(s, B, lg);
    return hipGetLastError();
}

int device_cu_count()
{
    static int cus = 0;
    if (!cus)
    {
        int dev = 0;
        (void)hipGetDevice(&dev);
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, dev) == hipSuccess) cus = prop.multiProcessorCount;
        if (cus <= 0) cus = 256;
    }
    return cus;
}


// ---------------------------------------------------------------------------------------
// Recovery scans: CommandsForKey.mapReduceFull (CommandsForKey.java:809-908) for
// the four BeginRecovery queries (BeginRecovery.java:329-380), one wave per (request, key) probe,
// emitting into the K1 arena in the k_scan layout so that k_build assembles the Deps.
// ---------------------------------------------------------------------------------------
// Txn.Kind.witnessedBy() (Txn.java:247-262) as a kinds mask; 0xFFFF for an AssertionError
__device__ __forceinline__ uint32_t kind_witnessed_by(uint32_t kind)
{
    switch (kind)
    {
        case 2: return 0u;                                            // EphemeralRead: Nothing
        case 0: return (1u << 1) | (1u << 3) | (1u << 4);             // Read: WsOrSyncPoints
        case 1: return KINDS_ANY_GLOBALLY_VISIBLE;                    // Write
        case 3: case 4: return 1u << 4;                               // (Exclusive)SyncPoint: ExclusiveSyncPoints
        default: return 0xFFFFu;
    }
}

__global__ void k_encode_recover(DevSnapshot s, BatchBufs b)
{
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= b.n_txns) return;
    const uint64_t tm = b.q_txn_msb[t], tl = b.q_txn_lsb[t];
    const int32_t tn = b.q_txn_node[t];
    uint32_t kinds = kind_witnessed_by((uint32_t)((tl >> 1) & 7));   // testKind = txnId.kind().witnessedBy()
    if (kinds == 0xFFFFu) { set_error(b.ctl, ERR_INVAL); kinds = 0; }
    b.t_S[t] = encode_rank(s, tm, tl, tn);                            // testTxnId
    b.t_self[t] = 0;
    b.t_kinds[t] = kinds;
    b.t_epoch[t] = 0;
    for (uint64_t p = b.q_key_off[t]; p < b.q_key_off[t + 1]; ++p) b.p_txn[p] = (uint32_t)t;
}

// scan: AD_RECOVER_* = (TestStartedAt, TestDep, TestStatus) of BeginRecovery.java:334,348,365,378:
//   0 STARTED_BEFORE WITHOUT IS_PROPOSED, 1 STARTED_BEFORE WITH IS_STABLE,
//   2 STARTED_AFTER WITHOUT IS_PROPOSED,  3 ANY WITHOUT IS_STABLE
// Every scan wants executeAt > testTxnId (:861-866). The entries are found without walking the
// probed range: a WITHOUT scan of a known testTxnId wants entries whose missing() holds it -- the
// key's inverted missing() index (missing id, entry) lists exactly those; every other scan descends
// the 64-ary max-executeAt tree of its status set over [start, end), so a wave touches only the
// entries executing after testTxnId (plus a root-to-leaf path per 64-entry block it reports).
__global__ __launch_bounds__(256) void k_recover(RecoveryView v, BatchBufs b, uint32_t scan)
{
    __shared__ uint32_t stage[K1_WAVES][K1_CAP];
    __shared__ uint64_t stk[K1_WAVES][2 * MAX_LEVELS];
    const int wv = threadIdx.x >> 6;
    const uint32_t lane = lane_id();
    const uint64_t nw = (uint64_t)gridDim.x * K1_WAVES;
    ChunkAlloc alloc;
    const unsigned long long cap = b.ctl->key_cap;
    const bool with = scan == 1;
    const bool proposed = scan == 0 || scan == 2;
    const int set = proposed ? 0 : 1;

    for (uint64_t p = (uint64_t)blockIdx.x * K1_WAVES + wv; p < b.n_probes; p += nw)
    {
        const uint4 pr = b.p_rec[p];
        const uint32_t ki = pr.x;
        const uint32_t T = pr.y, kinds = pr.w & 0xFF;
        uint64_t start = 0, end = 0;
        bool known = false;
        if (ki != NO_KEY && kinds != 0)
        {
            const uint64_t lo = v.seg[ki], hi = v.seg[ki + 1];
            // insertPos = Arrays.binarySearch(byId, testTxnId) (:821-825)
            const uint64_t pos = wave_lower_bound(lo, hi, [&](uint64_t i) { return v.ent[i].x; },
                                                  [&](uint32_t r) { return r < T; });
            known = pos < hi && v.ent[pos].x == T;
            // unknown + WITH: nothing unless testTxnId < prunedBefore (:832-836; NONE = rank 0)
            const bool skip = !known && with && !(T < v.pruned[ki]);
            if (!skip)
            {
                if (scan == 2) { start = pos; end = hi; }            // STARTED_AFTER
                else if (scan == 3) { start = lo; end = hi; }       // ANY
                else { start = lo; end = pos; }                     // STARTED_BEFORE
            }
        }
        // the loop body of :854-906 for entry i
        auto want_of = [&](uint64_t i, bool& is1, uint32_t& r) -> bool {
            if (i < start || i >= end) return false;
            const uint4 e = v.ent[i];
            r = e.x;
            const uint32_t st = e.z & 0xFF, kd = (e.z >> 8) & 7;
            is1 = ((KINDS_RS_OR_WS >> kd) & 1) == 0;                 // Deps.AbstractBuilder.add routing
            if (!((kinds >> kd) & 1)) return false;                  // testKind.test(txn.kind())
            if (proposed ? !(st == 3u || st == 4u)   // ACCEPTED, COMMITTED
                         : !(st == 5u || st == 6u)) return false;   // STABLE, APPLIED
            // testDep != ANY_DEPS: hasExecuteAtOrDeps (implied by the status sets), executeAt > testTxnId
            if (e.y <= T) return false;
            bool has_as_dep = false;
            if (known)
            {
                const uint32_t nm = e.z >> RV_MISS_SHIFT;
                uint32_t a = e.w, c = e.w + nm;                       // Arrays.binarySearch(missing, testTxnId)
                while (a < c)
                {
                    const uint32_t m = (a + c) >> 1;
                    if (v.miss[m] < T) a = m + 1;
                    else c = m;
                }
                has_as_dep = !(a < e.w + nm && v.miss[a] == T);
            }
            return has_as_dep == with;
        };
        const bool by_missing = !with && known && end > start;
        uint64_t ia = 0, ib = 0;
        if (by_missing)
        {
            // the key's (missing id, entry) pairs naming testTxnId, entries ascending
            const uint64_t a0 = v.inv_off[ki], a1 = v.inv_off[ki + 1];
            ia = wave_lower_bound(a0, a1, [&](uint64_t i) { return v.inv[i].x; }, [&](uint32_t x) { return x < T; });
            ib = wave_lower_bound(ia, a1, [&](uint64_t i) { return v.inv[i].x; }, [&](uint32_t x) { return x <= T; });
        }
        uint32_t cursor = 0, c0 = 0, c1 = 0;
        bool overflow = false;
        // one frame of 64 candidates (entry index per lane, or none): stage the wanted ones
        auto frame_stage = [&](bool cand, uint64_t e) {
            bool is1 = false;
            uint32_t r = 0;
            const bool want = cand && want_of(e, is1, r);
            const uint64_t wm = ballot(want), w1 = ballot(want && is1);
            c0 += __popcll(wm & ~w1);
            c1 += __popcll(w1);
            const uint32_t n = __popcll(wm);
            if (!overflow && cursor + n <= K1_CAP)
            {
                if (want) stage[wv][cursor + mbcnt(wm)] = r | (is1 ? CLASS_DIRECT_BIT : 0u);
                cursor += n;
            }
            else overflow = true;
        };
        auto node_want = [&](int lv, uint64_t node) { return v.lvl[set][lv][node] > T; };
        if (by_missing)
            for (uint64_t base = ia; base < ib; base += 64)
            {
                const uint64_t i = base + lane;
                frame_stage(i < ib, i < ib ? (uint64_t)v.inv[i].y : 0);
            }
        else if (end > start)
            wave_descent(start, end, v.n_levels, node_want, [&](uint64_t base, bool inr) { frame_stage(inr, base + lane); },
                         stk[wv]);
        wave_lds_sync();
        const uint32_t tot = c0 + c1;
        const uint64_t off = tot ? alloc.take(&b.ctl->key_top, cap, &b.ctl->overflow, 1u, tot, K1_CHUNK) : 0;
        const bool fits = off + tot <= cap;
        if (fits && tot)
        {
            uint32_t run0 = 0, run1 = 0;
            auto put = [&](bool want, uint32_t r, bool is1) {
                const uint64_t w0 = ballot(want && !is1), w1 = ballot(want && is1);
                if (want && !is1) b.arena[off + run0 + mbcnt(w0)] = r;       // keyDeps, byId (= rank) order
                if (want && is1) b.arena[off + c0 + run1 + mbcnt(w1)] = r;   // directKeyDeps
                run0 += __popcll(w0);
                run1 += __popcll(w1);
            };
            if (!overflow)
                for (uint32_t i0 = 0; i0 < cursor; i0 += 64)
                {
                    const uint32_t i = i0 + lane;
                    const bool ok = i < cursor;
                    const uint32_t x = ok ? stage[wv][i] : 0u;
                    put(ok, x & ~CLASS_DIRECT_BIT, ok && (x & CLASS_DIRECT_BIT));
                }
            else
            {
                // staging overflowed: replay the walk writing straight to the exact allocation
                auto frame_put = [&](bool cand, uint64_t e) {
                    bool is1 = false;
                    uint32_t r = 0;
                    const bool want = cand && want_of(e, is1, r);
                    put(want, r, is1);
                };
                if (by_missing)
                    for (uint64_t base = ia; base < ib; base += 64)
                    {
                        const uint64_t i = base + lane;
                        frame_put(i < ib, i < ib ? (uint64_t)v.inv[i].y : 0);
                    }
                else
                    wave_descent(start, end, v.n_levels, node_want,
                                 [&](uint64_t base, bool inr) { frame_put(inr, base + lane); }, stk[wv]);
            }
        }
        if (lane == 0)
        {
            b.p_off[p] = fits ? (uint32_t)off : 0u;
            b.p_c0[p] = fits ? c0 : 0u;
            b.p_c1[p] = fits ? c1 : 0u;
        }
    }
}

// The range-command half of the recovery scans (InMemorySafeStore.mapReduceFull ->
// mapReduceRangesInternal, InMemoryCommandStore.java:884-958): one wave per (request, key) probe
// finds the range entries holding the key by the K4 descent (start before the key, max-end tree of
// the all-kinds class) -- or, for a sliced range of a Range-domain request, the entries intersecting
// it -- and keeps those of live commands passing the scan's tests; their (range id,
// txnId) pairs go to the K4 arena, so k_build assembles rangeDeps (one txnId per range, as the
// collect fold does).
__global__ __launch_bounds__(256) void k_range_recover(DevSnapshot s, RecoveryView v, BatchBufs b, uint32_t scan)
{
    __shared__ uint64_t stage[K4_WAVES][K4_CAP];
    __shared__ uint64_t stk[K4_WAVES][2 * MAX_LEVELS];
    const int wv = threadIdx.x >> 6;
    const uint32_t lane = lane_id();
    const uint64_t nw = (uint64_t)gridDim.x * K4_WAVES;
    ChunkAlloc alloc;
    const unsigned long long cap = b.ctl->rng_cap;
    const bool incl = s.start_inclusive != 0;
    const bool with = scan == 1, before = scan == 0 || scan == 1, after = scan == 2;
    const uint32_t need = (scan == 0 || scan == 2) ? 1u : 2u;     // AD_RS_PROPOSED / AD_RS_STABLE
    for (uint64_t p = (uint64_t)blockIdx.x * K4_WAVES + wv; p < b.n_probes; p += nw)
    {
        const int64_t x = b.q_keys[p];
        const uint32_t t = b.p_txn[p];
        const uint32_t T = b.t_S[t], kinds = b.t_kinds[t];
        const NormTid Tn = norm_tid(b.q_txn_msb[t], b.q_txn_lsb[t], b.q_txn_node[t]);
        uint32_t cnt = 0;
        uint64_t off = 0;
        const bool in_slice = (b.p_rec[p].w >> 12) & 1;
        // a Range-domain request (k_range_fill): its sliced range [x, xe) probes the commands whose ranges
        // intersect it (Routables.foldl over the sliced ranges, InMemoryCommandStore.java:951-956) -- the
        // K4 prefix on start < xe, threshold end > x; the CommandsForKey keys inside it probe nothing here
        const uint32_t pk = b.p_kind ? b.p_kind[p] : PK_KEY;
        const bool rq = pk == PK_RANGE;
        const int64_t xe = rq ? b.q_keys_hi[p] : 0;
        if (in_slice && s.n_rent && kinds && pk != PK_RANGE_KEY)
        {
            const uint64_t hi = wave_lower_bound(0, s.n_rent, [&](uint64_t i) { return s.r_start[i]; },
                                                 [&](int64_t val) { return rq ? val < xe : (incl ? val <= x : val < x); });
            auto end_ok = [&](int64_t e) { return rq ? e > x : (incl ? e > x : e >= x); };
            auto node_want = [&](int lv, uint64_t node) { return end_ok(s.rlvl[2][lv][node]); };
            auto want_of = [&](uint64_t i, bool inr, uint64_t& val) -> bool {
                val = 0;
                if (!inr || !end_ok(s.r_end[i])) return false;
                const uint32_t c = v.r_cmd[i];
                if (c == ~0u) return false;                              // not a live rangeCommands entry
                const uint32_t txw = s.r_txw[i], r = txw & RANK_MASK, kd = txw >> RANK_BITS;
                const uint32_t fl = v.rc_flags[c];
                const NormTid ex{v.rc_ex_hi[c], v.rc_ex_lo[c], v.rc_ex_node[c]};
                if (after && !(r > T)) return false;                     // STARTED_AFTER (:902-904)
                if (before && !(r < T)) return false;                    // STARTED_BEFORE (:905-906)
                if (!after && norm_cmp(ex, Tn) < 0) return false;        // executeAtOrTxnId >= testTxnId (:907-908)
                if (!(fl & need)) return false;                          // IS_PROPOSED / IS_STABLE (:915-928)
                if (!((kinds >> kd) & 1)) return false;                  // testKind (:931)
                if (!(fl & 4u)) return false;                            // hasProposedOrDecidedDeps (:936)
                uint32_t a = v.rc_dep_off[c], z = v.rc_dep_off[c + 1];   // partialDeps().intersects (:946)
                while (a < z)
                {
                    const uint32_t m = (a + z) >> 1;
                    if (norm_cmp(NormTid{v.rc_dep_hi[m], v.rc_dep_lo[m], v.rc_dep_node[m]}, Tn) < 0) a = m + 1;
                    else z = m;
                }
                const bool inter = a < v.rc_dep_off[c + 1] && norm_cmp(NormTid{v.rc_dep_hi[a], v.rc_dep_lo[a], v.rc_dep_node[a]}, Tn) == 0;
                if (inter != with) return false;
                if (scan == 0 && !(norm_cmp(ex, Tn) > 0)) return false;  // the lambda: executeAt > startedBefore (BeginRecovery.java:335)
                val = ((uint64_t)s.r_rid[i] << 32) | r;
                return true;
            };
            uint32_t cursor = 0;
            bool overflow = false;
            auto leaf_stage = [&](uint64_t base, bool inr) {
                uint64_t val;
                const bool want = want_of(base + lane, inr, val);
                const uint64_t wm = ballot(want);
                const uint32_t n = __popcll(wm);
                if (!overflow && cursor + n <= K4_CAP)
                {
                    if (want) stage[wv][cursor + mbcnt(wm)] = val;
                }
                else overflow = true;
                cursor += n;
            };
            wave_descent(0, hi, s.n_rlevels, node_want, leaf_stage, stk[wv]);
            wave_lds_sync();
            cnt = cursor;
            off = cnt ? alloc.take(&b.ctl->rng_top, cap, &b.ctl->overflow, 2u, cnt, K4_CHUNK) : 0;
            if (off + cnt > cap)
            {
                off = 0;
                cnt = 0;                 // overflow: the host grows the arena and reruns
            }
            else if (cnt)
            {
                if (!overflow)
                    for (uint32_t i = lane; i < cnt; i += 64) b.rarena[off + i] = stage[wv][i];
                else
                {
                    uint32_t run = 0;
                    auto leaf_direct = [&](uint64_t base, bool inr) {
                        uint64_t val;
                        const bool want = want_of(base + lane, inr, val);
                        const uint64_t wm = ballot(want);
                        if (want) b.rarena[off + run + mbcnt(wm)] = val;
                        run += __popcll(wm);
                    };
                    wave_descent(0, hi, s.n_rlevels, node_want, leaf_direct, stk[wv]);
                }
            }
        }
        if (lane == 0)
        {
            b.p_roff[p] = (uint32_t)off;
            b.p_rcnt[p] = cnt;
            b.p_rb[p] = NO_RB;
        }
    }
}

hipError_t run_recovery(const DevSnapshot& s, const RecoveryView& v, const BatchBufs& b, uint32_t scan, hipStream_t st)
{
    if (b.n_txns)
        k_encode_recover<<<(unsigned)((b.n_txns + 255) / 256), 256, 0, st>>>(s, b);
    if (b.n_probes)
    {
        k_probe_keys<<<(unsigned)((b.n_probes + 255) / 256), 256, 0, st>>>(s, b);
        const uint64_t blocks_needed = (b.n_probes + K1_WAVES - 1) / K1_WAVES;
        const unsigned grid = (unsigned)std::min<uint64_t>(blocks_needed, (uint64_t)device_cu_count() * 8);
        k_recover<<<grid, 256, 0, st>>>(v, b, scan);
        if (v.ranges)
            k_range_recover<<<grid, 256, 0, st>>>(s, v, b, scan);
        else
        {
            // no live range commands: no range pairs (empty K4 lists)
            hipError_t e = hipMemsetAsync(b.p_rcnt, 0, sizeof(uint32_t) * b.n_probes, st);
            if (e == hipSuccess) e = hipMemsetAsync(b.p_rb, 0xFF, sizeof(uint64_t) * b.n_probes, st);
            if (e != hipSuccess) return e;
        }
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return run_build(s, b, st);
}

struct Bases9 { uint64_t b[9]; };

__global__ void k_add_bases(uint64_t* off, uint64_t n1, Bases9 base)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= 9 * n1) return;
    off[i] += base.b[i / n1];
}

hipError_t run_add_bases(uint64_t* off, uint64_t n1, const uint64_t* base, hipStream_t st)
{
    Bases9 b;
    bool any = false;
    for (int a = 0; a < 9; ++a) any |= (b.b[a] = base[a]) != 0;
    if (!any || !n1) return hipSuccess;
    k_add_bases<<<(unsigned)((9 * n1 + 255) / 256), 256, 0, st>>>(off, n1, b);
    return hipGetLastError();
}

// Copy-out of a slice of ad_deps_batch_into straight into the caller's pinned host arrays (their
// device-mapped addresses): the CUs' stores cross PCIe, so the copy-out runs beside the next slice's
// SDMA H2D (measured on the box, scripts/mb_pcie2.hip: kernel D2H 54 GB/s; with an SDMA H2D beside it
// 84 GB/s in all, against 57 GB/s in all for SDMA copies both ways). Offsets segments get the slice's
// base added on the way.
__global__ __launch_bounds__(256) void k_copy_out(OutSegs g)
{
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint32_t k = 0; k < g.n; ++k)
    {
        const OutSeg sg = g.s[k];
        const uintptr_t al = (uintptr_t)sg.src | (uintptr_t)sg.dst | (uintptr_t)sg.bytes;
        if (sg.mode == 1)
        {
            const uint64_t* a = (const uint64_t*)sg.src;
            uint64_t* d = (uint64_t*)sg.dst;
            for (uint64_t i = tid; i < sg.bytes / 8; i += stride) d[i] = a[i] + sg.add;
        }
        else if (sg.mode == 2)
        {
            // u32 -> u16, two per lane when aligned
            const uint32_t* a = (const uint32_t*)sg.src;
            uint16_t* d = (uint16_t*)sg.dst;
            const uint64_t m = sg.bytes / 4;
            if ((((uintptr_t)a | (uintptr_t)d) & 7) == 0)
            {
                for (uint64_t i = tid; 2 * i + 1 < m; i += stride)
                {
                    const uint2 v = ((const uint2*)a)[i];
                    ((uint32_t*)d)[i] = (v.x & 0xFFFFu) | (v.y << 16);
                }
                if (tid == 0 && (m & 1)) d[m - 1] = (uint16_t)a[m - 1];
            }
            else
                for (uint64_t i = tid; i < m; i += stride) d[i] = (uint16_t)a[i];
        }
        else if ((al & 15) == 0)
        {
            const uint4* a = (const uint4*)sg.src;
            uint4* d = (uint4*)sg.dst;
            for (uint64_t i = tid; i < sg.bytes / 16; i += stride) d[i] = a[i];
        }
        else if ((al & 7) == 0)
        {
            const uint64_t* a = (const uint64_t*)sg.src;
            uint64_t* d = (uint64_t*)sg.dst;
            for (uint64_t i = tid; i < sg.bytes / 8; i += stride) d[i] = a[i];
        }
        else if ((al & 3) == 0)
        {
            const uint32_t* a = (const uint32_t*)sg.src;
            uint32_t* d = (uint32_t*)sg.dst;
            for (uint64_t i = tid; i < sg.bytes / 4; i += stride) d[i] = a[i];
        }
        else
        {
            const uint8_t* a = (const uint8_t*)sg.src;
            uint8_t* d = (uint8_t*)sg.dst;
            for (uint64_t i = tid; i < sg.bytes; i += stride) d[i] = a[i];
        }
    }
}

// per request: its keyDeps keys (ascending, a subset of its query keys, ascending) as indices into the
// query keys; the u16 fit of its k2t segment and unique txns. off: the slice's 9 offset rows (map 0:
// rows 0 keys, 1 txns, 2 k2t), n + 1 entries each.
__global__ __launch_bounds__(256) void k_key_index(uint64_t n, const uint64_t* __restrict__ q_key_off,
                                                   const int64_t* __restrict__ q_keys, const uint64_t* __restrict__ off,
                                                   const int64_t* __restrict__ o_keys, uint8_t* __restrict__ idx,
                                                   uint32_t* flag)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t f = 0;
    if (i < n)
    {
        const uint64_t n1 = n + 1;
        const uint64_t qa = q_key_off[i], qb = q_key_off[i + 1];
        uint64_t q = qa;
        for (uint64_t k = off[i]; k < off[i + 1]; ++k)
        {
            const int64_t key = o_keys[k];
            while (q < qb && q_keys[q] < key) ++q;
            if (q >= qb || q_keys[q] != key || q - qa > 255)
            {
                f |= 1u;
                break;
            }
            idx[k] = (uint8_t)(q - qa);
        }
        if (off[2 * n1 + i + 1] - off[2 * n1 + i] > 65535 || off[n1 + i + 1] - off[n1 + i] > 65535) f |= 2u;
    }
    f = (ballot((f & 1u) != 0) ? 1u : 0u) | (ballot((f & 2u) != 0) ? 2u : 0u);
    if (lane_id() == 0 && f) atomicOr(flag, f);
}

hipError_t run_key_index(uint64_t n, const uint64_t* q_key_off, const int64_t* q_keys, const uint64_t* off,
                         const int64_t* o_keys, uint8_t* idx, uint32_t* flag, hipStream_t st)
{
    hipError_t e = hipMemsetAsync(flag, 0, 4, st);
    if (e != hipSuccess || !n) return e;
    k_key_index<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(n, q_key_off, q_keys, off, o_keys, idx, flag);
    return hipGetLastError();
}

hipError_t run_copy_out(const OutSegs& g, hipStream_t st)
{
    if (!g.n) return hipSuccess;
    unsigned blocks = 64;       // 64 blocks fill PCIe (6.5-6.8 ms per config-2 batch against 6.7-7.7 at 256); the CUs stay with the resolve
    k_copy_out<<<blocks, 256, 0, st>>>(g);
    return hipGetLastError();
}

// ---- RecoveryView of a live store (BeginRecovery.java:329-380 over CommandsForKey.mapReduceFull
// :809-908): built from the per-entry device state after ad_cfk_update / ad_cfk_prune ---------------
__global__ __launch_bounds__(256) void k_rv_entries(RvDevIn in, uint4* ent, uint32_t* cnt, uint32_t* err)
{
    const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= in.n_ent) return;
    const uint32_t txw = in.ent[e].y;
    uint32_t nm = 0, mo = 0;
    if (in.mref)
    {
        const uint32_t L = in.mref[e];
        if (L != 0xFFFFFFFFu && L != 0xFFFFFFFEu)          // MREF_NONE / MREF_BORN: NO_TXNIDS
        {
            const uint64_t a = in.moff[L], b = in.moff[L + 1];
            if (b - a > RV_MAX_MISS) atomicOr(err, 1u);
            nm = (uint32_t)min<uint64_t>(b - a, RV_MAX_MISS);
            mo = (uint32_t)a;
        }
    }
    ent[e] = make_uint4(txw & RANK_MASK, in.xrank[e], (uint32_t)in.status[e] | ((txw >> RANK_BITS) << 8) | (nm << RV_MISS_SHIFT), mo);
    cnt[e] = nm;
}

__global__ void k_rv_keys(RvDevIn in, uint32_t* seg, uint32_t* pruned)
{
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < in.n_keys)
    {
        seg[k] = in.krec[k].seg_lo;
        pruned[k] = in.krec[k].pruned;
    }
    if (k == in.n_keys) seg[k] = (uint32_t)in.n_ent;
}

hipError_t run_rv_entries(const RvDevIn& in, uint4* ent, uint32_t* seg, uint32_t* pruned, uint32_t* cnt, uint32_t* err,
                          hipStream_t st)
{
    if (in.n_ent) k_rv_entries<<<(unsigned)((in.n_ent + 255) / 256), 256, 0, st>>>(in, ent, cnt, err);
    k_rv_keys<<<(unsigned)((in.n_keys + 1 + 255) / 256), 256, 0, st>>>(in, seg, pruned);
    return hipGetLastError();
}

// level 1: one wave per 64-entry block, the max executeAt rank of the block's entries in each set
__global__ __launch_bounds__(256) void k_rv_tree_leaf(RvDevIn in, uint32_t* l0, uint32_t* l1, uint64_t n_blocks)
{
    const uint64_t blk = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (blk >= n_blocks) return;
    const uint64_t e = blk * 64 + lane_id();
    uint32_t a = 0, b = 0;
    if (e < in.n_ent)
    {
        const uint32_t stt = in.status[e], x = in.xrank[e];
        a = (stt == 3 || stt == 4) ? x : 0u;          // ACCEPTED, COMMITTED
        b = (stt == 5 || stt == 6) ? x : 0u;          // STABLE, APPLIED
    }
#pragma unroll
    for (int d = 32; d; d >>= 1)
    {
        a = max(a, (uint32_t)__shfl_xor(a, d, 64));
        b = max(b, (uint32_t)__shfl_xor(b, d, 64));
    }
    if (lane_id() == 0)
    {
        l0[blk] = a;
        l1[blk] = b;
    }
}

__global__ void k_rv_tree_up(const uint32_t* c0, const uint32_t* c1, uint64_t n_child, uint32_t* p0, uint32_t* p1, uint64_t n_parent)
{
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n_parent) return;
    uint32_t a = 0, b = 0;
    for (uint64_t i = j * 64; i < min<uint64_t>(n_child, j * 64 + 64); ++i)
    {
        a = max(a, c0[i]);
        b = max(b, c1[i]);
    }
    p0[j] = a;
    p1[j] = b;
}

hipError_t run_rv_trees(const RvDevIn& in, uint32_t* const* lvl0, uint32_t* const* lvl1, const uint64_t* lvl_n, int n_levels,
                        hipStream_t st)
{
    if (n_levels < 2) return hipSuccess;
    k_rv_tree_leaf<<<(unsigned)std::max<uint64_t>(1, (lvl_n[1] + 3) / 4), 256, 0, st>>>(in, lvl0[1], lvl1[1], lvl_n[1]);
    for (int l = 2; l < n_levels; ++l)
        k_rv_tree_up<<<(unsigned)std::max<uint64_t>(1, (lvl_n[l] + 255) / 256), 256, 0, st>>>(lvl0[l - 1], lvl1[l - 1], lvl_n[l - 1],
                                                                                             lvl0[l], lvl1[l], lvl_n[l]);
    return hipGetLastError();
}

__global__ __launch_bounds__(256) void k_rv_inv_pairs(RvDevIn in, const uint64_t* eoff, uint64_t* key, uint32_t* val)
{
    const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= in.n_ent) return;
    const uint64_t o = eoff[e], nm = eoff[e + 1] - o;
    if (!nm) return;
    const uint32_t L = in.mref[e];
    const uint64_t a = in.moff[L];
    const uint64_t k = (uint64_t)in.ekey[e] << 32;
    for (uint64_t j = 0; j < nm; ++j)
    {
        key[o + j] = k | in.mids[a + j];
        val[o + j] = (uint32_t)e;
    }
}

__global__ void k_rv_inv_off(RvDevIn in, const uint64_t* eoff, uint64_t* inv_off)
{
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < in.n_keys) inv_off[k] = eoff[in.krec[k].seg_lo];
    if (k == in.n_keys) inv_off[k] = eoff[in.n_ent];
}

__global__ void k_rv_inv_out(const uint64_t* skey, const uint32_t* sval, uint64_t n, uint2* inv)
{
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p < n) inv[p] = make_uint2((uint32_t)skey[p], sval[p]);
}

hipError_t run_rv_inv_pairs(const RvDevIn& in, const uint64_t* eoff, uint64_t* key, uint32_t* val, hipStream_t st)
{
    if (in.n_ent && in.mref) k_rv_inv_pairs<<<(unsigned)((in.n_ent + 255) / 256), 256, 0, st>>>(in, eoff, key, val);
    return hipGetLastError();
}

hipError_t run_rv_inv_finish(const RvDevIn& in, const uint64_t* eoff, const uint64_t* skey, const uint32_t* sval,
                             uint64_t n_pairs, uint64_t* inv_off, uint2* inv, hipStream_t st)
{
    k_rv_inv_off<<<(unsigned)((in.n_keys + 1 + 255) / 256), 256, 0, st>>>(in, eoff, inv_off);
    if (n_pairs) k_rv_inv_out<<<(unsigned)((n_pairs + 255) / 256), 256, 0, st>>>(skey, sval, n_pairs, inv);
    return hipGetLastError();
}

}  // namespace adx
