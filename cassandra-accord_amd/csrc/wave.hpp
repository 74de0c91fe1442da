// wave.hpp — wave64 building blocks for gfx950 (CDNA4): ballot/mbcnt compaction, 64-ary
// searches and the max-tree range-threshold descent used by the conflict scan (K1) and the
// range probe (K4).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "common.hpp"

namespace adx {

__device__ __forceinline__ int lane_id() { return __lane_id(); }

__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }

// blockIdx.x relabelled so that the blocks of one XCD (blocks are dealt round-robin over the 8 XCDs)
// hold consecutive ids: work handed out by block id in order then shares L2 lines inside an XCD, not
// across XCDs. Bijective for any grid size (cdna_hip_programming.md §T1).
__device__ __forceinline__ uint32_t xcd_block()
{
    const uint32_t nwg = gridDim.x, bid = blockIdx.x, x = bid & 7u, q = nwg >> 3, r = nwg & 7u;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
}

// number of set bits of m below this lane
__device__ __forceinline__ uint32_t mbcnt(uint64_t m)
{
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// compiler-level ordering of LDS/global accesses between lanes of one wave (the hardware keeps
// one wave's LDS operations in order; this stops the compiler from reordering across it)
__device__ __forceinline__ void wave_lds_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// The value of lane (lane ^ J), J a power of two below 64: DPP quad permutes (J = 1, 2), row shifts
// (J = 4, 8: the lanes with bit J clear read lane + J, the others lane - J, inside 16-lane rows) and
// gfx950's permlane16 / permlane32 swaps (J = 16, 32) -- VALU latency instead of a ds_bpermute round
// trip through the LDS unit. Every lane of the wave must execute it (a disabled source reads 0).
template <uint32_t J>
__device__ __forceinline__ uint32_t xor_lane_c(uint32_t v)
{
    const int x = (int)v;
    if constexpr (J == 1) return (uint32_t)__builtin_amdgcn_mov_dpp(x, 0xB1, 0xF, 0xF, true);    // quad_perm [1,0,3,2]
    else if constexpr (J == 2) return (uint32_t)__builtin_amdgcn_mov_dpp(x, 0x4E, 0xF, 0xF, true);   // quad_perm [2,3,0,1]
    else if constexpr (J == 4 || J == 8)
    {
        const uint32_t up = (uint32_t)__builtin_amdgcn_mov_dpp(x, 0x100 + (int)J, 0xF, 0xF, true);   // row_shl:J
        const uint32_t dn = (uint32_t)__builtin_amdgcn_mov_dpp(x, 0x110 + (int)J, 0xF, 0xF, true);   // row_shr:J
        return (__lane_id() & J) ? dn : up;
    }
    else if constexpr (J == 16)
    {
        const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
        return (__lane_id() & 16) ? r[0] : r[1];
    }
    else if constexpr (J == 32)
    {
        const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
        return (__lane_id() & 32) ? r[0] : r[1];
    }
    else return (uint32_t)__shfl_xor(x, (int)J, 64);
}
// j known after unrolling
__device__ __forceinline__ uint32_t xor_lane(uint32_t v, uint32_t j)
{
    switch (j)
    {
        case 1: return xor_lane_c<1>(v);
        case 2: return xor_lane_c<2>(v);
        case 4: return xor_lane_c<4>(v);
        case 8: return xor_lane_c<8>(v);
        case 16: return xor_lane_c<16>(v);
        case 32: return xor_lane_c<32>(v);
        default: return (uint32_t)__shfl_xor((int)v, (int)j, 64);
    }
}
__device__ __forceinline__ uint64_t xor_lane64(uint64_t v, uint32_t j)
{
    return ((uint64_t)xor_lane((uint32_t)(v >> 32), j) << 32) | xor_lane((uint32_t)v, j);
}
// lane - d inside 16-lane rows (d in 1, 2, 4, 8, known after unrolling); lanes with (lane % 16) < d read 0
__device__ __forceinline__ uint32_t row_up(uint32_t v, uint32_t d)
{
    const int x = (int)v;
    switch (d)
    {
        case 1: return (uint32_t)__builtin_amdgcn_mov_dpp(x, 0x111, 0xF, 0xF, true);
        case 2: return (uint32_t)__builtin_amdgcn_mov_dpp(x, 0x112, 0xF, 0xF, true);
        case 4: return (uint32_t)__builtin_amdgcn_mov_dpp(x, 0x114, 0xF, 0xF, true);
        default: return (uint32_t)__builtin_amdgcn_mov_dpp(x, 0x118, 0xF, 0xF, true);
    }
}
// lane - 1 over the whole wave (lane 0 reads 0)
__device__ __forceinline__ uint32_t wave_up1(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x138, 0xF, 0xF, true);      // wave_shr:1
}

// inclusive prefix sum over the 64 lanes in DPP steps (row shifts, then the row broadcasts of lanes 15
// and 31): VALU latency per step instead of a ds_bpermute round trip. Every lane must execute it.
__device__ __forceinline__ uint32_t wave_incl_scan_dpp(uint32_t x)
{
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);     // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);     // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);     // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);     // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);     // row_bcast:15 -> rows 1, 3
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);     // row_bcast:31 -> rows 2, 3
    return x;
}

// inclusive prefix max over the 64 lanes in DPP steps (as wave_incl_scan_dpp; values >= 0, absent lanes read 0)
__device__ __forceinline__ uint32_t wave_incl_max_dpp(uint32_t x)
{
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false));     // row_shr:1
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false));     // row_shr:2
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false));     // row_shr:4
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false));     // row_shr:8
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false));     // row_bcast:15 -> rows 1, 3
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false));     // row_bcast:31 -> rows 2, 3
    return x;
}

// inclusive prefix sum of 64-bit values over the 64 lanes: DPP steps in 32 bits while the wave's sum
// surely fits (every value below 2^25), else the shuffle scan. Every lane must execute it.
__device__ __forceinline__ uint64_t wave_incl_scan64(uint64_t v)
{
    if (__ballot(v >= (1ull << 25)) == 0) return wave_incl_scan_dpp((uint32_t)v);
    const int l = __lane_id();
#pragma unroll
    for (int d = 1; d < 64; d <<= 1)
    {
        const uint64_t t = __shfl_up(v, d, 64);
        if (l >= d) v += t;
    }
    return v;
}

__device__ __forceinline__ uint32_t uniform(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t uniform64(uint64_t v)
{
    uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

// inclusive wave prefix sum
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v)
{
    const int l = lane_id();
#pragma unroll
    for (int d = 1; d < 64; d <<= 1)
    {
        uint32_t t = __shfl_up(v, d, 64);
        if (l >= d) v += t;
    }
    return v;
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v)
{
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}

// lower_bound over a sorted sequence key(i), i in [lo, hi): the first i with !(key(i) < x),
// or hi. 64-ary: each round every lane loads one pivot (64 independent loads, one round trip).
template <class KeyAt, class Less>
__device__ __forceinline__ uint64_t wave_lower_bound(uint64_t lo, uint64_t hi, KeyAt key, Less less)
{
    const uint32_t l = lane_id();
    while (hi - lo > 64)
    {
        const uint64_t n = hi - lo;
        const uint64_t p = lo + (((uint64_t)(l + 1) * n) >> 6) - 1;     // p_63 = hi - 1
        const uint64_t m = ballot(less(key(p)));
        const uint32_t c = __popcll(m);
        if (c == 64) return hi;
        const uint64_t pc = lo + (((uint64_t)(c + 1) * n) >> 6) - 1;
        const uint64_t nlo = c == 0 ? lo : lo + (((uint64_t)c * n) >> 6);   // p_{c-1} + 1
        lo = nlo;
        hi = pc;                       // key(pc) >= x: the answer is in [nlo, pc]
    }
    const uint64_t i = lo + l;
    const bool v = i < hi && less(key(i));
    return lo + __popcll(ballot(v));
}

// Max-tree range-threshold descent.
//   Report, in ascending index order, every leaf i in [lo, end) for which leaf_want(i) holds,
//   pruning with a 64-ary tree whose level-l node j summarises leaves [j*64^l, (j+1)*64^l):
//   node_want(l, j) must be true whenever any leaf below j may be wanted.
//   `leaf(base, want_lane)` is called for every level-0 frame (64 consecutive leaves from
//   base) with the lane's own want bit; it runs the emission.
// Stack of (base, pending-children mask) per level lives in wave-private LDS `stk`; every lane
// writes the same (wave-uniform) value and reads back its own write, so no cross-lane sync.
template <class NodeWant, class LeafFrame>
__device__ __forceinline__ void wave_descent(uint64_t lo, uint64_t end, int n_levels, NodeWant node_want,
                                             LeafFrame leaf, uint64_t* stk /* [2*MAX_LEVELS] */)
{
    if (end <= lo) return;
    const uint32_t l = lane_id();
    int k = 0;
    while (k + 1 < n_levels && (((end - 1) >> (6 * k)) - (lo >> (6 * k))) >= 64) ++k;

    auto frame = [&](int lv, uint64_t base) -> uint64_t {
        const uint64_t node = base + l;
        const bool inr = node >= (lo >> (6 * lv)) && node <= ((end - 1) >> (6 * lv));
        if (lv == 0)
        {
            leaf(base, inr);
            return 0;
        }
        return ballot(inr && node_want(lv, node));
    };

    uint64_t m = frame(k, lo >> (6 * k));
    if (k == 0) return;
    int lv = k;
    stk[2 * lv] = lo >> (6 * k);
    stk[2 * lv + 1] = m;
    uint64_t base = lo >> (6 * k);
    while (true)
    {
        if (m == 0)
        {
            if (++lv > k) break;
            base = stk[2 * lv];
            m = stk[2 * lv + 1];
            continue;
        }
        const int b = __ffsll((unsigned long long)m) - 1;
        m &= m - 1;
        const uint64_t cbase = (base + b) << 6;
        if (lv == 1)
        {
            frame(0, cbase);           // leaves: emitted inline, nothing to push
            continue;
        }
        stk[2 * lv] = base;
        stk[2 * lv + 1] = m;
        lv -= 1;
        base = cbase;
        m = frame(lv, cbase);
    }
}

}  // namespace adx
