// levels.hip — K5: execution-ordering levels for apply scheduling.
//
// Reference: a committed txn T executes once everything it waits on has applied
// (Command.WaitingOn, Command.java:1224-1381; Commands.updateWaitingOn / maybeExecute,
// Commands.java:617-775; CommandsForKey.notifyManaged, CommandsForKey.java:1193-1274). On each
// key T waits for every txn P executing before it (executeAt order) whose kind T witnesses
// (Txn.Kind.witnesses, Txn.java:221-235), and for its direct deps executing before it.
// level(T) = 0 if T waits on nothing, else 1 + max level(P): the apply round of T when every txn
// applies as soon as all it waits on has applied (oracle: rc_levels, oracle/refcpu.c).
//
// Device pipeline (all integer, HBM/latency bound, no MFMA):
//   1. rank executeAts: LSD radix sort of txn indices by the normalised Timestamp
//      (node, then lowHlc|flags, then msb; digits that are constant over the batch are skipped)
//   2. key chains: the (key, exec rank) occurrences, generated in rank order and stably radix
//      sorted by key, give every key's txns in executeAt order
//   3. sparsified predecessors: per occurrence a backward walk of its chain that keeps P only
//      while no later predecessor already dominates P's kind (a predecessor Q witnessing kind c
//      has level(Q) > level of every earlier kind-c txn) -> successor CSR + in-degrees
//   4. frontier loop (Kahn by levels): frontier L = txns whose in-degree reached 0 while
//      frontier L-1 was processed; one launch per level, launched in chunks between host checks
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/accord_deps.h"
#include "common.hpp"
#include "kernels.hpp"
#include "levels.hpp"
#include "wave.hpp"
#include "devmem.hpp"

namespace adx {

// ---------------------------------------------------------------------------------------------
// LSD radix sort of (u64 key, u32 val), 8-bit digits, stable
// ---------------------------------------------------------------------------------------------
constexpr int RS_THREADS = 256;
constexpr int RS_WAVES = RS_THREADS / 64;
constexpr int RS_CHUNKS = 16;                       // 64-element chunks per wave
constexpr int RS_TILE = RS_THREADS * RS_CHUNKS;     // 4096 elements per block

uint64_t radix_hist_entries(uint64_t n)
{
    // 256 digit counts per RS_TILE tile
    return 256 * std::max<uint64_t>(1, (n + RS_TILE - 1) / RS_TILE);
}

// per block digit counts -> hist[d * nblk + b] (digit-major, so one flat exclusive scan gives
// every (digit, block) its output base)
__global__ __launch_bounds__(RS_THREADS) void k_radix_count(const uint64_t* __restrict__ k, uint64_t n, int shift,
                                                             uint32_t* __restrict__ hist, uint32_t nblk)
{
    __shared__ uint32_t h[256];
    h[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * RS_TILE;
#pragma unroll 4
    for (int c = 0; c < RS_CHUNKS; ++c)
    {
        const uint64_t i = base + (uint64_t)c * RS_THREADS + threadIdx.x;
        if (i < n) atomicAdd(&h[(uint32_t)(k[i] >> shift) & 255u], 1u);
    }
    __syncthreads();
    hist[(uint64_t)threadIdx.x * nblk + blockIdx.x] = h[threadIdx.x];
}

// stable scatter: wave w of block b owns elements [b*TILE + w*1024, +1024) in 16 chunks of 64;
// rank inside a chunk = lanes below with the same digit (8 ballots), chunk order kept by a
// per-wave running count per digit in LDS
__global__ __launch_bounds__(RS_THREADS) void k_radix_scatter(const uint64_t* __restrict__ k, const uint32_t* __restrict__ v,
                                                               uint64_t n, int shift, const uint64_t* __restrict__ off,
                                                               uint32_t nblk, uint64_t* __restrict__ ko,
                                                               uint32_t* __restrict__ vo)
{
    __shared__ uint64_t cnt[RS_WAVES][256];
    const uint32_t w = threadIdx.x >> 6, lane = lane_id();
    for (int d = threadIdx.x; d < RS_WAVES * 256; d += RS_THREADS) (&cnt[0][0])[d] = 0;
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * RS_TILE + (uint64_t)w * (RS_CHUNKS * 64);
    uint64_t key[RS_CHUNKS];
    uint32_t val[RS_CHUNKS];
#pragma unroll
    for (int c = 0; c < RS_CHUNKS; ++c)
    {
        const uint64_t i = base + (uint64_t)c * 64 + lane;
        key[c] = i < n ? k[i] : 0;
        val[c] = i < n ? v[i] : 0;
        if (i < n) atomicAdd((unsigned long long*)&cnt[w][(uint32_t)(key[c] >> shift) & 255u], 1ull);
    }
    __syncthreads();
    // cnt[w][d] <- global base of (d, block) + elements of digit d in earlier waves
    {
        const uint32_t d = threadIdx.x;
        uint64_t run = off[(uint64_t)d * nblk + blockIdx.x];
        for (int ww = 0; ww < RS_WAVES; ++ww)
        {
            const uint64_t c = cnt[ww][d];
            cnt[ww][d] = run;
            run += c;
        }
    }
    __syncthreads();
    const uint64_t lt = (1ull << lane) - 1;
#pragma unroll
    for (int c = 0; c < RS_CHUNKS; ++c)
    {
        const uint64_t i = base + (uint64_t)c * 64 + lane;
        const bool live = i < n;
        const uint32_t d = (uint32_t)(key[c] >> shift) & 255u;
        uint64_t m = ballot(live);
#pragma unroll
        for (int bit = 0; bit < 8; ++bit)
        {
            const uint64_t b = ballot((d >> bit) & 1u);
            m &= ((d >> bit) & 1u) ? b : ~b;
        }
        const uint64_t pos0 = live ? cnt[w][d] : 0;
        wave_lds_sync();
        if (live)
        {
            const uint64_t pos = pos0 + __popcll(m & lt);
            ko[pos] = key[c];
            vo[pos] = val[c];
            if ((m >> lane) == 1ull) cnt[w][d] = pos0 + __popcll(m);    // highest lane of its digit group
        }
        wave_lds_sync();
    }
}

hipError_t radix_sort_pairs(uint64_t* k_in, uint32_t* v_in, uint64_t* k_tmp, uint32_t* v_tmp, uint64_t n,
                            uint32_t digit_mask, uint32_t* hist, uint64_t* off, uint64_t* bsum, hipStream_t st,
                            uint64_t** k_res, uint32_t** v_res)
{
    // (a onesweep variant -- one kernel per digit with a decoupled look-back -- measured no faster on the K5
    // sorts: 0.039 ms per digit against 0.052 for count + scan + scatter, but its global count pass and two
    // fills per sort ate the difference; deleted in round 6)
    uint64_t* ka = k_in;
    uint32_t* va = v_in;
    uint64_t* kb = k_tmp;
    uint32_t* vb = v_tmp;
    const uint32_t nblk = (uint32_t)std::max<uint64_t>(1, (n + RS_TILE - 1) / RS_TILE);
    if (n > 1)
        for (int d = 0; d < 8; ++d)
        {
            if (!((digit_mask >> d) & 1u)) continue;
            k_radix_count<<<nblk, RS_THREADS, 0, st>>>(ka, n, 8 * d, hist, nblk);
            hipError_t e = run_scan_arrays(hist, off, 256ull * nblk, 1, bsum, st);
            if (e != hipSuccess) return e;
            k_radix_scatter<<<nblk, RS_THREADS, 0, st>>>(ka, va, n, 8 * d, off, nblk, kb, vb);
            std::swap(ka, kb);
            std::swap(va, vb);
        }
    *k_res = ka;
    *v_res = va;
    return hipGetLastError();
}

static uint32_t digits_of(uint64_t diff)
{
    uint32_t m = 0;
    for (int d = 0; d < 8; ++d)
        if ((diff >> (8 * d)) & 0xFF) m |= 1u << d;
    return m;
}

// ---------------------------------------------------------------------------------------------
// Stable LSD radix sort of packed u64 keys (no values) on the bit field [lo, lo + bits): digits of
// DB = 8..11 bits, as few passes as the field needs (a 17-bit field: two 9-bit passes, 42 bits: four
// 11-bit ones). Same count / scan / scatter structure as the pair sort above; per-wave digit counts
// in LDS as u32 (below 2^32 elements).
// ---------------------------------------------------------------------------------------------
template <int DB>
__global__ __launch_bounds__(RS_THREADS) void k_rk_count(const uint64_t* __restrict__ k, uint64_t n, int shift,
                                                          uint32_t* __restrict__ hist, uint32_t nblk)
{
    constexpr uint32_t R = 1u << DB;
    __shared__ uint32_t h[R];
    for (uint32_t d = threadIdx.x; d < R; d += RS_THREADS) h[d] = 0;
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * RS_TILE;
    uint64_t key[RS_CHUNKS];
#pragma unroll
    for (int c = 0; c < RS_CHUNKS; ++c)
    {
        const uint64_t i = base + (uint64_t)c * RS_THREADS + threadIdx.x;
        key[c] = i < n ? k[i] : 0;
    }
#pragma unroll
    for (int c = 0; c < RS_CHUNKS; ++c)
        if (base + (uint64_t)c * RS_THREADS + threadIdx.x < n) atomicAdd(&h[(uint32_t)(key[c] >> shift) & (R - 1)], 1u);
    __syncthreads();
    for (uint32_t d = threadIdx.x; d < R; d += RS_THREADS) hist[(uint64_t)d * nblk + blockIdx.x] = h[d];
}

template <int DB>
__global__ __launch_bounds__(RS_THREADS) void k_rk_scatter(const uint64_t* __restrict__ k, uint64_t n, int shift,
                                                            const uint64_t* __restrict__ off, uint32_t nblk,
                                                            uint64_t* __restrict__ ko)
{
    constexpr uint32_t R = 1u << DB;
    __shared__ uint32_t cnt[RS_WAVES][R];
    const uint32_t w = threadIdx.x >> 6, lane = lane_id();
    for (uint32_t d = threadIdx.x; d < RS_WAVES * R; d += RS_THREADS) (&cnt[0][0])[d] = 0;
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * RS_TILE + (uint64_t)w * (RS_CHUNKS * 64);
    uint64_t key[RS_CHUNKS];
#pragma unroll
    for (int c = 0; c < RS_CHUNKS; ++c)
    {
        const uint64_t i = base + (uint64_t)c * 64 + lane;
        key[c] = i < n ? k[i] : 0;
        if (i < n) atomicAdd(&cnt[w][(uint32_t)(key[c] >> shift) & (R - 1)], 1u);
    }
    __syncthreads();
    for (uint32_t d = threadIdx.x; d < R; d += RS_THREADS)
    {
        uint32_t run = (uint32_t)off[(uint64_t)d * nblk + blockIdx.x];
#pragma unroll
        for (int ww = 0; ww < RS_WAVES; ++ww)
        {
            const uint32_t c = cnt[ww][d];
            cnt[ww][d] = run;
            run += c;
        }
    }
    __syncthreads();
    const uint64_t lt = (1ull << lane) - 1;
#pragma unroll
    for (int c = 0; c < RS_CHUNKS; ++c)
    {
        const uint64_t i = base + (uint64_t)c * 64 + lane;
        const bool live = i < n;
        const uint32_t d = (uint32_t)(key[c] >> shift) & (R - 1);
        uint64_t m = ballot(live);
#pragma unroll
        for (int bit = 0; bit < DB; ++bit)
        {
            const uint64_t b = ballot((d >> bit) & 1u);
            m &= ((d >> bit) & 1u) ? b : ~b;
        }
        const uint32_t pos0 = live ? cnt[w][d] : 0u;
        wave_lds_sync();
        if (live)
        {
            ko[pos0 + (uint32_t)__popcll(m & lt)] = key[c];
            if ((m >> lane) == 1ull) cnt[w][d] = pos0 + (uint32_t)__popcll(m);    // highest lane of its digit group
        }
        wave_lds_sync();
    }
}

// the sorted keys end in *k_res (k_in or k_tmp)
static hipError_t radix_sort_keys(uint64_t* k_in, uint64_t* k_tmp, uint64_t n, int lo, int bits, uint32_t* hist,
                                  uint64_t* off, uint64_t* bsum, hipStream_t st, uint64_t** k_res)
{
    uint64_t* ka = k_in;
    uint64_t* kb = k_tmp;
    *k_res = ka;
    if (n <= 1 || bits <= 0) return hipSuccess;
    const int passes = (bits + 10) / 11;
    const int db = std::max(8, (bits + passes - 1) / passes);
    const uint32_t nblk = (uint32_t)std::max<uint64_t>(1, (n + RS_TILE - 1) / RS_TILE);
    for (int p = 0; p < passes; ++p)
    {
        const int shift = lo + p * db;
        switch (db)
        {
            case 8: k_rk_count<8><<<nblk, RS_THREADS, 0, st>>>(ka, n, shift, hist, nblk); break;
            case 9: k_rk_count<9><<<nblk, RS_THREADS, 0, st>>>(ka, n, shift, hist, nblk); break;
            case 10: k_rk_count<10><<<nblk, RS_THREADS, 0, st>>>(ka, n, shift, hist, nblk); break;
            default: k_rk_count<11><<<nblk, RS_THREADS, 0, st>>>(ka, n, shift, hist, nblk); break;
        }
        hipError_t e = run_scan_arrays(hist, off, ((uint64_t)1 << db) * nblk, 1, bsum, st);
        if (e != hipSuccess) return e;
        switch (db)
        {
            case 8: k_rk_scatter<8><<<nblk, RS_THREADS, 0, st>>>(ka, n, shift, off, nblk, kb); break;
            case 9: k_rk_scatter<9><<<nblk, RS_THREADS, 0, st>>>(ka, n, shift, off, nblk, kb); break;
            case 10: k_rk_scatter<10><<<nblk, RS_THREADS, 0, st>>>(ka, n, shift, off, nblk, kb); break;
            default: k_rk_scatter<11><<<nblk, RS_THREADS, 0, st>>>(ka, n, shift, off, nblk, kb); break;
        }
        std::swap(ka, kb);
    }
    *k_res = ka;
    return hipGetLastError();
}

// hist entries the keys-only sort needs (2^11 digits per tile)
static uint64_t radix_keys_hist_entries(uint64_t n)
{
    return 2048 * std::max<uint64_t>(1, (n + RS_TILE - 1) / RS_TILE);
}

// parallel bit extract: the bits of x under mask m, packed from bit 0 up in order (m uniform)
__device__ __forceinline__ uint64_t pext64(uint64_t x, uint64_t m)
{
    uint64_t r = 0;
    uint32_t o = 0;
    while (m)
    {
        const uint32_t s = (uint32_t)__builtin_ctzll(m);
        const uint64_t sh = m >> s;
        const uint32_t len = ~sh == 0 ? 64u - s : (uint32_t)__builtin_ctzll(~sh);
        const uint64_t lm = len >= 64 ? ~0ull : ((1ull << len) - 1);
        r |= ((x >> s) & lm) << o;
        o += len;
        m &= ~(lm << s);
    }
    return r;
}

// ---------------------------------------------------------------------------------------------
// K5 kernels
// ---------------------------------------------------------------------------------------------
struct LevelsCtl {
    unsigned long long diff[4];     // OR of (word ^ word of element 0): exec node, lo, hi; occurrence keys
    unsigned int error;             // AD_E_* (negated)
    unsigned int maxk;              // most keys of one txn
    unsigned long long n_edges;     // packed path: key-chain + direct predecessors
    unsigned long long pool_used;   // packed path: overflow predecessor words asked for
    unsigned int mink_inv;          // ~(fewest keys of one txn)
    unsigned int pad;
};

// k_exec_words' per-block partials, combined by k_exec_words_reduce (one block): a few hundred
// blocks each ORing into the same control line would queue their atomics on it
struct WordsPart {
    unsigned long long diff[4];
    unsigned int maxk, mink_inv;
};

constexpr unsigned RED_BLOCKS = 512;     // grid of the reducing kernels: one atomic per block and word

// OR of v over the block (256 threads) -> one atomicOr per block
__device__ __forceinline__ void block_or_to(unsigned long long* dst, uint64_t v, uint64_t* red /* LDS [4] */)
{
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v |= __shfl_xor(v, d, 64);
    if (lane_id() == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0)
    {
        const uint64_t x = red[0] | red[1] | red[2] | red[3];
        if (x) atomicOr(dst, (unsigned long long)x);
    }
    __syncthreads();
}

// normalised executeAt words (Timestamp.compareTo order, Timestamp.java:208-217, common.hpp
// norm_tid): w0 = node with the sign flipped (signed compare), w1 = lowHlc|identity flags, w2 = msb.
// w0/idx null: the diffs only. Also the occurrence keys' diff (n_occ keys) and the most / fewest keys
// of one txn, per block into part[blockIdx.x].
__global__ __launch_bounds__(256) void k_exec_words(LevelsIn g, uint64_t* __restrict__ w0, uint32_t* __restrict__ idx,
                                                    WordsPart* __restrict__ part)
{
    // occurrences: key_off[n] read here, so the host learns it with the diffs in one round trip (a value
    // past 2^40 is refused by the host before anything reads the keys past the first pass)
    const uint64_t n_occ_raw = g.key_off[g.n];
    const uint64_t n_occ = n_occ_raw > (1ull << 40) ? 0 : n_occ_raw;
    __shared__ uint64_t red[4][6];
    uint64_t d0 = 0, d1 = 0, d2 = 0, dk = 0;
    uint32_t mk = 0, mi = 0;
    const NormTid z = norm_tid(g.exec_msb[0], g.exec_lsb[0], g.exec_node[0]);
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < g.n; i += stride)
    {
        const NormTid x = norm_tid(g.exec_msb[i], g.exec_lsb[i], g.exec_node[i]);
        if (w0)
        {
            w0[i] = (uint64_t)((uint32_t)x.node ^ 0x80000000u);
            idx[i] = (uint32_t)i;
        }
        d0 |= (uint64_t)((uint32_t)x.node ^ (uint32_t)z.node);
        d1 |= x.lo ^ z.lo;
        d2 |= x.hi ^ z.hi;
        const uint32_t kc = (uint32_t)std::min<uint64_t>(g.key_off[i + 1] - g.key_off[i], 0xFFFFFFFFull);
        mk = max(mk, kc);
        mi = max(mi, ~kc);
    }
    if (n_occ)
    {
        const uint64_t k0 = (uint64_t)g.keys[0];
        const uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
        uint64_t i = i0;
        for (; i + 3 * stride < n_occ; i += 4 * stride)
        {
            const uint64_t a = (uint64_t)g.keys[i], b = (uint64_t)g.keys[i + stride], c = (uint64_t)g.keys[i + 2 * stride],
                           d = (uint64_t)g.keys[i + 3 * stride];
            dk |= (a ^ k0) | (b ^ k0) | (c ^ k0) | (d ^ k0);
        }
        for (; i < n_occ; i += stride) dk |= (uint64_t)g.keys[i] ^ k0;
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1)
    {
        d0 |= __shfl_xor(d0, d, 64);
        d1 |= __shfl_xor(d1, d, 64);
        d2 |= __shfl_xor(d2, d, 64);
        dk |= __shfl_xor(dk, d, 64);
        mk = max(mk, (uint32_t)__shfl_xor(mk, d, 64));
        mi = max(mi, (uint32_t)__shfl_xor(mi, d, 64));
    }
    const uint32_t w = threadIdx.x >> 6;
    if (lane_id() == 0)
    {
        red[w][0] = d0;
        red[w][1] = d1;
        red[w][2] = d2;
        red[w][3] = dk;
        red[w][4] = mk;
        red[w][5] = mi;
    }
    __syncthreads();
    if (threadIdx.x < 6)
    {
        const uint32_t f = threadIdx.x;
        uint64_t v = red[0][f];
        for (uint32_t ww = 1; ww < (blockDim.x >> 6); ++ww) v = f < 4 ? (v | red[ww][f]) : std::max(v, red[ww][f]);
        if (f < 4) part[blockIdx.x].diff[f] = v;
        else if (f == 4) part[blockIdx.x].maxk = (uint32_t)v;
        else part[blockIdx.x].mink_inv = (uint32_t)v;
    }
}

__global__ __launch_bounds__(256) void k_exec_words_reduce(const WordsPart* __restrict__ part, uint32_t nb, LevelsCtl* ctl)
{
    __shared__ uint64_t red[4][6];
    uint64_t d[4] = {0, 0, 0, 0};
    uint32_t mk = 0, mi = 0;
    for (uint32_t b = threadIdx.x; b < nb; b += blockDim.x)
    {
#pragma unroll
        for (int f = 0; f < 4; ++f) d[f] |= part[b].diff[f];
        mk = max(mk, part[b].maxk);
        mi = max(mi, part[b].mink_inv);
    }
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1)
    {
#pragma unroll
        for (int f = 0; f < 4; ++f) d[f] |= __shfl_xor(d[f], s, 64);
        mk = max(mk, (uint32_t)__shfl_xor(mk, s, 64));
        mi = max(mi, (uint32_t)__shfl_xor(mi, s, 64));
    }
    const uint32_t w = threadIdx.x >> 6;
    if (lane_id() == 0)
    {
        for (int f = 0; f < 4; ++f) red[w][f] = d[f];
        red[w][4] = mk;
        red[w][5] = mi;
    }
    __syncthreads();
    if (threadIdx.x == 0)
    {
        for (uint32_t ww = 1; ww < (blockDim.x >> 6); ++ww)
        {
            for (int f = 0; f < 4; ++f) red[0][f] |= red[ww][f];
            red[0][4] = std::max(red[0][4], red[ww][4]);
            red[0][5] = std::max(red[0][5], red[ww][5]);
        }
        for (int f = 0; f < 4; ++f) ctl->diff[f] = red[0][f];
        ctl->maxk = (uint32_t)red[0][4];
        ctl->mink_inv = (uint32_t)red[0][5];
    }
}

// next (more significant) word of the current order
__global__ void k_exec_gather(LevelsIn g, const uint32_t* __restrict__ idx, int word, uint64_t* __restrict__ out)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= g.n) return;
    const uint32_t t = idx[i];
    const NormTid x = norm_tid(g.exec_msb[t], g.exec_lsb[t], g.exec_node[t]);
    out[i] = word == 1 ? x.lo : x.hi;
}

// An occurrence carries its txn's exec rank and kind in one word: rank | kind << OCC_KIND_SHIFT (ranks
// below 2^29). Kinds 6 and above (no Txn.Kind) all behave alike in the chain walk -- they witness
// nothing and nothing witnesses them -- so they are clamped to 7.
constexpr uint32_t OCC_KIND_SHIFT = 29;
constexpr uint32_t OCC_RANK_MASK = (1u << OCC_KIND_SHIFT) - 1;
__host__ __device__ inline uint32_t occ_word(uint32_t rank, uint32_t kind)
{
    return rank | ((kind < 7u ? kind : 7u) << OCC_KIND_SHIFT);
}

// rank[order[r]] = r; key count by rank; duplicate executeAt -> AD_E_DUP_EXEC
// (the reference's committedByExecuteAt never holds two, CommandsForKey.java:1439)
__global__ void k_exec_rank(LevelsIn g, const uint32_t* __restrict__ order, uint32_t* __restrict__ rank,
                            uint32_t* __restrict__ kcnt_r, LevelsCtl* ctl)
{
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= g.n) return;
    const uint32_t t = order[r];
    rank[t] = (uint32_t)r;
    kcnt_r[r] = (uint32_t)(g.key_off[t + 1] - g.key_off[t]);
    if (r > 0)
    {
        const uint32_t p = order[r - 1];
        const NormTid a = norm_tid(g.exec_msb[p], g.exec_lsb[p], g.exec_node[p]);
        const NormTid b = norm_tid(g.exec_msb[t], g.exec_lsb[t], g.exec_node[t]);
        if (norm_cmp(a, b) == 0) atomicCAS(&ctl->error, 0u, (unsigned)(-AD_E_DUP_EXEC));
    }
}

// occurrences in exec-rank order: okey = key with the sign flipped, oval = occ_word(rank, kind)
__global__ __launch_bounds__(256) void k_occ_fill(LevelsIn g, const uint32_t* __restrict__ order,
                                                  const uint64_t* __restrict__ occ_off, uint64_t* __restrict__ okey,
                                                  uint32_t* __restrict__ oval, LevelsCtl* ctl)
{
    __shared__ uint64_t red[4];
    uint64_t d = 0;
    for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < g.n; r += (uint64_t)gridDim.x * blockDim.x)
    {
        const uint32_t t = order[r];
        const uint64_t s = g.key_off[t], e = g.key_off[t + 1], o = occ_off[r];
        const uint64_t ref = (uint64_t)g.keys[0];
        const uint32_t w = occ_word((uint32_t)r, g.kind[t]);
        for (uint64_t j = s; j < e; ++j)
        {
            const uint64_t k = (uint64_t)g.keys[j];
            okey[o + (j - s)] = k ^ 0x8000000000000000ull;
            oval[o + (j - s)] = w;
            d |= k ^ ref;
        }
    }
    block_or_to(&ctl->diff[3], d, red);
}

// Sparsified predecessors of the occurrence at p (chain sorted by (key, rank)): walk back while
// some kind T witnesses is not yet dominated. A txn P of kind c is dominated once a predecessor
// (or a dominated txn) found later in the walk witnesses c: that one executes after P and waits
// on it, so its level is larger. Pass 0: in-degree of T and (outdeg non-null) out-degree of each P;
// pass 1: succ (successor lists); pass 2: pred (predecessor lists, offsets succ_off = scan of indeg).
// The walk reads only the sorted occurrences (key, rank | kind): sequential, no per-step gather.
template <int PASS>
__global__ void k_chain(const uint64_t* __restrict__ okey, const uint32_t* __restrict__ oval, uint64_t n_occ,
                        uint32_t* __restrict__ indeg, uint32_t* __restrict__ outdeg,
                        const uint64_t* __restrict__ succ_off, uint32_t* __restrict__ cursor, uint32_t* __restrict__ succ)
{
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n_occ) return;
    const uint64_t key = okey[p];
    const uint32_t wT = oval[p];
    const uint32_t T = wT & OCC_RANK_MASK;
    const uint32_t A = kind_witnesses(wT >> OCC_KIND_SHIFT);
    uint32_t D = 0, npred = 0;
    for (uint64_t q = p; q-- > 0 && (A & ~D) != 0;)
    {
        if (okey[q] != key) break;
        const uint32_t wP = oval[q];
        const uint32_t P = wP & OCC_RANK_MASK;
        const uint32_t kp = wP >> OCC_KIND_SHIFT;
        const uint32_t bit = kp < 32 ? 1u << kp : 0u;
        if (A & bit & ~D)
        {
            ++npred;
            if (PASS == 0) { if (outdeg) atomicAdd(&outdeg[P], 1u); }
            else if (PASS == 1) succ[succ_off[P] + atomicAdd(&cursor[P], 1u)] = T;
            else succ[succ_off[T] + atomicAdd(&cursor[T], 1u)] = P;
            D |= kind_witnesses(kp);
        }
        else if (D & bit)
            D |= kind_witnesses(kp);
    }
    if (PASS == 0 && npred) atomicAdd(&indeg[T], npred);
}

// direct deps (Commands.updateWaitingOn keeps only those executing earlier, Commands.java:700-775)
template <int PASS>
__global__ void k_direct(LevelsIn g, const uint32_t* __restrict__ rank, uint32_t* __restrict__ indeg,
                         uint32_t* __restrict__ outdeg, const uint64_t* __restrict__ succ_off,
                         uint32_t* __restrict__ cursor, uint32_t* __restrict__ succ, LevelsCtl* ctl)
{
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= g.n) return;
    const uint32_t T = rank[t];
    uint32_t npred = 0;
    for (uint64_t d = g.dep_off[t]; d < g.dep_off[t + 1]; ++d)
    {
        const uint32_t src = g.deps[d];
        if (src >= g.n)
        {
            atomicCAS(&ctl->error, 0u, (unsigned)(-AD_E_INVAL));
            return;
        }
        const uint32_t P = rank[src];
        if (P >= T) continue;
        ++npred;
        if (PASS == 0) { if (outdeg) atomicAdd(&outdeg[P], 1u); }
        else if (PASS == 1) succ[succ_off[P] + atomicAdd(&cursor[P], 1u)] = T;
        else succ[succ_off[T] + atomicAdd(&cursor[T], 1u)] = P;
    }
    if (PASS == 0 && npred) atomicAdd(&indeg[T], npred);
}

// ---------------------------------------------------------------------------------------------
// Packed path (the default when the fields fit one u64):
//   exec word  = hi | lo | node bits that vary over the batch (pext, order kept) << rb | txn index
//   occurrence = key bits that vary << (rb + 3 + jb) | exec rank << (3 + jb) | kind (clamped to 7)
//                << jb | index of the key in the txn's key list
// Both are sorted keys-only, on the varying field alone: the exec words by their Timestamp bits,
// the occurrences (generated in rank order) stably by key. One walk over the sorted occurrences
// writes every occurrence's sparsified predecessors into the txn-major record of that occurrence
// (PredRec at occ_off[rank] + j: up to three inline, more in an overflow pool), so a txn's
// predecessors sit in its own consecutive records -- no in-degree pass, no atomics per edge.
// ---------------------------------------------------------------------------------------------
struct PackCfg {
    uint64_t m_node, m_lo, m_hi, m_key;     // varying bits
    uint32_t rb, jb;                        // rank bits, key-list index bits
    uint32_t s_lo, s_hi;                    // exec word: shifts of the lo and hi fields
    uint32_t ks;                            // occurrence: shift of the key field
    uint32_t kuni;                          // every txn has kuni keys (occ_off[r] = r * kuni), else 0
};

// A predecessor record (uint4 rec[o], uint4 rec2[o]): x = count (0..7), y/z/w the first three, rec2's
// x..w the next four; or x = REC_OVF, y = pool offset, z = count for more than REC_INLINE.
constexpr uint32_t REC_OVF = 0x80000000u;
constexpr uint32_t REC_INLINE = 7;

__global__ __launch_bounds__(256) void k_exec_pack(LevelsIn g, PackCfg p, uint64_t* __restrict__ out)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= g.n) return;
    const NormTid x = norm_tid(g.exec_msb[i], g.exec_lsb[i], g.exec_node[i]);
    const uint64_t node = (uint64_t)((uint32_t)x.node ^ 0x80000000u);
    out[i] = (pext64(x.hi, p.m_hi) << p.s_hi) | (pext64(x.lo, p.m_lo) << p.s_lo) | (pext64(node, p.m_node) << p.rb) | i;
}

// order[r] = txn of exec rank r, rank[t] = r, key count by rank; equal Timestamps are adjacent ->
// AD_E_DUP_EXEC (CommandsForKey.java:1439)
__global__ void k_exec_rank_p(LevelsIn g, const uint64_t* __restrict__ sorted, uint32_t rb, uint32_t* __restrict__ order,
                              uint32_t* __restrict__ rank, uint32_t* __restrict__ kcnt_r, LevelsCtl* ctl)
{
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= g.n) return;
    const uint64_t e = sorted[r];
    const uint32_t t = (uint32_t)(e & ((1ull << rb) - 1));
    order[r] = t;
    rank[t] = (uint32_t)r;
    kcnt_r[r] = (uint32_t)(g.key_off[t + 1] - g.key_off[t]);
    if (r > 0 && (sorted[r - 1] >> rb) == (e >> rb)) atomicCAS(&ctl->error, 0u, (unsigned)(-AD_E_DUP_EXEC));
}

__global__ __launch_bounds__(256) void k_occ_pack(LevelsIn g, PackCfg p, const uint32_t* __restrict__ order,
                                                  const uint64_t* __restrict__ occ_off, uint64_t* __restrict__ out,
                                                  uint64_t n_occ)
{
    if (p.kuni)
    {
        // thread per occurrence: consecutive threads read one txn's keys and write consecutive words
        for (uint64_t o = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; o < n_occ; o += (uint64_t)gridDim.x * blockDim.x)
        {
            const uint64_t r = o / p.kuni, j = o - r * p.kuni;
            const uint32_t t = order[r];
            const uint32_t kd = g.kind[t];
            out[o] = (pext64((uint64_t)g.keys[(uint64_t)t * p.kuni + j], p.m_key) << p.ks) | (r << (3 + p.jb)) |
                     ((uint64_t)(kd < 7u ? kd : 7u) << p.jb) | j;
        }
        return;
    }
    for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < g.n; r += (uint64_t)gridDim.x * blockDim.x)
    {
        const uint32_t t = order[r];
        const uint64_t s = g.key_off[t], e = g.key_off[t + 1], o = occ_off[r];
        const uint32_t kd = g.kind[t];
        const uint64_t w = (r << (3 + p.jb)) | ((uint64_t)(kd < 7u ? kd : 7u) << p.jb);
        for (uint64_t j = s; j < e; ++j)
            out[o + (j - s)] = (pext64((uint64_t)g.keys[j], p.m_key) << p.ks) | w | (j - s);
    }
}

// walk the chain back from occurrence p (sorted by key, then rank) as k_chain does: the first seven
// predecessors to P[0..6], every one to dst[i] when dst is given
__device__ __forceinline__ uint32_t walk_preds(const uint64_t* __restrict__ occ, uint64_t p, uint64_t e, PackCfg c,
                                               uint32_t rmask, uint32_t (&P)[REC_INLINE], uint32_t* __restrict__ dst)
{
    const uint64_t key = e >> c.ks;
    const uint32_t A = kind_witnesses((uint32_t)(e >> c.jb) & 7u);
    uint32_t D = 0, np = 0;
    uint64_t q = p;
    bool go = A != 0 && q > 0;
    while (go)
    {
        // four occurrences per step: most walks end within them
        uint64_t w[4];
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) w[k] = q > k ? occ[q - 1 - k] : 0ull;
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k)
        {
            if (!go) continue;
            if (q <= k || (w[k] >> c.ks) != key)
            {
                go = false;
                continue;
            }
            const uint32_t kp = (uint32_t)(w[k] >> c.jb) & 7u;
            const uint32_t bit = 1u << kp;
            if (A & bit & ~D)
            {
                const uint32_t v = (uint32_t)(w[k] >> (3 + c.jb)) & rmask;
                if (dst) dst[np] = v;
                else
                {
#pragma unroll
                    for (uint32_t z = 0; z < REC_INLINE; ++z)
                        if (np == z) P[z] = v;
                }
                ++np;
                D |= kind_witnesses(kp);
            }
            else if (D & bit)
                D |= kind_witnesses(kp);
            if ((A & ~D) == 0) go = false;
        }
        q = q > 4 ? q - 4 : 0;
        if (q == 0) go = false;
    }
    return np;
}

// Counters written by many blocks are sharded (NSHARD words each, block b on shard b % NSHARD): one
// device-scope atomic per block or wave then meets few others on its address.
constexpr uint32_t NSHARD = 256;
struct PackCnt {
    unsigned long long edges[NSHARD];      // key-chain + direct predecessors
    unsigned long long pool[NSHARD];       // overflow words taken from each pool shard
};

// wave-wide exclusive prefix of v and the total (lane 63's inclusive)
__device__ __forceinline__ uint32_t wave_excl(uint32_t v, uint32_t* total)
{
    const uint32_t inc = wave_incl_scan(v);
    *total = (uint32_t)__shfl(inc, 63, 64);
    return inc - v;
}

__device__ __forceinline__ void block_sum_to(unsigned long long* dst, uint64_t v, uint64_t* red /* LDS [4] */)
{
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    if (lane_id() == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0)
    {
        const uint64_t x = red[0] + red[1] + red[2] + red[3];
        if (x) atomicAdd(dst, (unsigned long long)x);
    }
    __syncthreads();
}

// Occurrence p's predecessors -> its record rec[occ_off[T] + j]: up to three inline, more in the
// pool shard of the block (one atomic per wave; a shard that runs out is reported by its count and
// the host repeats the run with larger shards)
__global__ __launch_bounds__(256) void k_walk(const uint64_t* __restrict__ occ, uint64_t n_occ, PackCfg c,
                                              const uint64_t* __restrict__ occ_off, uint4* __restrict__ rec,
                                              uint4* __restrict__ rec2, uint32_t* __restrict__ pool, uint64_t shard_cap,
                                              PackCnt* cnt)
{
    __shared__ uint64_t red[4];
    const uint32_t shard = blockIdx.x % NSHARD;
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t rmask = (uint32_t)((1ull << c.rb) - 1);
    uint64_t e = 0;
    uint32_t P[REC_INLINE] = {0, 0, 0, 0, 0, 0, 0}, np = 0;
    if (p < n_occ)
    {
        e = occ[p];
        np = walk_preds(occ, p, e, c, rmask, P, nullptr);
    }
    // overflow words: one allocation per wave
    const uint32_t want = np > REC_INLINE ? np : 0u;
    uint32_t wtot = 0;
    const uint32_t wpre = wave_excl(want, &wtot);
    uint64_t base = 0;
    if (wtot)
    {
        if (lane_id() == 0) base = atomicAdd(&cnt->pool[shard], (unsigned long long)wtot);
        base = __shfl(base, 0, 64);
    }
    if (p < n_occ)
    {
        const uint32_t T = (uint32_t)(e >> (3 + c.jb)) & rmask;
        const uint32_t j = (uint32_t)(e & ((1ull << c.jb) - 1));
        const uint64_t o = (c.kuni ? (uint64_t)T * c.kuni : occ_off[T]) + j;
        if (np <= REC_INLINE)
        {
            rec[o] = make_uint4(np, P[0], P[1], P[2]);
            if (np > 3) rec2[o] = make_uint4(P[3], P[4], P[5], P[6]);
        }
        else
        {
            const uint64_t at = base + wpre;
            if (at + np <= shard_cap) walk_preds(occ, p, e, c, rmask, P, pool + shard * shard_cap + at);
            rec[o] = make_uint4(REC_OVF, (uint32_t)(shard * shard_cap + std::min<uint64_t>(at, shard_cap)), np, 0);
        }
    }
    block_sum_to(&cnt->edges[shard], np, red);
}

// direct deps: index check, the count of those executing earlier (Commands.java:700-775), and per
// exec rank T (dirp zeroed before): P + 1 when exactly one direct dep executes earlier (rank P),
// DIRP_MANY | txn when more do (the level kernel then reads them itself), 0 when none does
constexpr uint32_t DIRP_MANY = 0x80000000u;
__global__ __launch_bounds__(256) void k_direct_check(LevelsIn g, const uint32_t* __restrict__ rank,
                                                      uint32_t* __restrict__ dirp, PackCnt* cnt, LevelsCtl* ctl)
{
    __shared__ uint64_t red[4];
    uint64_t ne = 0;
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < g.n; t += (uint64_t)gridDim.x * blockDim.x)
    {
        const uint64_t d0 = g.dep_off[t], d1 = g.dep_off[t + 1];
        if (d0 == d1) continue;
        const uint32_t T = rank[t];
        uint32_t np = 0, first = 0;
        for (uint64_t d = d0; d < d1; ++d)
        {
            const uint32_t src = g.deps[d];
            if (src >= g.n)
            {
                atomicCAS(&ctl->error, 0u, (unsigned)(-AD_E_INVAL));
                np = 0;
                break;
            }
            const uint32_t P = rank[src];
            if (P < T)
            {
                if (np == 0) first = P;
                ++np;
            }
        }
        if (np) dirp[T] = np == 1 ? first + 1u : (DIRP_MANY | (uint32_t)t);
        ne += np;
    }
    block_sum_to(&cnt->edges[blockIdx.x % NSHARD], ne, red);
}

__device__ __forceinline__ void wave_append(uint32_t* __restrict__ front, uint32_t* cnt, bool take, uint32_t v)
{
    const uint64_t m = ballot(take);
    if (!m) return;
    uint32_t base = 0;
    const uint32_t leader = __ffsll((unsigned long long)m) - 1;
    if (lane_id() == leader) base = atomicAdd(cnt, (uint32_t)__popcll(m));
    base = __shfl(base, leader, 64);
    if (take) front[base + mbcnt(m)] = v;
}

__global__ void k_frontier_init(const uint32_t* __restrict__ indeg, uint64_t n, uint32_t* __restrict__ level,
                                uint32_t* __restrict__ front, uint32_t* cnt)
{
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool take = r < n && indeg[r] == 0;
    if (take) level[r] = 0;
    wave_append(front, cnt, take, (uint32_t)r);
}

// one level: every txn of frontier L releases its successors; those whose last predecessor this
// was form frontier L+1 (their longest path from a source is exactly L+1). Edge-parallel: a wave
// takes STEP_GROUP frontier txns and spreads their successor edges over its 64 lanes, so a txn
// with many successors costs rounds of 64 independent atomics, not a serial per-lane loop.
constexpr uint32_t STEP_GROUP = 16;

__global__ __launch_bounds__(256) void k_level_step(uint32_t L, const uint32_t* __restrict__ cnt,
                                                    const uint32_t* __restrict__ front_in, uint32_t* __restrict__ front_out,
                                                    uint32_t* cnt_out, const uint64_t* __restrict__ succ_off,
                                                    const uint32_t* __restrict__ succ, uint32_t* __restrict__ indeg,
                                                    uint32_t* __restrict__ level)
{
    const uint32_t F = cnt[L];
    if (F == 0) return;
    const uint32_t lane = lane_id();
    const uint32_t n_waves = gridDim.x * (blockDim.x >> 6);
    const uint32_t wid = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    for (uint32_t g0 = wid * STEP_GROUP; g0 < F; g0 += n_waves * STEP_GROUP)
    {
        // lanes j < STEP_GROUP: frontier txn g0 + j, its first edge and degree
        uint64_t e0 = 0;
        uint32_t deg = 0;
        if (lane < STEP_GROUP && g0 + lane < F)
        {
            const uint32_t u = front_in[g0 + lane];
            e0 = succ_off[u];
            deg = (uint32_t)(succ_off[u + 1] - e0);
        }
        uint32_t inc = deg;
#pragma unroll
        for (uint32_t d = 1; d < STEP_GROUP; d <<= 1)
        {
            const uint32_t t = __shfl_up(inc, d, 64);
            if (lane >= d) inc += t;
        }
        uint32_t incl[STEP_GROUP];
#pragma unroll
        for (uint32_t j = 0; j < STEP_GROUP; ++j) incl[j] = __shfl(inc, j, 64);
        const uint32_t total = incl[STEP_GROUP - 1];
        for (uint32_t x0 = 0; x0 < total; x0 += 64)
        {
            const uint32_t x = x0 + lane;
            bool take = false;
            uint32_t s = 0;
            uint32_t owner = 0;
#pragma unroll
            for (uint32_t j = 0; j < STEP_GROUP; ++j) owner += incl[j] <= x ? 1u : 0u;
            const uint64_t eo = __shfl(e0, owner & (STEP_GROUP - 1), 64);
            // shuffles by every lane (a lane outside the exec mask reads back 0)
            const uint32_t prev = __shfl(inc, (owner - 1) & (STEP_GROUP - 1), 64);
            const uint32_t before = owner == 0 ? 0u : prev;
            if (x < total)
            {
                s = succ[eo + (x - before)];
                take = atomicSub(&indeg[s], 1u) == 1u;
                if (take) level[s] = L + 1;
            }
            wave_append(front_out, cnt_out, take, s);
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Rank-ordered dataflow leveling. level[] (by exec rank) starts LV_UNSET. A wave takes the next 64
// ranks by ticket, so the lowest unfinished rank always belongs to a running wave and every wait is
// on a lower rank: a running wave (or a finished one) -- no deadlock whatever the dispatch order.
// Each lane takes its predecessor list in batches of PULL_BATCH: the indices stay in registers and
// every level of the batch is loaded at once; the unset ones are polled again after a sleep (one
// load each, no index reload), and a lane whose list is done publishes its level at
// once (lanes of the same wave may wait on it). The level word is its own flag (set once, from
// LV_UNSET to its value): agent-scope relaxed atomics, i.e. sc1 stores and sc1 loads, the
// single-granule hand-off of MI355X_MICROARCH.md (no payload to order). A wave still waiting after
// `budget` wall-clock ticks gives up and flags the run (the host reports AD_E_STATE).
// ---------------------------------------------------------------------------------------------
constexpr uint32_t LV_UNSET = 0xFFFFFFFFu;
constexpr uint32_t PULL_BATCH = 8;

__device__ __forceinline__ uint32_t lv_poll(const uint32_t* p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// (An XCD-local variant -- blocks off the first block's XCD leaving, levels stored sc0 and polled sc1 so a
// hand-off stays in one L2 -- measured 0.60 / 0.86 / 1.13 ms at 2 / 4 / 8 waves per CU of the owner XCD against
// 0.59 on all CUs; deleted in round 6.)
__global__ __launch_bounds__(256) void k_level_pull(uint64_t n, const uint64_t* __restrict__ pred_off,
                                                    const uint32_t* __restrict__ pred, uint32_t* level, uint32_t* ticket,
                                                    uint32_t* fail, uint64_t budget, uint32_t naps)
{
    const uint32_t lane = lane_id();
    const uint64_t t_end = wall_clock64() + budget;
    while (true)
    {
        uint32_t c = 0;
        if (lane == 0) c = atomicAdd(ticket, 1u);
        c = __shfl(c, 0, 64);
        if ((uint64_t)c * 64 >= n) return;
        const uint64_t T = (uint64_t)c * 64 + lane;
        const bool on = T < n;
        uint64_t j = on ? pred_off[T] : 0;
        const uint64_t e = on ? pred_off[T + 1] : 0;
        uint32_t mx = 0, pend = 0, nb = 0;
        uint32_t pi[PULL_BATCH];
        bool pending = on, fresh = true;
        while (true)
        {
            if (pending)
            {
                // a batch of up to PULL_BATCH predecessors: indices kept in registers, every level
                // loaded at once; only the unset ones (bits of pend) are polled again
                while (true)
                {
                    if (fresh)
                    {
                        nb = (uint32_t)std::min<uint64_t>(PULL_BATCH, e - j);
#pragma unroll
                        for (uint32_t k = 0; k < PULL_BATCH; ++k) pi[k] = k < nb ? pred[j + k] : 0u;
                        uint32_t v[PULL_BATCH];
#pragma unroll
                        for (uint32_t k = 0; k < PULL_BATCH; ++k) v[k] = k < nb ? lv_poll(level + pi[k]) : 0u;
                        pend = 0;
#pragma unroll
                        for (uint32_t k = 0; k < PULL_BATCH; ++k)
                            if (k < nb)
                            {
                                if (v[k] == LV_UNSET) pend |= 1u << k;
                                else mx = max(mx, v[k] + 1u);
                            }
                        fresh = false;
                    }
                    else if (pend)
                    {
                        uint32_t v[PULL_BATCH];
#pragma unroll
                        for (uint32_t k = 0; k < PULL_BATCH; ++k) v[k] = (pend >> k) & 1u ? lv_poll(level + pi[k]) : LV_UNSET;
#pragma unroll
                        for (uint32_t k = 0; k < PULL_BATCH; ++k)
                            if (((pend >> k) & 1u) && v[k] != LV_UNSET)
                            {
                                pend &= ~(1u << k);
                                mx = max(mx, v[k] + 1u);
                            }
                    }
                    if (pend) break;
                    j += nb;
                    if (j >= e)
                    {
                        __hip_atomic_store(level + T, mx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        pending = false;
                        break;
                    }
                    fresh = true;
                }
            }
            if (!ballot(pending)) break;
            if (wall_clock64() > t_end)
            {
                if (lane == 0) atomicOr(fail, 1u);
                return;
            }
            for (uint32_t z = 0; z < naps; ++z) __builtin_amdgcn_s_sleep(4);
        }
    }
}

// The same dataflow over the packed path's predecessor records: txn T's predecessors are the records
// [occ_off[T], occ_off[T+1]) (up to seven inline each, or an overflow run in the pool) and its direct
// deps executing earlier (dirp[T]). Every predecessor index is fetched before the first level poll, so
// a wait is only ever on levels: a txn with at most four keys and at most REC_SLOTS predecessors in all
// takes them in one batch, compacted into the slots; any other takes one record / overflow chunk /
// deps chunk per batch.
constexpr uint32_t REC_SLOTS = 16;

__device__ __forceinline__ uint32_t sel4(uint32_t i, uint32_t a, uint32_t b, uint32_t c, uint32_t d)
{
    return i == 0 ? a : (i == 1 ? b : (i == 2 ? c : d));
}

__global__ __launch_bounds__(256) void k_level_rec(LevelsIn g, const uint64_t* __restrict__ occ_off,
                                                   const uint4* __restrict__ rec, const uint4* __restrict__ rec2,
                                                   const uint32_t* __restrict__ pool, uint64_t pool_cap,
                                                   const uint32_t* __restrict__ dirp, const uint32_t* __restrict__ rank,
                                                   uint32_t* level, uint32_t* ticket, uint32_t* fail, uint64_t budget,
                                                   uint32_t naps, uint32_t kuni)
{
    const uint64_t n = g.n;
    const uint32_t lane = lane_id();
    const uint64_t t_end = wall_clock64() + budget;
    while (true)
    {
        uint32_t c = 0;
        if (lane == 0) c = atomicAdd(ticket, 1u);
        c = __shfl(c, 0, 64);
        if ((uint64_t)c * 64 >= n) return;
        const uint64_t T = (uint64_t)c * 64 + lane;
        const bool on = T < n;
        const uint64_t o0 = !on ? 0 : (kuni ? T * kuni : occ_off[T]);
        const uint64_t o1 = !on ? 0 : (kuni ? o0 + kuni : occ_off[T + 1]);
        const uint32_t dp = (on && dirp) ? dirp[T] : 0u;
        const uint32_t nk = (uint32_t)(o1 - o0);
        uint4 r4[4], q4[4];
#pragma unroll
        for (uint32_t i = 0; i < 4; ++i) r4[i] = i < nk ? rec[o0 + i] : make_uint4(0, 0, 0, 0);
#pragma unroll
        for (uint32_t i = 0; i < 4; ++i)
            q4[i] = (i < nk && r4[i].x > 3 && !(r4[i].x & REC_OVF)) ? rec2[o0 + i] : make_uint4(0, 0, 0, 0);
        // direct deps: one (its rank in dirp), or several (read here)
        uint64_t d0 = 0, d1 = 0;
        const bool dmany = (dp & DIRP_MANY) != 0;
        if (dmany)
        {
            d0 = g.dep_off[dp & ~DIRP_MANY];
            d1 = g.dep_off[(dp & ~DIRP_MANY) + 1];
        }
        const uint32_t nd = dmany ? (uint32_t)std::min<uint64_t>(d1 - d0, 0xFFFFull) : (dp ? 1u : 0u);
        uint32_t cn[4];
#pragma unroll
        for (uint32_t i = 0; i < 4; ++i)
        {
            const bool ovf = (r4[i].x & REC_OVF) != 0;
            cn[i] = ovf ? (r4[i].y + (uint64_t)r4[i].z <= pool_cap ? r4[i].z : 0u) : r4[i].x;
        }
        const uint32_t b1 = cn[0], b2 = b1 + cn[1], b3 = b2 + cn[2], tot = b3 + cn[3];
        uint32_t pi[REC_SLOTS];
        uint32_t vm = 0;
        // phase 0: the one-batch form (done when loaded); 1: a record per batch (s, pos); 2: several
        // direct deps (pos); 3: done
        uint32_t ph = 3, s = 0;
        uint64_t pos = 0;
        if (on && nk <= 4 && tot + nd <= REC_SLOTS)
        {
#pragma unroll
            for (uint32_t k = 0; k < REC_SLOTS; ++k)
            {
                uint32_t v = 0;
                bool valid = false;
                if (k < tot)
                {
                    const uint32_t i = (k >= b1 ? 1u : 0u) + (k >= b2 ? 1u : 0u) + (k >= b3 ? 1u : 0u);
                    const uint32_t q = k - sel4(i, 0u, b1, b2, b3);
                    const uint32_t x = sel4(i, r4[0].x, r4[1].x, r4[2].x, r4[3].x);
                    const uint32_t y = sel4(i, r4[0].y, r4[1].y, r4[2].y, r4[3].y);
                    if (x & REC_OVF) v = pool[(uint64_t)y + q];
                    else if (q == 0) v = y;
                    else if (q == 1) v = sel4(i, r4[0].z, r4[1].z, r4[2].z, r4[3].z);
                    else if (q == 2) v = sel4(i, r4[0].w, r4[1].w, r4[2].w, r4[3].w);
                    else if (q == 3) v = sel4(i, q4[0].x, q4[1].x, q4[2].x, q4[3].x);
                    else if (q == 4) v = sel4(i, q4[0].y, q4[1].y, q4[2].y, q4[3].y);
                    else if (q == 5) v = sel4(i, q4[0].z, q4[1].z, q4[2].z, q4[3].z);
                    else v = sel4(i, q4[0].w, q4[1].w, q4[2].w, q4[3].w);
                    valid = true;
                }
                else if (k < tot + nd)
                {
                    if (dmany)
                    {
                        const uint32_t src = g.deps[d0 + (k - tot)];
                        v = src < n ? rank[src] : 0xFFFFFFFFu;
                        valid = (uint64_t)v < T;
                    }
                    else
                    {
                        v = dp - 1u;
                        valid = true;
                    }
                }
                pi[k] = v;
                if (valid) vm |= 1u << k;
            }
        }
        else if (on)
            ph = 1;
        uint32_t mx = 0, pend = 0;
        const bool pending0 = on;
        bool pending = pending0, fresh = ph != 3;
        if (!fresh && on)
        {
            uint32_t v[REC_SLOTS];
#pragma unroll
            for (uint32_t k = 0; k < REC_SLOTS; ++k) v[k] = (vm >> k) & 1u ? lv_poll(level + pi[k]) : 0u;
#pragma unroll
            for (uint32_t k = 0; k < REC_SLOTS; ++k)
                if ((vm >> k) & 1u)
                {
                    if (v[k] == LV_UNSET) pend |= 1u << k;
                    else mx = max(mx, v[k] + 1u);
                }
        }
        while (true)
        {
            if (pending)
            {
                while (true)
                {
                    if (fresh)
                    {
                        vm = 0;
                        if (ph == 1)
                        {
                            if (s < nk)
                            {
                                const uint4 r = rec[o0 + s];
                                if (r.x & REC_OVF)
                                {
                                    const uint64_t cnt = r.z, at = r.y;
                                    const uint32_t m = (uint32_t)std::min<uint64_t>(REC_SLOTS, cnt - pos);
                                    const bool ok = at + cnt <= pool_cap;     // else the host repeats the run
#pragma unroll
                                    for (uint32_t k = 0; k < REC_SLOTS; ++k) pi[k] = (ok && k < m) ? pool[at + pos + k] : 0u;
                                    vm = ok ? (uint32_t)((1ull << m) - 1u) : 0u;
                                    pos += m;
                                    if (pos >= cnt)
                                    {
                                        ++s;
                                        pos = 0;
                                    }
                                }
                                else
                                {
                                    const uint4 q = r.x > 3 ? rec2[o0 + s] : make_uint4(0, 0, 0, 0);
                                    pi[0] = r.y;
                                    pi[1] = r.z;
                                    pi[2] = r.w;
                                    pi[3] = q.x;
                                    pi[4] = q.y;
                                    pi[5] = q.z;
                                    pi[6] = q.w;
                                    vm = (1u << r.x) - 1u;
                                    ++s;
                                }
                            }
                            else if (dp && !dmany)
                            {
                                pi[0] = dp - 1u;
                                vm = 1;
                                ph = 3;
                            }
                            else
                            {
                                ph = dmany && d0 < d1 ? 2 : 3;
                                pos = 0;
                            }
                        }
                        else if (ph == 2)
                        {
                            const uint32_t m = (uint32_t)std::min<uint64_t>(REC_SLOTS, d1 - d0 - pos);
#pragma unroll
                            for (uint32_t k = 0; k < REC_SLOTS; ++k)
                            {
                                const uint32_t src = k < m ? g.deps[d0 + pos + k] : 0xFFFFFFFFu;
                                const uint32_t P = src < n ? rank[src] : 0xFFFFFFFFu;
                                pi[k] = P;
                                if ((uint64_t)P < T) vm |= 1u << k;
                            }
                            pos += m;
                            if (d0 + pos >= d1) ph = 3;
                        }
                        uint32_t v[REC_SLOTS];
#pragma unroll
                        for (uint32_t k = 0; k < REC_SLOTS; ++k) v[k] = (vm >> k) & 1u ? lv_poll(level + pi[k]) : 0u;
                        pend = 0;
#pragma unroll
                        for (uint32_t k = 0; k < REC_SLOTS; ++k)
                            if ((vm >> k) & 1u)
                            {
                                if (v[k] == LV_UNSET) pend |= 1u << k;
                                else mx = max(mx, v[k] + 1u);
                            }
                        fresh = false;
                    }
                    else if (pend)
                    {
                        uint32_t v[REC_SLOTS];
#pragma unroll
                        for (uint32_t k = 0; k < REC_SLOTS; ++k) v[k] = (pend >> k) & 1u ? lv_poll(level + pi[k]) : LV_UNSET;
#pragma unroll
                        for (uint32_t k = 0; k < REC_SLOTS; ++k)
                            if (((pend >> k) & 1u) && v[k] != LV_UNSET)
                            {
                                pend &= ~(1u << k);
                                mx = max(mx, v[k] + 1u);
                            }
                    }
                    if (pend) break;
                    if (ph == 3)
                    {
                        __hip_atomic_store(level + T, mx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        pending = false;
                        break;
                    }
                    fresh = true;
                }
            }
            if (!ballot(pending)) break;
            if (wall_clock64() > t_end)
            {
                if (lane == 0) atomicOr(fail, 1u);
                return;
            }
            for (uint32_t z = 0; z < naps; ++z) __builtin_amdgcn_s_sleep(4);
        }
    }
}

__global__ void k_level_max(const uint32_t* __restrict__ level, uint64_t n, uint32_t* out_max)
{
    uint32_t v = 0;
    for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (uint64_t)gridDim.x * blockDim.x)
        v = max(v, level[r]);
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v = max(v, (uint32_t)__shfl_xor(v, d, 64));
    if (lane_id() == 0) atomicMax(out_max, v);
}

__global__ void k_level_out(const uint32_t* __restrict__ order, const uint32_t* __restrict__ level_r, uint64_t n,
                            uint32_t* __restrict__ out)
{
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r < n) out[order[r]] = level_r[r];
}

// ---------------------------------------------------------------------------------------------
// host driver
// ---------------------------------------------------------------------------------------------
using DBuf = DevBuf;

struct LevelsWork {
    DBuf ka, kb, va, vb, hist, off, bsum, ord, rank, kcnt, occ_off, indeg, outdeg, succ_off, cursor, succ,
        level, front0, front1, cnt, ctl, rec, rec2, pool, pcnt, dirp, wpart;
    LevelsCtl* h_ctl = nullptr;         // pinned
    struct PackCnt* h_pcnt = nullptr;   // pinned
    uint64_t* h_u64 = nullptr;          // pinned, 4 words
    hipEvent_t ev[3] = {};
    ~LevelsWork()
    {
        if (h_ctl) (void)hipHostFree(h_ctl);
        if (h_pcnt) (void)hipHostFree(h_pcnt);
        if (h_u64) (void)hipHostFree(h_u64);
        for (auto& e : ev)
            if (e) (void)hipEventDestroy(e);
    }
};

LevelsWork* levels_work_create() { return new LevelsWork(); }
void levels_work_destroy(LevelsWork* w) { delete w; }

constexpr uint32_t STEP_CHUNK = 32;     // frontier launches between host checks
constexpr unsigned STEP_BLOCKS = 64;

#define LV_CHK(expr)                                                                     \
    do {                                                                                 \
        hipError_t _e = (expr);                                                          \
        if (_e != hipSuccess)                                                            \
        {                                                                                \
            *err = std::string(#expr) + ": " + hipGetErrorString(_e);                    \
            return AD_E_DEVICE;                                                          \
        }                                                                                \
    } while (0)
#define LV_ALLOC(buf, bytes)                                                             \
    do {                                                                                 \
        if (!(buf).ensure(bytes))                                                        \
        {                                                                                \
            *err = "hipMalloc failed (" #buf ")";                                        \
            return AD_E_NOMEM;                                                           \
        }                                                                                \
    } while (0)

static unsigned blocks_for(uint64_t n, unsigned t) { return (unsigned)std::max<uint64_t>(1, (n + t - 1) / t); }

// leveling launch of the rank-ordered dataflow
struct PullCfg {
    unsigned grid, threads;
    uint32_t naps;
    uint64_t budget;
};

static PullCfg pull_cfg(uint64_t n, bool packed)
{
    int dev = 0, cus = 256, khz = 100000;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev);
    // measured on config 5 (scripts/c5_sweep.sh, c5_packed.sh): the CSR kernel at one wave per CU
    // (0.59 ms; a 256-thread block per CU or 2 / 4 blocks were slower in round 4: the polls of more
    // resident waiters load the memory system the hand-offs go through); the record kernel, whose
    // per-task setup is longer, at four waves per CU (0.60 ms; 1.00 / 0.62 at one / two)
    PullCfg c;
    int per_cu = packed ? 4 : 1, threads = 64;
    // tests vary the residency (every wave count must give the same levels)
    if (const char* e = getenv("AD_LEVELS_PULL_PER_CU")) per_cu = std::max(1, std::min(8, atoi(e)));
    if (const char* e = getenv("AD_LEVELS_PULL_THREADS")) threads = atoi(e) == 64 ? 64 : (atoi(e) == 128 ? 128 : 256);
    c.threads = (unsigned)threads;
    c.naps = 1;
    c.budget = (uint64_t)std::max(khz, 1000) * 1000ull;       // one second of wall clock
    const uint64_t tasks = (n + threads - 1) / threads;
    c.grid = std::max(1u, (unsigned)std::min<uint64_t>((uint64_t)cus * per_cu, tasks));
    return c;
}

struct PackPlan {
    bool ok = false;
    PackCfg cfg{};
    uint32_t exec_bits = 0, key_bits = 0;
};

static uint32_t bit_len(uint64_t v) { return v ? 64u - (uint32_t)__builtin_clzll(v) : 0u; }

// the packed path applies when both packed words fit 64 bits (and not under AD_LEVELS_FRONTIER /
// AD_LEVELS_PACKED=0)
static PackPlan pack_plan(const LevelsCtl& h, uint64_t n, uint64_t n_occ)
{
    PackPlan p;
    if (getenv("AD_LEVELS_FRONTIER")) return p;
    if (const char* e = getenv("AD_LEVELS_PACKED"))
        if (atoi(e) == 0) return p;
    if (n >= (1ull << 31) || n_occ >= (1ull << 32)) return p;     // dirp: rank + 1 or DIRP_MANY | txn
    PackCfg& c = p.cfg;
    c.m_node = h.diff[0] & 0xFFFFFFFFull;
    c.m_lo = h.diff[1];
    c.m_hi = h.diff[2];
    c.m_key = h.diff[3];
    c.rb = std::max(1u, bit_len(n - 1));
    c.jb = h.maxk > 1 ? bit_len(h.maxk - 1) : 0u;
    const uint32_t b0 = (uint32_t)__builtin_popcountll(c.m_node), b1 = (uint32_t)__builtin_popcountll(c.m_lo),
                   b2 = (uint32_t)__builtin_popcountll(c.m_hi), bk = (uint32_t)__builtin_popcountll(c.m_key);
    if (c.rb + b0 + b1 + b2 > 64 || bk + c.rb + 3 + c.jb > 64) return p;
    c.kuni = h.maxk == ~h.mink_inv ? h.maxk : 0u;
    c.s_lo = c.rb + b0;
    c.s_hi = c.s_lo + b1;
    c.ks = c.rb + 3 + c.jb;
    p.exec_bits = b0 + b1 + b2;
    p.key_bits = bk;
    p.ok = true;
    return p;
}

static int run_levels_packed(LevelsWork* w, const LevelsIn& g, const PackPlan& pp, uint64_t n_occ, uint32_t* level_out,
                             hipStream_t st, LevelsOut* out, std::string* err);

int run_levels(LevelsWork* w, const LevelsIn& g, uint32_t* level_out, hipStream_t st, LevelsOut* out, std::string* err)
{
    *out = LevelsOut{};
    const uint64_t n = g.n;
    if (n == 0) return AD_OK;
    if (n >= (1ull << OCC_KIND_SHIFT) - 64)
    {
        *err = "ad_levels: too many txns (ranks below 2^29)";
        return AD_E_CAPACITY;
    }
    if (!w->h_ctl) LV_CHK(hipHostMalloc((void**)&w->h_ctl, sizeof(LevelsCtl), hipHostMallocDefault));
    if (!w->h_u64) LV_CHK(hipHostMalloc((void**)&w->h_u64, 4 * sizeof(uint64_t), hipHostMallocDefault));
    for (auto& e : w->ev)
        if (!e) LV_CHK(timing_event(&e));

    // one round trip: the occurrence count (key_off[n]; key_off[0] must be 0) and the exec words' diffs,
    // key diff and key-count range (k_exec_words reads key_off[n] itself)
    LV_ALLOC(w->ctl, sizeof(LevelsCtl));
    LV_ALLOC(w->wpart, sizeof(WordsPart) * RED_BLOCKS);
    LV_ALLOC(w->cnt, 4 * (n + 2 + STEP_CHUNK));
    LevelsCtl* ctl = w->ctl.as<LevelsCtl>();
    uint32_t* cnt = w->cnt.as<uint32_t>();
    LV_CHK(hipEventRecord(w->ev[0], st));
    LV_CHK(hipMemsetAsync(ctl, 0, sizeof(LevelsCtl), st));
    LV_CHK(hipMemsetAsync(cnt, 0, 4 * (n + 2 + STEP_CHUNK), st));
    const unsigned wb = std::min(blocks_for(n, 64), RED_BLOCKS);
    k_exec_words<<<wb, 256, 0, st>>>(g, nullptr, nullptr, w->wpart.as<WordsPart>());
    k_exec_words_reduce<<<1, 256, 0, st>>>(w->wpart.as<WordsPart>(), wb, ctl);
    LV_CHK(d2h(&w->h_u64[0], g.key_off, 8, st));
    LV_CHK(d2h(&w->h_u64[1], g.key_off + n, 8, st));
    LV_CHK(d2h(w->h_ctl, ctl, sizeof(LevelsCtl), st));
    LV_CHK(hipStreamSynchronize(st));
    if (w->h_u64[0] != 0 || w->h_u64[1] > (1ull << 40))
    {
        *err = "ad_levels: key_off must start at 0";
        return AD_E_INVAL;
    }
    const uint64_t n_occ = w->h_u64[1];
    out->n_occ = n_occ;
    const uint64_t cap = std::max(n, n_occ);
    const uint64_t hist_n = radix_hist_entries(cap);
    LV_ALLOC(w->ka, 8 * cap);
    LV_ALLOC(w->kb, 8 * cap);
    LV_ALLOC(w->va, 4 * cap);
    LV_ALLOC(w->vb, 4 * cap);
    LV_ALLOC(w->hist, 4 * hist_n);
    LV_ALLOC(w->off, 8 * (hist_n + 1));
    LV_ALLOC(w->bsum, 8 * (std::max(hist_n, n) / 1024 + 2));
    LV_ALLOC(w->ord, 4 * n);
    LV_ALLOC(w->rank, 4 * n);
    LV_ALLOC(w->kcnt, 4 * n);
    LV_ALLOC(w->occ_off, 8 * (n + 1));
    LV_ALLOC(w->level, 4 * n);
    {
        const PackPlan pp = pack_plan(*w->h_ctl, n, n_occ);
        if (pp.ok) return run_levels_packed(w, g, pp, n_occ, level_out, st, out, err);
    }
    // the CSR path: its buffers, and the exec words (node word + index) its first sort starts from
    LV_ALLOC(w->indeg, 4 * n);
    LV_ALLOC(w->outdeg, 4 * n);
    LV_ALLOC(w->cursor, 4 * n);
    LV_ALLOC(w->succ_off, 8 * (n + 1));
    LV_ALLOC(w->front0, 4 * n);
    LV_ALLOC(w->front1, 4 * n);
    uint64_t* ka = w->ka.as<uint64_t>();
    uint64_t* kb = w->kb.as<uint64_t>();
    uint32_t* va = w->va.as<uint32_t>();
    uint32_t* vb = w->vb.as<uint32_t>();
    uint32_t* hist = w->hist.as<uint32_t>();
    uint64_t* off = w->off.as<uint64_t>();
    uint64_t* bsum = w->bsum.as<uint64_t>();
    uint32_t* order = w->ord.as<uint32_t>();
    uint32_t* indeg = w->indeg.as<uint32_t>();
    uint32_t* outdeg = w->outdeg.as<uint32_t>();
    uint32_t* cursor = w->cursor.as<uint32_t>();
    uint64_t* succ_off = w->succ_off.as<uint64_t>();
    uint32_t* level = w->level.as<uint32_t>();
    k_exec_words<<<wb, 256, 0, st>>>(g, ka, va, w->wpart.as<WordsPart>());
    LV_CHK(hipMemsetAsync(indeg, 0, 4 * n, st));
    LV_CHK(hipMemsetAsync(outdeg, 0, 4 * n, st));
    LV_CHK(hipMemsetAsync(cursor, 0, 4 * n, st));
    const uint64_t dx[3] = {w->h_ctl->diff[0], w->h_ctl->diff[1], w->h_ctl->diff[2]};
    uint64_t* kcur = ka;
    uint32_t* vcur = va;
    for (int word = 0; word < 3; ++word)
    {
        const uint32_t dm = digits_of(dx[word]);
        if (!dm) continue;
        if (word > 0) k_exec_gather<<<blocks_for(n, 256), 256, 0, st>>>(g, vcur, word, kcur);
        LV_CHK(radix_sort_pairs(kcur, vcur, kcur == ka ? kb : ka, vcur == va ? vb : va, n, dm, hist, off, bsum, st,
                                &kcur, &vcur));
    }
    LV_CHK(hipMemcpyAsync(order, vcur, 4 * n, hipMemcpyDeviceToDevice, st));
    k_exec_rank<<<blocks_for(n, 256), 256, 0, st>>>(g, order, w->rank.as<uint32_t>(), w->kcnt.as<uint32_t>(), ctl);
    LV_CHK(run_scan_arrays(w->kcnt.as<uint32_t>(), w->occ_off.as<uint64_t>(), n, 1, bsum, st));

    // leveling scheme: the dataflow over a predecessor CSR (default) or the frontier loop (AD_LEVELS_FRONTIER)
    const bool pull = getenv("AD_LEVELS_FRONTIER") == nullptr;

    // ---- 2. key chains: occurrences in rank order, stably sorted by key
    uint64_t* okey = ka;
    uint32_t* oval = va;
    if (n_occ)
    {
        k_occ_fill<<<std::min(blocks_for(n, 256), RED_BLOCKS), 256, 0, st>>>(g, order, w->occ_off.as<uint64_t>(), okey, oval, ctl);
        LV_CHK(d2h(w->h_ctl, ctl, sizeof(LevelsCtl), st));
        LV_CHK(hipStreamSynchronize(st));
        LV_CHK(radix_sort_pairs(okey, oval, kb, vb, n_occ, digits_of(w->h_ctl->diff[3]), hist, off, bsum, st, &okey,
                                &oval));
    }

    // ---- 3. sparsified predecessors -> predecessor CSR (pull) or successor CSR + in-degrees (frontier)
    if (n_occ)
        k_chain<0><<<blocks_for(n_occ, 256), 256, 0, st>>>(okey, oval, n_occ, indeg,
                                                           pull ? nullptr : outdeg, nullptr, nullptr, nullptr);
    if (g.dep_off)
        k_direct<0><<<blocks_for(n, 256), 256, 0, st>>>(g, w->rank.as<uint32_t>(), indeg, pull ? nullptr : outdeg, nullptr,
                                                        nullptr, nullptr, ctl);
    LV_CHK(run_scan_arrays(pull ? indeg : outdeg, succ_off, n, 1, bsum, st));
    LV_CHK(d2h(&w->h_u64[2], succ_off + n, 8, st));
    LV_CHK(d2h(w->h_ctl, ctl, sizeof(LevelsCtl), st));
    LV_CHK(hipStreamSynchronize(st));
    if (w->h_ctl->error)
    {
        const int code = -(int)w->h_ctl->error;
        *err = code == AD_E_DUP_EXEC ? "ad_levels: two txns with the same executeAt (CommandsForKey.java:1439)"
                                     : "ad_levels: direct dep index out of range";
        return code;
    }
    const uint64_t n_edges = w->h_u64[2];
    out->n_edges = n_edges;
    LV_ALLOC(w->succ, 4 * std::max<uint64_t>(n_edges, 1));
    uint32_t* succ = w->succ.as<uint32_t>();     // pull: predecessor lists (offsets succ_off)
    if (pull)
    {
        if (n_occ)
            k_chain<2><<<blocks_for(n_occ, 256), 256, 0, st>>>(okey, oval, n_occ, nullptr, nullptr,
                                                               succ_off, cursor, succ);
        if (g.dep_off)
            k_direct<2><<<blocks_for(n, 256), 256, 0, st>>>(g, w->rank.as<uint32_t>(), nullptr, nullptr, succ_off, cursor,
                                                            succ, ctl);
    }
    else
    {
        if (n_occ)
            k_chain<1><<<blocks_for(n_occ, 256), 256, 0, st>>>(okey, oval, n_occ, nullptr, nullptr,
                                                               succ_off, cursor, succ);
        if (g.dep_off)
            k_direct<1><<<blocks_for(n, 256), 256, 0, st>>>(g, w->rank.as<uint32_t>(), nullptr, nullptr, succ_off, cursor,
                                                            succ, ctl);
    }
    LV_CHK(hipEventRecord(w->ev[1], st));

    // ---- 4. level the DAG: rank-ordered dataflow (default) or the level-synchronous frontier loop
    // (AD_LEVELS_FRONTIER)
    uint64_t nl = 0;
    if (pull)
    {
        const PullCfg pc = pull_cfg(n, false);
        LV_CHK(hipMemsetAsync(level, 0xFF, 4 * n, st));
        k_level_pull<<<pc.grid, pc.threads, 0, st>>>(n, succ_off, succ, level, cnt, cnt + 1, pc.budget, pc.naps);
        LV_CHK(hipGetLastError());
        out->n_launch = 1;
        k_level_max<<<256, 256, 0, st>>>(level, n, cnt + 2);
        k_level_out<<<blocks_for(n, 256), 256, 0, st>>>(order, level, n, level_out);
        LV_CHK(hipEventRecord(w->ev[2], st));
        uint32_t tail[3];
        LV_CHK(d2h(tail, cnt, sizeof(tail), st));
        LV_CHK(hipStreamSynchronize(st));
        if (tail[1])
        {
            *err = "ad_levels: a wave waited more than a second for a predecessor's level";
            return AD_E_STATE;
        }
        nl = (uint64_t)tail[2] + 1;
    }
    else
    {
        uint32_t* fr[2] = {w->front0.as<uint32_t>(), w->front1.as<uint32_t>()};
        k_frontier_init<<<blocks_for(n, 256), 256, 0, st>>>(indeg, n, level, fr[0], cnt);
        uint32_t L = 0;
        while (true)
        {
            for (uint32_t c = 0; c < STEP_CHUNK; ++c, ++L)
                k_level_step<<<STEP_BLOCKS, 256, 0, st>>>(L, cnt, fr[L & 1], fr[(L + 1) & 1], cnt + L + 1, succ_off, succ,
                                                          indeg, level);
            out->n_launch += STEP_CHUNK;
            LV_CHK(hipGetLastError());
            LV_CHK(d2h(&w->h_u64[3], cnt + L, 4, st));
            LV_CHK(hipStreamSynchronize(st));
            if ((uint32_t)w->h_u64[3] == 0) break;
            if (L >= n + 1)
            {
                *err = "ad_levels: frontier did not drain";
                return AD_E_STATE;
            }
        }
        k_level_out<<<blocks_for(n, 256), 256, 0, st>>>(order, level, n, level_out);
        LV_CHK(hipEventRecord(w->ev[2], st));
        // levels = frontiers before the first empty one; every txn must have been levelled
        std::vector<uint32_t> counts(L + 1);
        LV_CHK(d2h(counts.data(), cnt, 4 * (L + 1), st));
        LV_CHK(hipStreamSynchronize(st));
        uint64_t total = 0;
        for (uint32_t i = 0; i <= L && counts[i]; ++i)
        {
            total += counts[i];
            nl = i + 1;
        }
        if (total != n)
        {
            *err = "ad_levels: " + std::to_string(n - total) + " txns never became ready";
            return AD_E_STATE;
        }
    }
    out->n_levels = nl;
    float a = 0, b = 0;
    (void)hipEventElapsedTime(&a, w->ev[0], w->ev[1]);
    (void)hipEventElapsedTime(&b, w->ev[1], w->ev[2]);
    out->ms_build = a;
    out->ms_frontier = b;
    out->ms_total = a + b;
    return AD_OK;
}

static int run_levels_packed(LevelsWork* w, const LevelsIn& g, const PackPlan& pp, uint64_t n_occ, uint32_t* level_out,
                             hipStream_t st, LevelsOut* out, std::string* err)
{
    const uint64_t n = g.n;
    const PackCfg& c = pp.cfg;
    const uint64_t cap = std::max(n, n_occ);
    const uint64_t hist_n = std::max(radix_hist_entries(cap), radix_keys_hist_entries(cap));
    LV_ALLOC(w->hist, 4 * hist_n);
    LV_ALLOC(w->off, 8 * (hist_n + 1));
    LV_ALLOC(w->bsum, 8 * (std::max(hist_n, n) / 1024 + 2));
    LV_ALLOC(w->rec, 16 * std::max<uint64_t>(n_occ, 1));
    LV_ALLOC(w->rec2, 16 * std::max<uint64_t>(n_occ, 1));
    LV_ALLOC(w->pcnt, sizeof(PackCnt));
    if (g.dep_off) LV_ALLOC(w->dirp, 4 * n);
    if (!w->h_pcnt) LV_CHK(hipHostMalloc((void**)&w->h_pcnt, sizeof(PackCnt), hipHostMallocDefault));
    // overflow pool: NSHARD shards; grown to what a run asked for when that run did not fit (it is then
    // repeated)
    uint64_t shard_cap = std::max<uint64_t>(w->pool.cap / 4 / NSHARD, std::max<uint64_t>(n_occ / 8 / NSHARD, 64));
    if (shard_cap * NSHARD >= (1ull << 32))
    {
        *err = "ad_levels: predecessor pool beyond 2^32 words";
        return AD_E_CAPACITY;
    }
    LV_ALLOC(w->pool, 4 * shard_cap * NSHARD);
    LevelsCtl* ctl = w->ctl.as<LevelsCtl>();
    PackCnt* pcnt = w->pcnt.as<PackCnt>();
    uint32_t* dirp = g.dep_off ? w->dirp.as<uint32_t>() : nullptr;
    uint64_t* ka = w->ka.as<uint64_t>();
    uint64_t* kb = w->kb.as<uint64_t>();
    uint32_t* hist = w->hist.as<uint32_t>();
    uint64_t* off = w->off.as<uint64_t>();
    uint64_t* bsum = w->bsum.as<uint64_t>();
    uint32_t* order = w->ord.as<uint32_t>();
    uint32_t* rank = w->rank.as<uint32_t>();
    uint64_t* occ_off = w->occ_off.as<uint64_t>();
    uint32_t* level = w->level.as<uint32_t>();
    uint32_t* cnt = w->cnt.as<uint32_t>();
    uint4* rec = w->rec.as<uint4>();
    uint4* rec2 = w->rec2.as<uint4>();

    LV_CHK(hipMemsetAsync(pcnt, 0, sizeof(PackCnt), st));
    // ---- 1. exec ranking: one keys-only sort of the packed exec words
    k_exec_pack<<<blocks_for(n, 256), 256, 0, st>>>(g, c, ka);
    uint64_t* sorted = nullptr;
    LV_CHK(radix_sort_keys(ka, kb, n, (int)c.rb, (int)pp.exec_bits, hist, off, bsum, st, &sorted));
    k_exec_rank_p<<<blocks_for(n, 256), 256, 0, st>>>(g, sorted, c.rb, order, rank, w->kcnt.as<uint32_t>(), ctl);
    LV_CHK(run_scan_arrays(w->kcnt.as<uint32_t>(), occ_off, n, 1, bsum, st));
    if (g.dep_off)
    {
        LV_CHK(hipMemsetAsync(dirp, 0, 4 * n, st));
        k_direct_check<<<std::min(blocks_for(n, 256), 1024u), 256, 0, st>>>(g, rank, dirp, pcnt, ctl);
    }

    // ---- 2. occurrences (rank order) sorted stably by key, one walk -> predecessor records
    uint64_t* occ = sorted == ka ? kb : ka;
    uint64_t* otmp = sorted;
    if (n_occ)
    {
        k_occ_pack<<<std::min(blocks_for(c.kuni ? n_occ : n, 256), 8192u), 256, 0, st>>>(g, c, order, occ_off, occ, n_occ);
        LV_CHK(radix_sort_keys(occ, otmp, n_occ, (int)c.ks, (int)pp.key_bits, hist, off, bsum, st, &occ));
    }
    const PullCfg pc = pull_cfg(n, true);
    for (int attempt = 0;; ++attempt)
    {
        uint32_t* pool = w->pool.as<uint32_t>();
        if (n_occ)
            k_walk<<<blocks_for(n_occ, 256), 256, 0, st>>>(occ, n_occ, c, occ_off, rec, rec2, pool, shard_cap, pcnt);
        LV_CHK(hipEventRecord(w->ev[1], st));

        // ---- 3. level the DAG (rank-ordered dataflow over the records)
        LV_CHK(hipMemsetAsync(level, 0xFF, 4 * n, st));
        const uint64_t pool_cap = shard_cap * NSHARD;
        k_level_rec<<<pc.grid, pc.threads, 0, st>>>(g, occ_off, rec, rec2, pool, pool_cap, dirp, rank, level, cnt, cnt + 1,
                                                    pc.budget, pc.naps, c.kuni);
        LV_CHK(hipGetLastError());
        out->n_launch = 1;
        k_level_max<<<256, 256, 0, st>>>(level, n, cnt + 2);
        k_level_out<<<blocks_for(n, 256), 256, 0, st>>>(order, level, n, level_out);
        LV_CHK(hipEventRecord(w->ev[2], st));
        uint32_t tail[3];
        LV_CHK(d2h(tail, cnt, sizeof(tail), st));
        LV_CHK(d2h(w->h_ctl, ctl, sizeof(LevelsCtl), st));
        LV_CHK(d2h(w->h_pcnt, pcnt, sizeof(PackCnt), st));
        LV_CHK(hipStreamSynchronize(st));
        if (w->h_ctl->error)
        {
            const int code = -(int)w->h_ctl->error;
            *err = code == AD_E_DUP_EXEC ? "ad_levels: two txns with the same executeAt (CommandsForKey.java:1439)"
                                         : "ad_levels: direct dep index out of range";
            return code;
        }
        uint64_t need = 0, edges = 0;
        for (uint32_t i = 0; i < NSHARD; ++i)
        {
            need = std::max<uint64_t>(need, w->h_pcnt->pool[i]);
            edges += w->h_pcnt->edges[i];
        }
        if (need > shard_cap)
        {
            // a pool shard was too small: repeat the walk and the leveling with the size asked for
            if (attempt > 0)
            {
                *err = "ad_levels: predecessor pool did not fit twice";
                return AD_E_STATE;
            }
            shard_cap = need;
            if (shard_cap * NSHARD >= (1ull << 32))
            {
                *err = "ad_levels: predecessor pool beyond 2^32 words";
                return AD_E_CAPACITY;
            }
            LV_ALLOC(w->pool, 4 * shard_cap * NSHARD);
            LV_CHK(hipMemsetAsync(cnt, 0, 4 * 4, st));
            LV_CHK(hipMemsetAsync(pcnt, 0, sizeof(PackCnt), st));
            if (g.dep_off) k_direct_check<<<std::min(blocks_for(n, 256), 1024u), 256, 0, st>>>(g, rank, dirp, pcnt, ctl);
            continue;
        }
        if (tail[1])
        {
            *err = "ad_levels: a wave waited more than a second for a predecessor's level";
            return AD_E_STATE;
        }
        out->n_edges = edges;
        out->n_levels = (uint64_t)tail[2] + 1;
        out->packed = true;
        break;
    }
    float a = 0, b = 0;
    (void)hipEventElapsedTime(&a, w->ev[0], w->ev[1]);
    (void)hipEventElapsedTime(&b, w->ev[1], w->ev[2]);
    out->ms_build = a;
    out->ms_frontier = b;
    out->ms_total = a + b;
    return AD_OK;
}

}  // namespace adx
