// lean.hip — the lean fused kernel: the common case of PreAccept.calculatePartialDeps
// (PreAccept.java:245-267) on a CommandStore without range commands or RedundantBefore entries,
// for requests whose keys' last committed Writes execute before them. Two (or four) requests per wave (lanes 0-31
// and 32-63), no LDS, no trees:
//
//   * executeAt (and txnId) newer than every dictionary id: S = 2 * n_dict without a search
//   * every key's last committed Write executes before S (and S is above prunedBefore): then
//     maxCommittedWriteBefore(S) is the key's last committed Write, so the mapReduceActive
//     emissions (CommandsForKey.java:930-950) are the key's two precomputed lists (KeyEntry,
//     common.hpp) restricted to txnIds below S (insertPos(S), :912-928) -- loaded one element per
//     lane and filtered by rank; a request newer than the whole key keeps every element
//   * Deps.AbstractBuilder.add routing (Deps.java:80-106) and the RelationMultiMap build
//     (RelationMultiMap.java:147-260): a 32-lane bitonic sort of (rank, key) per map
//
// Anything else (more than 8 keys, more than 32 emissions, a key needing the tree, an older id)
// is appended to the deferred list and resolved by the general fused kernel (resolve.hip).
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "common.hpp"
#include "kernels.hpp"
#include "wave.hpp"

namespace adx {

constexpr int LEAN_WAVES = 4;
#ifndef LEAN_OCC_N
#define LEAN_OCC_N 5
#endif
constexpr int LEAN_OCC = LEAN_OCC_N;        // waves per SIMD the register budget is sized for
// the same for the range-command kernels (RNG): at 5 waves per SIMD they spill 36-52 bytes per lane; at 4
// they do not, and config 4 measured faster (round 5: pass 1 0.594 -> 0.589, pass 2 0.166 -> 0.154 ms)
#ifndef LEAN_OCC_RNG
#define LEAN_OCC_RNG 4
#endif
// and for the wide kernels (two emissions per lane)
#ifndef LEAN_OCC_WIDE
#define LEAN_OCC_WIDE 4
#endif
template <bool RNG, bool WIDE> constexpr int lean_occ() { return WIDE ? LEAN_OCC_WIDE : (RNG ? LEAN_OCC_RNG : LEAN_OCC); }
constexpr uint32_t LEAN_MAXP = 8;      // keys per request
#ifndef LEAN_CHUNK_LOG
#define LEAN_CHUNK_LOG 16
#endif
constexpr uint32_t LEAN_CHUNK = 1u << LEAN_CHUNK_LOG;   // region bytes a wave takes from the arena at a time

// Per probe, its KeyLine: k_prepare does the slice test
// (InMemoryCommandStore.java:280) and the perfect-hash displacement, one thread per probe, so that the
// lean passes load a probe's key and its line position side by side -- one dependent load shorter,
// and no displacement gather inside them. The line still proves the key is the store's.
constexpr uint32_t LS_NONE = 0xFFFFFFFFu;
// A wave's items (it0, it0 + nw, ...) from its XCD-relabelled block id (wave.hpp xcd_block): consecutive
// items -- whose request records, keys, size and offset words share cache lines -- run on one XCD's L2
// instead of being dealt over all eight
__device__ __forceinline__ uint32_t lean_block() { return xcd_block(); }
// Loads use clamped addresses on every lane (branch-free, so the loop's wait counts stay exact); at two
// requests per wave a request's KeyLine headers are loaded by all 32 of its lanes, one 16-byte quarter of one
// key's first 64 bytes per lane (one vector load per item instead of four, each line touched once), and
// handed to the key lanes through a per-wave LDS stage (QL below). Sorting networks and segment scans
// exchange lanes by DPP / permlane swaps (wave.hpp xor_lane), not ds_bpermute.
// Wide pass 1 (run_resolve_lean's wide1, chosen per batch by the host): pass 1 also takes the requests of
// 33..64 raw emissions (two per lane, the pass-2 path), at pass 2's register budget (4 waves per SIMD);
// pass 2 then sees only what exceeds 64. Measured on config 2: passes 1 + 2 0.613 -> 0.560 ms; on
// config 3's store (uniform keys, almost nothing above 32) 0.743 -> 0.841 ms

// ascending bitonic sort within each LPR-lane segment (a request's lanes)
template <uint32_t K, uint32_t LPR>
__device__ __forceinline__ void seg_bitonic(uint32_t& key)
{
    const uint32_t l = lane_id() & (LPR - 1);
#pragma unroll
    for (uint32_t k = 2; k <= K; k <<= 1)
#pragma unroll
        for (uint32_t j = k >> 1; j > 0; j >>= 1)
        {
            const uint32_t ok = xor_lane(key, j);
            const bool up = (l & k) == 0;
            const bool lower = (l & j) == 0;
            key = (lower == up) ? min(key, ok) : max(key, ok);
        }
}

template <uint32_t K, uint32_t LPR>
__device__ __forceinline__ void seg_bitonic64(uint64_t& key)
{
    const uint32_t l = lane_id() & (LPR - 1);
#pragma unroll
    for (uint32_t k = 2; k <= K; k <<= 1)
#pragma unroll
        for (uint32_t j = k >> 1; j > 0; j >>= 1)
        {
            const uint64_t ok = xor_lane64(key, j);
            const bool up = (l & k) == 0;
            const bool lower = (l & j) == 0;
            key = (lower == up) ? min(key, ok) : max(key, ok);
        }
}

// ascending bitonic sort of the 2 x 32 elements of each 32-lane segment, element i = 32 s + lane
// held in register s (x0: s = 0, x1: s = 1); a partner at distance 32 is the lane's other register
template <class T>
__device__ __forceinline__ void seg_bitonic_wide(T& x0, T& x1)
{
    const uint32_t l = lane_id() & 31u;
#pragma unroll
    for (uint32_t k = 2; k <= 64; k <<= 1)
#pragma unroll
        for (uint32_t j = k >> 1; j > 0; j >>= 1)
        {
            if (j == 32)
            {
                // i = l (lower) against i = l + 32; direction from bit k of i (k == 64: ascending)
                const bool up = (l & k) == 0;
                const T lo = min(x0, x1), hi = max(x0, x1);
                x0 = up ? lo : hi;
                x1 = up ? hi : lo;
            }
            else
            {
                T o0, o1;
                if constexpr (sizeof(T) == 4)
                {
                    o0 = xor_lane(x0, j);
                    o1 = xor_lane(x1, j);
                }
                else
                {
                    o0 = __shfl_xor(x0, (int)j, 64);
                    o1 = __shfl_xor(x1, (int)j, 64);
                }
                const bool lower = (l & j) == 0;
                const bool up0 = (l & k) == 0, up1 = ((l + 32) & k) == 0;
                x0 = (lower == up0) ? min(x0, o0) : max(x0, o0);
                x1 = (lower == up1) ? min(x1, o1) : max(x1, o1);
            }
        }
}

// ascending bitonic sort of the 2 x LPR elements of each LPR-lane segment (LPR <= 16: partners within a DPP
// row), element i = LPR s + l held in register s; a partner LPR away is the lane's other register
template <class T, uint32_t LPR>
__device__ __forceinline__ void seg_bitonic_w(T& x0, T& x1)
{
    const uint32_t l = lane_id() & (LPR - 1);
#pragma unroll
    for (uint32_t k = 2; k <= 2 * LPR; k <<= 1)
#pragma unroll
        for (uint32_t j = k >> 1; j > 0; j >>= 1)
        {
            if (j == LPR)
            {
                const T lo = min(x0, x1), hi = max(x0, x1);      // k == 2 LPR: ascending
                x0 = lo;
                x1 = hi;
            }
            else
            {
                const T o0 = xor_lane(x0, j), o1 = xor_lane(x1, j);
                const bool lower = (l & j) == 0;
                const bool up0 = (l & k) == 0, up1 = ((l + LPR) & k) == 0;
                x0 = (lower == up0) ? min(x0, o0) : max(x0, o0);
                x1 = (lower == up1) ? min(x1, o1) : max(x1, o1);
            }
        }
}

struct LeanChunk {
    // wave-uniform bump allocation from the region arena, offsets in 8-byte units (regions and chunks
    // are multiples of 8 bytes; the arena stays below 32 GB), in fixed chunks. (Refills sized for what the
    // wave will still write kept the arena dense -- 304 MB in use for 272 MB of config-2 regions -- but
    // measured 0.06 ms slower per config-2 step: the estimator's registers spilled in pass 1.)
    uint32_t cur = 0, end = 0;
    template <int PASS>
    __device__ __forceinline__ uint64_t take(BatchCtl* ctl, uint64_t nbytes, uint64_t cap, uint32_t it, uint32_t n_items,
                                             uint32_t nw)
    {
        const uint32_t n8 = (uint32_t)(nbytes >> 3);
        if (n8 > end - cur)
        {
            // fixed chunks: pass 1's waves write ~50 KB each (config 2), pass 2's ~13 KB
            const uint64_t want = PASS == 1 ? LEAN_CHUNK : LEAN_CHUNK / 4;
            const uint64_t sz = nbytes > want ? nbytes : want;
            unsigned long long base = 0;
            if (lane_id() == 0) base = atomicAdd(&ctl->reg_top, (unsigned long long)sz);
            base = uniform64(base);
            if (base + sz > cap && lane_id() == 0) atomicOr(&ctl->overflow, 8u);
            cur = (uint32_t)(base >> 3);
            end = (uint32_t)((base + sz) >> 3);
        }
        const uint64_t r = (uint64_t)cur << 3;
        cur += n8;
        return r;
    }
};

// Request lists: `in` (null = all requests) with *in_count entries; the requests this pass cannot
// take are appended to `out` (*out_count entries; *out_real counts them too).
struct LeanLists {
    const uint32_t* in;
    const unsigned long long* in_count;
    uint32_t* out;
    unsigned long long* out_count;
    unsigned long long* out_real;
};

// segmented prefix helpers over the 8 key lanes of each request segment
__device__ __forceinline__ uint32_t key_lanes_incl_scan(uint32_t v, uint32_t hl)
{
#pragma unroll
    for (uint32_t d = 1; d < 8; d <<= 1)
    {
        const uint32_t t = row_up(v, d);
        if ((hl & 7) >= d) v += t;
    }
    return v;
}

// RPW requests per wave (8: 8 lanes each, up to 8 raw emissions -- a store's share of requests that
// span many stores, ~1 key each; 4: 16 lanes, up to 16; 2: 32 lanes, up to 32; 1: 64 lanes, up to 64).
// RNG: the store has range commands (with a stabbing index): each request also gets its
// rangeDeps from the cells of its keys (mapReduceRangesInternal, InMemoryCommandStore.java:884-1017).
// WIDE (RPW 2, no range commands: lean pass 2): requests with up to 64 raw emissions, two per lane.
template <uint32_t RPW, bool RNG, bool WIDE, int PASS>
__global__ __launch_bounds__(64 * LEAN_WAVES, (lean_occ<RNG, WIDE>())) void k_resolve_lean(DevSnapshot s, BatchBufs b)
{
    constexpr uint32_t pass = PASS;
    // pass 1: all requests -> deferred1; pass 2: deferred1 -> deferred2 (lists derived from b
    // where used, so they hold no scalar registers across the loop)
    auto lists = [&]() -> LeanLists {
        if (pass == 1) return LeanLists{nullptr, nullptr, b.deferred1, &b.ctl->n_deferred1, &b.ctl->n_real1};
        return LeanLists{b.deferred1, &b.ctl->n_deferred1, b.deferred2, &b.ctl->n_deferred2, &b.ctl->n_real2};
    };
    constexpr uint32_t LPR = 64 / RPW;                       // lanes per request
    const uint32_t lane = lane_id(), h = lane / LPR, hl = lane & (LPR - 1), sb = h * LPR;
    const uint64_t below = (1ull << hl) - 1;                 // lanes below this one in its segment
    constexpr uint64_t SEGMASK = LPR == 64 ? ~0ull : ((1ull << LPR) - 1);
    auto seg = [&](uint64_t m) -> uint64_t { return RPW == 1 ? m : ((m >> sb) & SEGMASK); };
    // wave-uniform max over the segments' values of v (read at each segment's lane 0)
    auto seg_max = [&](uint32_t v) -> uint32_t {
        uint32_t mx = 0;
#pragma unroll
        for (uint32_t k = 0; k < RPW; ++k) mx = max(mx, (uint32_t)__builtin_amdgcn_readlane((int)v, (int)(k * LPR)));
        return mx;
    };
    const uint64_t n = b.n_txns;
    const uint32_t n_slots = pass == 1 ? (uint32_t)n : (uint32_t)uniform64(b.ctl->n_deferred1);
    const uint32_t n_items = (n_slots + RPW - 1) / RPW;
    const uint32_t nw = gridDim.x * LEAN_WAVES;
    const uint64_t reg_cap = uniform64(b.ctl->reg_cap);

    LeanChunk ralloc;
    // one wave-uniform region allocation for the segments' byte counts (at each segment's lane 0):
    // returns this segment's offset; `fits` whether the whole allocation is inside the arena
    auto seg_alloc = [&](uint64_t bytes, bool& fits, uint32_t it) -> uint64_t {
        uint64_t total = 0, mine = 0;
#pragma unroll
        for (uint32_t k = 0; k < RPW; ++k)
        {
            const uint64_t bk = uniform64(__shfl(bytes, (int)(k * LPR), 64));
            if (k == h) mine = total;
            total += bk;
        }
        const uint64_t base = ralloc.template take<PASS>(b.ctl, total, reg_cap, it, n_items, nw);
        fits = base + total <= reg_cap;
        return base + mine;
    };
    // deferrals are gathered in a per-wave LDS buffer and appended to the out list in exact-size
    // blocks (one atomic per block, no holes)
    // Pass 1 keeps two: requests pass 2 can serve (more raw emissions than pass 1's lanes, within pass
    // 2's) go to D1, the rest -- a key needing the tree, a record the lean path cannot take, more raw
    // emissions than pass 2 takes -- straight to D2, the general kernel's list (pass 2 would only defer
    // them again: 99k late PreAccepts of the request mix cost pass 2 0.12 ms for nothing)
    constexpr int NBUF = PASS == 1 ? 2 : 1;
    constexpr uint32_t SPLIT_BIT = 0x80000000u, LEAN_SPLIT_T = 256;
    __shared__ uint32_t dbuf_all[LEAN_WAVES][NBUF][DEFER_CHUNK];
    uint32_t* dbuf = dbuf_all[threadIdx.x >> 6][0];
    uint32_t* hbuf = dbuf_all[threadIdx.x >> 6][NBUF - 1];
    uint32_t dn = 0, hn = 0;    // wave-uniform fills of dbuf (-> lists().out) and hbuf (pass 1: -> D2)
    auto flush_to = [&](uint32_t* buf, uint32_t& cnt, bool to_d2) {
        if (!cnt) return;
        wave_lds_sync();
        const uint32_t tv = lane_id() < cnt ? buf[lane_id()] : 0u;
        wave_lds_sync();
        // pass 1's hard deferrals: a Range-domain request of a mixed batch (REC_SPLIT, k_prepare) goes straight to
        // the split kernels' list; the rest to D2
        // (bit 31: a request with more raw emissions than the general kernel stages -- it would only defer it again)
        const bool sp = to_d2 && lane_id() < cnt && ((tv & SPLIT_BIT) != 0 || (b.q_rec[tv & ~SPLIT_BIT].z & REC_SPLIT) != 0);
        const uint64_t spm = ballot(sp);
        const uint32_t nsp = __popcll(spm), nrest = cnt - nsp;
        unsigned long long base = 0, sbase = 0;
        if (lane_id() == 0)
        {
            const LeanLists io = lists();
            unsigned long long* oc = to_d2 ? &b.ctl->n_deferred2 : io.out_count;
            unsigned long long* orl = to_d2 ? &b.ctl->n_real2 : io.out_real;
            if (nrest)
            {
                base = atomicAdd(oc, (unsigned long long)nrest);
                atomicAdd(orl, (unsigned long long)nrest);
            }
            if (nsp) sbase = atomicAdd(&b.ctl->n_deferred, (unsigned long long)nsp);
        }
        base = uniform64(base);
        sbase = uniform64(sbase);
        const uint64_t below = (1ull << lane_id()) - 1;
        if (sp) b.deferred[sbase + __popcll(spm & below)] = tv & ~SPLIT_BIT;
        else if (lane_id() < cnt) (to_d2 ? b.deferred2 : lists().out)[base + __popcll(~spm & below)] = tv;
        cnt = 0;
    };
    auto dflush = [&]() {
        flush_to(dbuf, dn, false);
        if (PASS == 1) flush_to(hbuf, hn, true);
    };

    // ---- software pipeline over the wave's items it, it + nw, ... (RPW requests each). Per
    // iteration the next item's raw inputs are derived and its keys/slots loaded at the top, its
    // KeyEntry quarters once this item's list loads are out: the chain key_off -> slot ->
    // KeyEntry -> lists costs about one round trip per iteration. Pipeline loads are branch-free
    // (clamped addresses, results masked where used) so the compiler's wait counts stay exact.
    using Raw = uint4;        // the request record of k_prepare
    struct Req { uint64_t k0; uint32_t np, cls, t, S, self; bool act, defer; };
    // the request of item `it` in this segment: pass 1 its index; pass 2 the deferred1 entry, loaded
    // (branch-free) by dload an iteration before its record is (req_of then only masks the hole)
    auto dload = [&](uint32_t it) -> uint32_t {
        if (PASS == 1) return 0u;
        const uint32_t si = it * RPW + h;
        const uint32_t v = b.deferred1[si < n_slots ? si : 0u];
        return si < n_slots ? v : DEFER_HOLE;
    };
    auto req_of = [&](uint32_t it, uint32_t loaded) -> uint32_t {
        if (PASS == 2) return loaded;
        const uint32_t si = it * RPW + h;
        return si >= n_slots ? DEFER_HOLE : si;
    };
    // one lane per request loads its 16-byte record (the texture data path moves 16 B per request, not
    // per lane); derive() broadcasts it over the request's lanes
    auto loadA = [&](uint32_t t) -> Raw {
        return b.q_rec[t != DEFER_HOLE ? t : 0u];
    };
    // the value of the segment's lane p (p known after unrolling) in every lane of the segment
    auto seg_lane = [&](uint32_t v, uint32_t p) -> uint32_t {
        return (uint32_t)__shfl((int)v, (int)(sb | p), 64);
    };
    // the record carries PreAccept.java:251-261's witness class, S and self as ranks (k_prepare)
    // and whether the request fits the lean path (<= 8 keys, valid kind); anything else defers
    auto derive = [&](uint32_t t, const Raw& r0) -> Req {
        const Raw& r = r0;
        Req q{0, 0, 0, t, 0, 0, false, false};
        q.act = t != DEFER_HOLE;
        q.k0 = r.x;
        q.S = r.y;             // rank of executeAt
        q.self = r.w;          // rank of the txnId unless it is the executeAt (0: none)
        q.np = r.z & 0xFFFFu;
        q.cls = (r.z >> 16) & 3u;
        q.defer = (r.z & REC_FAST) == 0;
        return q;
    };
    // the key (one lane per key) and its line position beside it (k_prepare: the slice test and the perfect
    // hash's displacement, so the line load waits on no displacement gather here; round 6, config 4's range
    // kernels: pass 1 0.622 -> 0.566 ms, k_prepare 0.020 -> 0.045)
    auto loadB = [&](const Req& q, int64_t& key, uint32_t& sl) {
        const bool on = q.act && !q.defer && hl < q.np;
        key = b.q_keys[on ? q.k0 + hl : 0];
        const uint32_t v = b.p_slot[on ? q.k0 + hl : 0];
        sl = on ? v : LS_NONE;
    };
    // the key's line (KeyLine, common.hpp): one random line per key -- its first 64 bytes: key, cell entries,
    // newest fields, meta, the class's {count, start} and the cwr tail start. A slot holding another key is
    // resolved when used.
    struct Hdr { uint4 h0, h1; uint2 h2, h3; uint4 q; uint32_t slot; bool look; };
    constexpr bool QL = !RNG && RPW == 2;
    __shared__ uint4 qst_all[QL ? LEAN_WAVES : 1][QL ? 64 : 1];
    auto load_line = [&](uint32_t slot, uint32_t cls, Hdr& H) {
        const uint4* L4 = reinterpret_cast<const uint4*>(s.kline + slot);
        H.h0 = L4[0];
        H.h1 = L4[1];
        H.h2 = reinterpret_cast<const uint2*>(L4 + 2)[cls];
        H.h3 = reinterpret_cast<const uint2*>(L4 + 3)[1];       // {cwr tail start, prunedBefore rank}
    };
    auto loadD = [&](const Req&, int64_t, uint32_t sl, bool& look, uint32_t& d) {
        look = sl != LS_NONE;
        d = sl;
    };
    auto loadC = [&](const Req& q, int64_t key, bool look, uint32_t d, Hdr& H) {
        H.look = look;
        H.slot = !look ? 0u : d;
        if (QL)
        {
            // lane hl loads quarter hl & 3 of key hl >> 2's line (unmasked: unpacked under the key lane's look)
            const uint32_t ks = __shfl(look ? H.slot : LS_NONE, (int)(sb | (hl >> 2)), 64);
            H.q = reinterpret_cast<const uint4*>(s.kline + (ks != LS_NONE ? ks : 0u))[hl & 3u];
            return;
        }
        load_line(H.slot, q.cls, H);
    };
    // (found, cell bounds) of a loaded line: the perfect hash put the key on this line if the
    // store holds it; a line of another key (or an empty one) means no CommandsForKey
    auto resolve_line = [&](int64_t key, uint32_t cls, Hdr& H, bool& found, uint2& cb) {
        if (QL)
        {
            uint4* st = qst_all[QL ? (threadIdx.x >> 6) : 0];
            st[lane] = H.q;
            wave_lds_sync();
            const uint32_t b4 = sb + 4 * (hl & 7u);
            H.h0 = st[b4];
            H.h1 = st[b4 + 1];
            const uint4 q2 = st[b4 + 2], q3 = st[b4 + 3];
            H.h2 = cls == 0 ? make_uint2(q2.x, q2.y) : (cls == 1 ? make_uint2(q2.z, q2.w) : make_uint2(q3.x, q3.y));
            H.h3 = make_uint2(q3.z, q3.w);
            wave_lds_sync();
        }
        auto key_of = [](const uint4& h0) { return (int64_t)(((uint64_t)h0.y << 32) | h0.x); };
        found = H.look && (H.h1.w & KL_USED) && key_of(H.h0) == key;
        cb = found ? make_uint2(H.h0.z, H.h0.w) : make_uint2(0, 0);
        if (RNG && H.look && !found && s.cell_off)
        {
            // a key without a CommandsForKey: its cell by search (rare)
            uint64_t lo = 0, hi = s.n_cell_E;
            while (lo < hi)
            {
                const uint64_t mid = (lo + hi) >> 1;
                const int64_t v = s.cell_E[mid];
                if (s.start_inclusive ? v <= key : v < key) lo = mid + 1;
                else hi = mid;
            }
            cb = make_uint2(s.cell_off[lo], s.cell_off[lo + 1]);
        }
    };

    // sizes of map m (keys, txnIds, keysToTxnIds) and its region offset: one store from lanes
    // hl = 0..3 of each segment (per-lane addresses keep the size arrays out of scalar registers)
    auto put_sizes = [&](bool on, uint32_t t, int m, uint32_t v0, uint32_t v1, uint32_t v2, uint64_t ro, bool with_ro) {
        if (on && hl < 3)
        {
            const uint32_t v = hl == 0 ? v0 : (hl == 1 ? v1 : v2);
            b.sz[(uint64_t)(3 * m + hl) * n + t] = v;
        }
        if (with_ro && on && hl == 3) b.t_reg[(uint64_t)m * n + t] = ro;
    };

    // Pipeline registers at the top of iteration `it`: item it's request and lines (qc, keyc, Hc); item
    // it + nw's request and keys / line positions (q1, key1, sl1); item it + 2 nw's record (t2, r2);
    // pass 2: item it + 3 nw's deferred1 entry (t3). Every load of a later item is issued after this
    // item's element loads and before its stores, and waited for an iteration later -- no wait of the
    // loop covers the stores just issued (vmcnt counts loads and stores in order).
    const uint32_t it0 = uniform(lean_block() * LEAN_WAVES + (threadIdx.x >> 6));
    // The pipeline registers, two sets used in turn (the loop body runs twice per trip, C -> N then N -> C):
    // every later item's load lands in the other set, so the loop never copies a register whose load is in
    // flight -- such a copy waits for it, and vmcnt counts loads and stores in order, so the back edge used to
    // wait for every load and store of the iteration.
    struct Pipe {
        Req qc;          // item it: its request,
        int64_t keyc;    //   its key lane's key,
        Hdr Hc;          //   its line (header quarter)
        Req q1;          // item it + nw: its request,
        int64_t key1;    //   key and line position loads
        uint32_t sl1;
        uint32_t t2;     // item it + 2 nw: request index and record
        Raw r2;
        uint32_t t3;     // pass 2: item it + 3 nw's deferred1 entry
    };
    Pipe PA, PB;
    {
        const uint32_t tc = req_of(it0, dload(it0));
        PA.qc = derive(tc, loadA(tc));
        uint32_t slc = LS_NONE;
        loadB(PA.qc, PA.keyc, slc);
        bool lookc;
        uint32_t dc;
        loadD(PA.qc, PA.keyc, slc, lookc, dc);
        loadC(PA.qc, PA.keyc, lookc, dc, PA.Hc);
        const uint32_t t1 = req_of(it0 + nw, dload(it0 + nw));
        PA.q1 = derive(t1, loadA(t1));
        PA.sl1 = LS_NONE;
        loadB(PA.q1, PA.key1, PA.sl1);
        PA.t2 = req_of(it0 + 2 * nw, dload(it0 + 2 * nw));
        PA.r2 = loadA(PA.t2);
        PA.t3 = dload(it0 + 3 * nw);
    }
    // the later items' loads of the step for item it (C -> N)
    auto prefetch = [&](uint32_t it, const Pipe& C, Pipe& N) {
        bool look1;
        uint32_t d1;
        loadD(C.q1, C.key1, C.sl1, look1, d1);
        loadC(C.q1, C.key1, look1, d1, N.Hc);
        N.q1 = derive(C.t2, C.r2);
        N.sl1 = LS_NONE;
        loadB(N.q1, N.key1, N.sl1);
        N.t2 = req_of(it + 3 * nw, C.t3);
        N.r2 = loadA(N.t2);
        N.t3 = dload(it + 4 * nw);
        N.qc = C.q1;
        N.keyc = C.key1;
    };
    uint32_t nwide = 0;         // wave-uniform: wide pass 1's requests above LPR raw emissions
    auto step = [&](const uint32_t it, Pipe& C, Pipe& N) {
        Req& qc = C.qc;
        const int64_t keyc = C.keyc;
        Hdr& Hc = C.Hc;
        const uint32_t t = qc.t;

        // ---- current item: per key p = hl < np, newest test and emission counts
        bool act = qc.act;
        bool defer = qc.defer;
        const uint32_t np = qc.np, cls = qc.cls, S = qc.S, self = qc.self;
        const bool kact = act && !defer && hl < np;
        bool has_cfk;
        uint2 cbc;
        resolve_line(keyc, cls, Hc, has_cfk, cbc);
        const uint32_t meta = Hc.h1.w;
        // lean-served: M = the last committed Write's executeAt (it executes before S,
        // CommandsForKey.java:912-928) and no prunedBefore substitute (S above prunedBefore,
        // :952-965); end = insertPos(S) is the element filter rank < S below
        const bool newest = !has_cfk || (Hc.h1.y < S && (Hc.h3.y == 0 || S > Hc.h3.y) && !(meta & KL_NOLEAN));
        const uint32_t n1 = has_cfk ? Hc.h2.x : 0u;
        const uint32_t n2 = !has_cfk ? 0u : (cls == 0 ? (Hc.h1.z != 0 ? 1u : 0u) : (meta & KL_NCWR_MASK));
        const uint32_t nn = kact ? n1 + n2 : 0u;
        uint32_t inc = nn;       // exclusive prefix of nn over the 8 key lanes of each request
#pragma unroll
        for (uint32_t d = 1; d < 8; d <<= 1)
        {
            const uint32_t v = row_up(inc, d);
            if ((hl & 7) >= d) inc += v;
        }
        const uint32_t start = inc - nn;
        const uint32_t T = seg_lane(inc, 7u);
        // range raw emissions: the entries of each key's cell
        const uint32_t rn = (RNG && kact) ? cbc.y - cbc.x : 0u;
        const uint32_t rinc = RNG ? key_lanes_incl_scan(rn, hl) : 0u;
        const uint32_t rstart = rinc - rn;
        const uint32_t TR = RNG ? seg_lane(rinc, 7u) : 0u;
        constexpr bool CAN_WIDE = WIDE && RPW == 2 && !RNG;
        // raw emissions pass 2 takes: 64 (two per lane) without range commands; with them 32 after a pass 1
        // of four requests per wave, else 64 (run_resolve_lean)
        constexpr uint32_t P2CAP = !RNG ? 64u : (RPW == 4 ? 32u : 64u);
        // four requests per wave with range commands (32-bit rangeDeps keys): a request of 17..32 range emissions
        // takes two per lane in the range round (rwide below) instead of lean pass 2
        const bool rw_ok = RNG && RPW == 4 && PASS == 1 && s.rng32;
        const bool hard = defer || seg(ballot(kact && !newest)) != 0 || (PASS == 1 && (T > P2CAP || TR > P2CAP));
        defer = hard || T > (CAN_WIDE ? 2 * LPR : LPR) || TR > (rw_ok ? 2 * LPR : LPR);
        {
            const bool soft = PASS == 1 ? !hard : true;
            const uint64_t dm = ballot(act && defer && soft && hl == 0);
            const uint32_t nd = __popcll(dm);
            if (nd)
            {
                if (dn + nd > DEFER_CHUNK) flush_to(dbuf, dn, false);
                if (act && defer && soft && hl == 0) dbuf[dn + __popcll(dm & ((1ull << lane) - 1))] = t;
                dn += nd;
            }
            if (PASS == 1)
            {
                const uint64_t hm = ballot(act && hard && hl == 0);
                const uint32_t nh = __popcll(hm);
                if (nh)
                {
                    if (hn + nh > DEFER_CHUNK) flush_to(hbuf, hn, true);
                    // (more raw emissions than the general kernel stages, 64 per map: straight to the split kernels)
                    if (act && hard && hl == 0)
                        hbuf[hn + __popcll(hm & ((1ull << lane) - 1))] = t | (T > LEAN_SPLIT_T ? SPLIT_BIT : 0u);
                    hn += nh;
                }
            }
        }
        act = act && !defer;
        // the later items' loads go out once, here, for both paths below, into the other register set (N); the
        // element loads' wait covers them too. (Behind the element loads instead, as before round 6: no faster --
        // config 2 pass 1 0.538 against 0.533 ms, config 4 / 3 / the mix within noise.)
        prefetch(it, C, N);

        // ---- the wide item: a request with 33..64 raw emissions -> two per lane (element x = hl and
        // hl + 32), sorted as 64 (seg_bitonic_wide), the rest as below with masks over both halves
        if (CAN_WIDE && seg_max(act && !defer ? T : 0u) > LPR)
        {
            const bool wact = act && !defer;
            if (PASS == 1) nwide += __popcll(ballot(wact && hl == 0 && T > LPR));
            auto raw_txw = [&](uint32_t x, uint32_t& ax) -> uint32_t {
                ax = 0;
#pragma unroll
                for (uint32_t p = 1; p < LEAN_MAXP; ++p)
                {
                    const uint32_t sp = seg_lane(start, p);
                    if (p < np && x >= sp) ax = p;
                }
                const uint32_t sx = sb | ax;
                const uint32_t x_start = __shfl(start, sx, 64), x_n1 = __shfl(n1, sx, 64);
                const uint32_t x_base = __shfl(Hc.h2.y, sx, 64), x_ct = __shfl(Hc.h3.x, sx, 64), x_lw = __shfl(Hc.h1.z, sx, 64);
                const uint32_t x_meta = __shfl(meta, sx, 64), x_slot = __shfl(Hc.slot, sx, 64);
                const bool lv_ = wact && x < T;
                const uint32_t ii = x - x_start;
                const bool fc = ii < x_n1;
                const uint32_t* lp_;
                if (x_meta & KL_INLINE)
                    lp_ = s.kline[x_slot].inl + (fc ? ii : ((x_meta >> KL_INL_SHIFT) & 31u) + (ii - x_n1));
                else
                    lp_ = fc ? s.cand + (x_base + ii) : s.cwr + (x_ct + (ii - x_n1));
                if (!lv_ || (!fc && cls == 0)) lp_ = s.cand;
                const uint32_t v = *lp_;
                return !lv_ ? 0u : ((fc || cls != 0) ? v : (x_lw | (1u << RANK_BITS)));
            };
            uint32_t ax0, ax1;
            const uint32_t tw0 = raw_txw(hl, ax0), tw1 = raw_txw(hl + 32, ax1);
            const uint32_t r0 = tw0 & RANK_MASK, r1 = tw1 & RANK_MASK;
            const bool want0 = wact && hl < T && r0 != self && r0 < S, want1 = wact && hl + 32 < T && r1 != self && r1 < S;
            const bool is1_0 = ((KINDS_RS_OR_WS >> (tw0 >> RANK_BITS)) & 1) == 0;
            const bool is1_1 = ((KINDS_RS_OR_WS >> (tw1 >> RANK_BITS)) & 1) == 0;
            for (int m = 0; m < 3; m += 2)
            {
                const bool mine0 = want0 && (m == 0 ? !is1_0 : is1_0), mine1 = want1 && (m == 0 ? !is1_1 : is1_1);
                const uint64_t mb0 = ballot(mine0), mb1 = ballot(mine1);
                const uint32_t tot = __popcll(seg(mb0)) + __popcll(seg(mb1));
                if ((mb0 | mb1) == 0)
                {
                    put_sizes(wact, t, m, 0, 0, 0, 0, false);
                    continue;
                }
                uint32_t k0 = mine0 ? ((r0 << 3) | ax0) : 0xFFFFFFFFu, k1 = mine1 ? ((r1 << 3) | ax1) : 0xFFFFFFFFu;
                seg_bitonic_wide(k0, k1);
                const bool v0 = hl < tot, v1 = hl + 32 < tot;
                const uint32_t x0 = k0 >> 3, x1 = k1 >> 3, ka0 = k0 & 7u, ka1 = k1 & 7u;
                const uint32_t p0 = wave_up1(k0);
                const uint32_t last0 = __shfl(k0, (int)(sb | 31u), 64);
                const uint32_t up1 = wave_up1(k1);   // by every lane (an inactive source reads 0)
                const uint32_t p1 = hl == 0 ? last0 : up1;
                const bool u0 = v0 && (hl == 0 || (p0 >> 3) != x0);
                const bool u1 = v1 && (p1 >> 3) != x1;
                const uint64_t um0 = seg(ballot(u0)), um1 = seg(ballot(u1));
                const uint32_t nu0 = __popcll(um0);
                const uint32_t U = nu0 + __popcll(um1);
                const uint32_t ur0 = __popcll(um0 & below) + (u0 ? 1u : 0u) - 1u;
                const uint32_t ur1 = nu0 + __popcll(um1 & below) + (u1 ? 1u : 0u) - 1u;
                // elements of the same key before each one (sorted order: half 0, then half 1)
                uint64_t s00 = ballot(v0), s01 = ballot(v0), s10 = ballot(v1), s11 = ballot(v1);
#pragma unroll
                for (int bit = 0; bit < 3; ++bit)
                {
                    const uint64_t b0 = ballot((ka0 >> bit) & 1u), b1 = ballot((ka1 >> bit) & 1u);
                    s00 &= ((ka0 >> bit) & 1u) ? b0 : ~b0;      // half-0 elements with key ka0
                    s10 &= ((ka0 >> bit) & 1u) ? b1 : ~b1;      // half-1 elements with key ka0
                    s01 &= ((ka1 >> bit) & 1u) ? b0 : ~b0;      // half-0 elements with key ka1
                    s11 &= ((ka1 >> bit) & 1u) ? b1 : ~b1;      // half-1 elements with key ka1
                }
                (void)s10;
                const uint32_t pk0 = __popcll(seg(s00) & below);
                const uint32_t pk1 = __popcll(seg(s01)) + __popcll(seg(s11) & below);
                // per key p: its map-m emissions in its raw range [start, start + nn) over both halves
                const uint64_t raw_m = seg(mb0) | (seg(mb1) << 32);
                const uint64_t rmask = nn >= 64 ? ~0ull : (((1ull << nn) - 1) << start);
                const uint32_t cnt = hl < 8 ? (uint32_t)__popcll(raw_m & rmask) : 0u;
                uint32_t cinc = cnt;
#pragma unroll
                for (uint32_t d = 1; d < 8; d <<= 1)
                {
                    const uint32_t v = row_up(cinc, d);
                    if ((hl & 7) >= d) cinc += v;
                }
                const uint32_t kstart_l = cinc - cnt;
                const uint64_t nem = seg(ballot(hl < 8 && cnt > 0));
                const uint32_t nk = __popcll(nem);
                const uint32_t kk = __popcll(nem & below);
                const uint32_t kst0 = __shfl(kstart_l, sb | ka0, 64), kst1 = __shfl(kstart_l, sb | ka1, 64);
                const uint64_t bytes = wact && tot ? (((uint64_t)nk * 8 + (uint64_t)U * 4 + (uint64_t)(nk + tot) * 4 + 7) & ~7ull) : 0;
                bool fits;
                const uint64_t ro = seg_alloc(bytes, fits, it);
                put_sizes(wact, t, m, fits ? nk : 0, fits ? U : 0, fits ? nk + tot : 0, ro, true);
                if (wact && tot && fits)
                {
                    int64_t* okeys = reinterpret_cast<int64_t*>(b.reg + ro);
                    uint32_t* otx = reinterpret_cast<uint32_t*>(okeys + nk);
                    int32_t* ok2t = reinterpret_cast<int32_t*>(otx + U);
                    if (hl < 8 && cnt > 0)
                    {
                        okeys[kk] = keyc;
                        ok2t[kk] = (int32_t)(nk + kstart_l + cnt);
                    }
                    if (u0) otx[ur0] = (x0 - 1) >> 1;
                    if (u1) otx[ur1] = (x1 - 1) >> 1;
                    if (v0) ok2t[nk + kst0 + pk0] = (int32_t)ur0;
                    if (v1) ok2t[nk + kst1 + pk1] = (int32_t)ur1;
                }
            }
            put_sizes(wact, t, 1, 0, 0, 0, 0, false);          // no range commands on this path
            return;
        }

        // ---- one raw emission per lane: element e = hl of key a
        uint32_t a = 0;
#pragma unroll
        for (uint32_t p = 1; p < LEAN_MAXP; ++p)
        {
            const uint32_t sp = seg_lane(start, p);
            if (p < np && hl >= sp) a = p;
        }
        const uint32_t src = sb | a;
        const uint32_t a_start = __shfl(start, src, 64), a_n1 = __shfl(n1, src, 64);
        const uint32_t a_base = __shfl(Hc.h2.y, src, 64), a_ct = __shfl(Hc.h3.x, src, 64), a_lw = __shfl(Hc.h1.z, src, 64);
        const uint32_t a_meta = __shfl(meta, src, 64), a_slot = __shfl(Hc.slot, src, 64);
        const bool live = act && hl < T;
        const uint32_t i = hl - a_start;
        const bool from_cand = i < a_n1;
        // the element: inline in the key's line (the line just read: cache-hot) or in the lists
        const uint32_t* lp;
        if (a_meta & KL_INLINE)
            lp = s.kline[a_slot].inl + (from_cand ? i : ((a_meta >> KL_INL_SHIFT) & 31u) + (i - a_n1));
        else
            lp = from_cand ? s.cand + (a_base + i) : s.cwr + (a_ct + (i - a_n1));
        // class Ws: the last Write, no load; lanes without an element load nothing
        const uint32_t lv = *((!live || (!from_cand && cls == 0)) ? s.cand : lp);
        // range elements (same round trip as the list loads)
        uint32_t ar = 0, ar1 = 0;
        uint64_t ce = 0, ce1 = 0;
        bool rlive = false, rlive1 = false;
        const bool rwide = rw_ok && seg_max(act ? TR : 0u) > LPR;      // wave-uniform
        if (RNG)
        {
#pragma unroll
            for (uint32_t p = 1; p < LEAN_MAXP; ++p)
            {
                const uint32_t sp = seg_lane(rstart, p);
                if (p < np && hl >= sp) ar = p;
            }
            const uint32_t rsrc = sb | ar;
            const uint32_t ar_start = __shfl(rstart, rsrc, 64), ar_lo = __shfl(cbc.x, rsrc, 64);
            // the cell's entries inline in the key's line (KL_CELLINL: the line just read) or in cell_ent
            const uint32_t ar_meta = __shfl(has_cfk ? meta : 0u, rsrc, 64), ar_slot = __shfl(Hc.slot, rsrc, 64);
            const bool cin = (ar_meta & KL_CELLINL) != 0;
            rlive = act && hl < TR;
            const uint64_t* kl64 = reinterpret_cast<const uint64_t*>(s.kline);
            const uint64_t cidx = cin ? (uint64_t)ar_slot * (sizeof(KeyLine) / 8) + offsetof(KeyLine, inl) / 8 +
                                            ((ar_meta >> KL_CELL_SHIFT) & 7u) + (hl - ar_start)
                                      : (uint64_t)ar_lo + (hl - ar_start);
            ce = (cin && rlive ? kl64 : s.cell_ent)[rlive ? cidx : 0u];
            if (rwide)
            {
                // element hl + LPR of the wide range round
                const uint32_t x1 = hl + LPR;
#pragma unroll
                for (uint32_t p = 1; p < LEAN_MAXP; ++p)
                {
                    const uint32_t sp = seg_lane(rstart, p);
                    if (p < np && x1 >= sp) ar1 = p;
                }
                const uint32_t rsrc1 = sb | ar1;
                const uint32_t ar1_start = __shfl(rstart, rsrc1, 64), ar1_lo = __shfl(cbc.x, rsrc1, 64);
                const uint32_t ar1_meta = __shfl(has_cfk ? meta : 0u, rsrc1, 64), ar1_slot = __shfl(Hc.slot, rsrc1, 64);
                const bool cin1 = (ar1_meta & KL_CELLINL) != 0;
                rlive1 = act && x1 < TR;
                const uint64_t cidx1 = cin1 ? (uint64_t)ar1_slot * (sizeof(KeyLine) / 8) + offsetof(KeyLine, inl) / 8 +
                                                  ((ar1_meta >> KL_CELL_SHIFT) & 7u) + (x1 - ar1_start)
                                            : (uint64_t)ar1_lo + (x1 - ar1_start);
                ce1 = (cin1 && rlive1 ? kl64 : s.cell_ent)[rlive1 ? cidx1 : 0u];
            }
        }

        const uint32_t txw = !live ? 0u : ((from_cand || cls != 0) ? lv : (a_lw | (1u << RANK_BITS)));
        const uint32_t r = txw & RANK_MASK, kd = txw >> RANK_BITS;
        const bool want = live && r != self && r < S;
        const bool is1 = ((KINDS_RS_OR_WS >> kd) & 1) == 0;       // !managesExecution -> directKeyDeps
        const int64_t key = keyc;

        // ---- keyDeps (m = 0) and directKeyDeps (m = 2)
        for (int m = 0; m < 3; m += 2)
        {
            const bool mine = want && (m == 0 ? !is1 : is1);
            const uint64_t mb = ballot(mine);
            const uint32_t tot = __popcll(seg(mb));
            if (mb == 0)
            {
                put_sizes(act, t, m, 0, 0, 0, 0, false);
                continue;
            }
            // sort (rank, key) per request; dedup -> txnIds; body = unique-rank index per key, ascending
            uint32_t k = mine ? ((r << 3) | a) : 0xFFFFFFFFu;
            // the sort must span every lane that may hold one (raw emissions: lanes [0, T))
            // (a deferred request of the wave may hold T > LPR: never sort across segments)
            const uint32_t kmax = min(seg_max(T), LPR);
            if (kmax <= 8) seg_bitonic<8, LPR>(k);
            else if (kmax <= 16 || LPR == 16) seg_bitonic<16, LPR>(k);
            else if (kmax <= 32 || LPR == 32) seg_bitonic<(LPR < 32 ? LPR : 32), LPR>(k);
            else seg_bitonic<LPR, LPR>(k);
            const bool valid = hl < tot;
            const uint32_t xr = k >> 3, ka = k & 7u;
            const uint32_t prev = wave_up1(k);
            const bool uniq = valid && (hl == 0 || (prev >> 3) != xr);
            // index of this lane's value among the distinct values: uniques up to and including this
            // lane, minus one (equal values sit in adjacent lanes)
            const uint64_t um = seg(ballot(uniq));
            const uint32_t U = __popcll(um);
            const uint32_t ur = __popcll(um & below) + (uniq ? 1u : 0u) - 1u;
            uint64_t same = ballot(valid);
#pragma unroll
            for (int bit = 0; bit < 3; ++bit)
            {
                const uint64_t bb = ballot((ka >> bit) & 1u);
                same &= ((ka >> bit) & 1u) ? bb : ~bb;
            }
            const uint32_t pos_in_key = __popcll(seg(same) & below);
            // per key p (lanes hl < 8): its number of values = its map-m emissions, counted over its
            // raw lane range [start, start + nn) (a key's list holds distinct txnIds), then body
            // starts and heads
            const uint64_t rmask = nn >= 64 ? ~0ull : (((1ull << nn) - 1) << start);
            const uint32_t cnt = hl < 8 ? (uint32_t)__popcll(seg(mb) & rmask) : 0u;
            uint32_t cinc = cnt;
#pragma unroll
            for (uint32_t d = 1; d < 8; d <<= 1)
            {
                const uint32_t v = row_up(cinc, d);
                if ((hl & 7) >= d) cinc += v;
            }
            const uint32_t kstart_l = cinc - cnt;
            const uint64_t nem = seg(ballot(hl < 8 && cnt > 0));
            const uint32_t nk = __popcll(nem);
            const uint32_t kk = __popcll(nem & below);
            const uint32_t kstart = __shfl(kstart_l, sb | ka, 64);
            // regions of the wave's requests from one wave-uniform allocation
            const uint64_t bytes = act && tot ? (((uint64_t)nk * 8 + (uint64_t)U * 4 + (uint64_t)(nk + tot) * 4 + 7) & ~7ull) : 0;
            bool fits;
            const uint64_t ro = seg_alloc(bytes, fits, it);
            put_sizes(act, t, m, fits ? nk : 0, fits ? U : 0, fits ? nk + tot : 0, ro, true);
            if (act && tot && fits)
            {
                int64_t* okeys = reinterpret_cast<int64_t*>(b.reg + ro);
                uint32_t* otx = reinterpret_cast<uint32_t*>(okeys + nk);
                int32_t* ok2t = reinterpret_cast<int32_t*>(otx + U);
                if (hl < 8 && cnt > 0)
                {
                    okeys[kk] = key;
                    ok2t[kk] = (int32_t)(nk + kstart_l + cnt);     // absolute end offsets (RelationMultiMap.java:245-257)
                }
                if (uniq) otx[ur] = (xr - 1) >> 1;                  // dictionary index of the TxnId
                if (valid) ok2t[nk + kstart + pos_in_key] = (int32_t)ur;
            }
        }
        // ---- rangeDeps (m = 1): (range, txnId) pairs of the cells, STARTED_BEFORE (txnId < S), kind
        // witnessed, not self; unique pairs in (Range.compare, TxnId) order
        const uint32_t rtxw = (uint32_t)ce, rk = rtxw & RANK_MASK, rkd = rtxw >> RANK_BITS;
        const bool rwant = RNG && rlive && ((CLASS_KINDS[cls] >> rkd) & 1) && rk < S && rk != self;
        const uint32_t rtxw1 = (uint32_t)ce1, rk1 = rtxw1 & RANK_MASK, rkd1 = rtxw1 >> RANK_BITS;
        const bool rwant1 = RNG && rwide && rlive1 && ((CLASS_KINDS[cls] >> rkd1) & 1) && rk1 < S && rk1 != self;
        const uint64_t rmb = ballot(rwant), rmb1 = RNG && rwide ? ballot(rwant1) : 0ull;
        if (!RNG || (rmb | rmb1) == 0)
        {
            put_sizes(act, t, 1, 0, 0, 0, 0, false);
        }
        else if (RNG && rwide)
        {
            // the 32-bit range round below over 2 x LPR elements (element hl in register 0, hl + LPR in 1): sort
            // (range id << 6 | element), keep the run of each range group's first key, then the distinct
            // txnIds by (rank << 6 | pair position)
            const uint32_t LW = LPR;
            uint32_t k1a = rwant ? ((uint32_t)(ce >> 32) << 6) | hl : 0xFFFFFFFFu;
            uint32_t k1b = rwant1 ? ((uint32_t)(ce1 >> 32) << 6) | (hl + LW) : 0xFFFFFFFFu;
            seg_bitonic_w<uint32_t, LPR>(k1a, k1b);
            const uint32_t totp = __popcll(seg(rmb)) + __popcll(seg(rmb1));
            const bool pva = hl < totp, pvb = hl + LW < totp;
            const uint32_t rida = k1a >> 6, ridb = k1b >> 6;
            // the pair's rank and key: element e of register e / LPR at lane e % LPR
            const uint32_t va0 = (rk << 3) | ar, va1 = (rk1 << 3) | ar1;
            auto elem = [&](uint32_t e, bool on) -> uint32_t {
                const int src = (int)(on ? (sb | (e & (LW - 1))) : lane);
                const uint32_t x0 = (uint32_t)__shfl((int)va0, src, 64), x1 = (uint32_t)__shfl((int)va1, src, 64);
                return (e & LW) ? x1 : x0;
            };
            const uint32_t rkaa = elem(k1a & 63u, pva), rkab = elem(k1b & 63u, pvb);
            const uint32_t lasta = (uint32_t)__shfl((int)rida, (int)(sb | (LW - 1)), 64);
            const uint32_t prida = wave_up1(rida);
            const uint32_t upb = wave_up1(ridb);
            const uint32_t pridb = hl == 0 ? lasta : upb;
            const bool gfra = pva && (hl == 0 || prida != rida), gfrb = pvb && pridb != ridb;
            // each element's range group start (its encoded position: lane, or 64 + lane in register 1); the
            // segment's first element starts a group, so register 0's absolute-lane max scan stays in the segment
            const uint32_t gsa = wave_incl_max_dpp(gfra ? lane : 0u);
            const uint32_t gsb_scan = wave_incl_max_dpp(gfrb ? 64u + lane : 0u);
            const uint32_t carry = (uint32_t)__shfl((int)gsa, (int)(sb | (LW - 1)), 64);
            const uint32_t gsb = (gsb_scan >= 64u + sb) ? gsb_scan : carry;
            auto key_at = [&](uint32_t g) -> uint32_t {
                const int src = (int)(g & 63u);
                const uint32_t x0 = (uint32_t)__shfl((int)(rkaa & 7u), src, 64), x1 = (uint32_t)__shfl((int)(rkab & 7u), src, 64);
                return g >= 64u ? x1 : x0;
            };
            const uint32_t ar0a = key_at(gsa), ar0b = key_at(gsb);
            const bool pua = pva && (rkaa & 7u) == ar0a, pub = pvb && (rkab & 7u) == ar0b;
            const uint64_t puma = seg(ballot(pua)), pumb = seg(ballot(pub));
            const uint32_t npa = __popcll(puma);
            const uint32_t UP = npa + __popcll(pumb);
            const uint32_t dsta = __popcll(puma & below), dstb = npa + __popcll(pumb & below);
            const bool gfa = pua && gfra, gfb = pub && gfrb;
            const uint64_t gma = seg(ballot(gfa)), gmb = seg(ballot(gfb));
            const uint32_t nR = __popcll(gma) + __popcll(gmb);
            uint32_t k2a = pua ? ((rkaa >> 3) << 6) | dsta : 0xFFFFFFFFu;
            uint32_t k2b = pub ? ((rkab >> 3) << 6) | dstb : 0xFFFFFFFFu;
            seg_bitonic_w<uint32_t, LPR>(k2a, k2b);
            const uint32_t last2 = (uint32_t)__shfl((int)k2a, (int)(sb | (LW - 1)), 64);
            const uint32_t p2a = wave_up1(k2a);
            const uint32_t up2b = wave_up1(k2b);
            const uint32_t p2b = hl == 0 ? last2 : up2b;
            const bool v2a = hl < UP, v2b = hl + LW < UP;
            const bool uqa = v2a && (hl == 0 || (p2a >> 6) != (k2a >> 6)), uqb = v2b && (p2b >> 6) != (k2b >> 6);
            const uint64_t uma = seg(ballot(uqa)), umb = seg(ballot(uqb));
            const uint32_t nua = __popcll(uma);
            const uint32_t UR = nua + __popcll(umb);
            const uint32_t ura = __popcll(uma & below) + (uqa ? 1u : 0u) - 1u;
            const uint32_t urb = nua + __popcll(umb & below) + (uqb ? 1u : 0u) - 1u;
            const uint64_t bytes = act && totp ? (((uint64_t)nR * 8 + (uint64_t)UR * 4 + (uint64_t)(nR + UP) * 4 + 7) & ~7ull) : 0;
            bool fits;
            const uint64_t ro = seg_alloc(bytes, fits, it);
            put_sizes(act, t, 1, fits ? nR : 0, fits ? UR : 0, fits ? nR + UP : 0, ro, true);
            if (act && totp && fits)
            {
                int64_t* okeys = reinterpret_cast<int64_t*>(b.reg + ro);
                uint32_t* otx = reinterpret_cast<uint32_t*>(okeys + nR);
                int32_t* ok2t = reinterpret_cast<int32_t*>(otx + UR);
                // 2 LPR-bit masks over the elements in order: register 0's lanes, then register 1's
                const uint32_t GM = (uint32_t)gma | ((uint32_t)gmb << LW), PUM = (uint32_t)puma | ((uint32_t)pumb << LW);
                auto group_end = [&](uint32_t e) -> uint32_t {
                    const uint32_t later = GM & ~((2u << e) - 1u);
                    const uint32_t nxt = later ? (uint32_t)(__ffs(later) - 1) : 0u;
                    return later ? (uint32_t)__popc(PUM & ((1u << nxt) - 1u)) : UP;
                };
                if (gfa)
                {
                    const uint32_t gi = __popcll(gma & below);
                    okeys[gi] = (int64_t)rida;                         // range id (ad_range_table)
                    ok2t[gi] = (int32_t)(nR + group_end(hl));
                }
                if (gfb)
                {
                    const uint32_t gi = __popcll(gma) + __popcll(gmb & below);
                    okeys[gi] = (int64_t)ridb;
                    ok2t[gi] = (int32_t)(nR + group_end(hl + LW));
                }
                if (uqa) otx[ura] = ((k2a >> 6) - 1) >> 1;
                if (uqb) otx[urb] = ((k2b >> 6) - 1) >> 1;
                if (v2a) ok2t[nR + (k2a & 63u)] = (int32_t)ura;
                if (v2b) ok2t[nR + (k2b & 63u)] = (int32_t)urb;
            }
        }
        else if (s.rng32)
        {
            // 32-bit keys. Every entry of a range id covers the same interval, so each cell holding the id
            // holds all its entries (in txnId order): a request's pairs of one range id are identical runs,
            // one per key whose cell has it. Sort (range id << 6 | lane) -- range-major, then by key and
            // txnId within a key's run -- and keep the run of the group's first key (the duplicates of the
            // 64-bit sort); then the distinct txnIds by (rank << 6 | pair position).
            const uint32_t kmaxr = min(seg_max(TR), LPR);
            uint32_t k1 = rwant ? ((uint32_t)(ce >> 32) << 6) | hl : 0xFFFFFFFFu;
            if (kmaxr <= 8) seg_bitonic<8, LPR>(k1);
            else if (kmaxr <= 16 || LPR == 16) seg_bitonic<16, LPR>(k1);
            else if (kmaxr <= 32 || LPR == 32) seg_bitonic<(LPR < 32 ? LPR : 32), LPR>(k1);
            else seg_bitonic<LPR, LPR>(k1);
            const uint32_t totp = __popcll(seg(rmb));
            const bool pv = hl < totp;
            const uint32_t rid = k1 >> 6, src = sb | (k1 & 63u);
            // the pair's rank and key (its source lane)
            const uint32_t rka = (uint32_t)__shfl((int)((rk << 3) | ar), (int)(pv ? src : lane), 64);
            const uint32_t prid = wave_up1(rid);
            const bool gfirst_raw = pv && (hl == 0 || prid != rid);
            // the key of the range id's first run (segment starts are group starts: an absolute-lane max scan)
            const uint32_t gs = wave_incl_max_dpp(gfirst_raw ? lane : 0u);
            const uint32_t ar0 = (uint32_t)__shfl((int)(rka & 7u), (int)gs, 64);
            const bool pu = pv && (rka & 7u) == ar0;
            const uint64_t pum = seg(ballot(pu));
            const uint32_t UP = __popcll(pum);
            const uint32_t dst = __popcll(pum & below);
            const bool gfirst = pu && gfirst_raw;
            const uint64_t gm = seg(ballot(gfirst));
            const uint32_t nR = __popcll(gm);
            // distinct txnIds of the unique pairs: sort (rank << 6 | pair position)
            uint32_t k2 = pu ? ((rka >> 3) << 6) | dst : 0xFFFFFFFFu;
            if (kmaxr <= 8) seg_bitonic<8, LPR>(k2);
            else if (kmaxr <= 16 || LPR == 16) seg_bitonic<16, LPR>(k2);
            else if (kmaxr <= 32 || LPR == 32) seg_bitonic<(LPR < 32 ? LPR : 32), LPR>(k2);
            else seg_bitonic<LPR, LPR>(k2);
            const uint32_t p2 = wave_up1(k2);
            const bool v2 = hl < UP;
            const bool uq2 = v2 && (hl == 0 || (p2 >> 6) != (k2 >> 6));
            const uint64_t um2 = seg(ballot(uq2));
            const uint32_t UR = __popcll(um2);
            const uint32_t ur2 = __popcll(um2 & below) + (uq2 ? 1u : 0u) - 1u;
            const uint64_t bytes = act && totp ? (((uint64_t)nR * 8 + (uint64_t)UR * 4 + (uint64_t)(nR + UP) * 4 + 7) & ~7ull) : 0;
            bool fits;
            const uint64_t ro = seg_alloc(bytes, fits, it);
            put_sizes(act, t, 1, fits ? nR : 0, fits ? UR : 0, fits ? nR + UP : 0, ro, true);
            if (act && totp && fits)
            {
                int64_t* okeys = reinterpret_cast<int64_t*>(b.reg + ro);
                uint32_t* otx = reinterpret_cast<uint32_t*>(okeys + nR);
                int32_t* ok2t = reinterpret_cast<int32_t*>(otx + UR);
                if (gfirst)
                {
                    // this group's end: the pair position of the next group's first pair (or UP)
                    const uint32_t gi = __popcll(gm & below);
                    const uint64_t later = gm & ~((2ull << hl) - 1) & SEGMASK;
                    const uint32_t nxt = later ? (uint32_t)(__ffsll((unsigned long long)later) - 1) : LPR;
                    const uint32_t gend = later ? __popcll(pum & ((1ull << nxt) - 1)) : UP;
                    okeys[gi] = (int64_t)rid;                          // range id (ad_range_table)
                    ok2t[gi] = (int32_t)(nR + gend);
                }
                if (uq2) otx[ur2] = ((k2 >> 6) - 1) >> 1;
                if (v2) ok2t[nR + (k2 & 63u)] = (int32_t)ur2;
            }
        }
        else
        {
            const uint32_t kmaxr = min(seg_max(TR), LPR);
            uint64_t pk = rwant ? ((ce & 0xFFFFFFFF00000000ull) | rk) : ~0ull;
            if (kmaxr <= 8) seg_bitonic64<8, LPR>(pk);
            else if (kmaxr <= 16 || LPR == 16) seg_bitonic64<16, LPR>(pk);
            else if (kmaxr <= 32 || LPR == 32) seg_bitonic64<(LPR < 32 ? LPR : 32), LPR>(pk);
            else seg_bitonic64<LPR, LPR>(pk);
            const uint32_t totp = __popcll(seg(rmb));
            const bool pv = hl < totp;
            const uint64_t pprev = (((uint64_t)wave_up1((uint32_t)(pk >> 32)) << 32) | wave_up1((uint32_t)pk))
                                           ;
            const bool pu = pv && (hl == 0 || pprev != pk);
            const uint64_t pum = seg(ballot(pu));
            const uint32_t UP = __popcll(pum);
            // the unique pairs, compacted to the first UP lanes of the segment
            const uint32_t dst = __popcll(pum & below);
            uint64_t up = ~0ull;
            {
                // lane dst takes the pair of this lane (ds_permute pushes). Lanes without a unique
                // pair push to the segment's last lane, which is read only when all LPR pairs are
                // unique, i.e. when there are no such lanes
                const uint32_t my = pu ? dst : LPR - 1;
                const int addr = (int)((sb + my) << 2);
                const uint32_t lo32 = __builtin_amdgcn_ds_permute(addr, (int)(uint32_t)pk);
                const uint32_t hi32 = __builtin_amdgcn_ds_permute(addr, (int)(uint32_t)(pk >> 32));
                if (hl < UP) up = ((uint64_t)hi32 << 32) | lo32;
            }
            const bool uplive = hl < UP;
            const uint32_t rid = (uint32_t)(up >> 32), urk = (uint32_t)up;
            const uint32_t prid = wave_up1(rid);
            const bool gfirst = uplive && (hl == 0 || prid != rid);
            const uint64_t gm = seg(ballot(gfirst));
            const uint32_t nR = __popcll(gm);
            // distinct txnIds of the pairs: sort (rank, pair index)
            uint64_t k2 = uplive ? (((uint64_t)urk << 8) | hl) : ~0ull;
            if (kmaxr <= 8) seg_bitonic64<8, LPR>(k2);
            else if (kmaxr <= 16 || LPR == 16) seg_bitonic64<16, LPR>(k2);
            else if (kmaxr <= 32 || LPR == 32) seg_bitonic64<(LPR < 32 ? LPR : 32), LPR>(k2);
            else seg_bitonic64<LPR, LPR>(k2);
            const uint64_t p2 = (((uint64_t)wave_up1((uint32_t)(k2 >> 32)) << 32) | wave_up1((uint32_t)k2))
                                        ;
            const bool v2 = hl < UP;
            const bool uq2 = v2 && (hl == 0 || (uint32_t)(p2 >> 8) != (uint32_t)(k2 >> 8));
            const uint64_t um2 = seg(ballot(uq2));
            const uint32_t UR = __popcll(um2);
            const uint32_t ur2 = __popcll(um2 & below) + (uq2 ? 1u : 0u) - 1u;
            const uint64_t bytes = act && totp ? (((uint64_t)nR * 8 + (uint64_t)UR * 4 + (uint64_t)(nR + UP) * 4 + 7) & ~7ull) : 0;
            bool fits;
            const uint64_t ro = seg_alloc(bytes, fits, it);
            put_sizes(act, t, 1, fits ? nR : 0, fits ? UR : 0, fits ? nR + UP : 0, ro, true);
            if (act && totp && fits)
            {
                int64_t* okeys = reinterpret_cast<int64_t*>(b.reg + ro);
                uint32_t* otx = reinterpret_cast<uint32_t*>(okeys + nR);
                int32_t* ok2t = reinterpret_cast<int32_t*>(otx + UR);
                if (gfirst)
                {
                    const uint32_t gi = __popcll(gm & below);
                    const uint64_t later = gm & ~((2ull << hl) - 1) & SEGMASK;
                    const uint32_t gend = later ? (uint32_t)(__ffsll((unsigned long long)later) - 1) : UP;
                    okeys[gi] = (int64_t)rid;                          // range id (ad_range_table)
                    ok2t[gi] = (int32_t)(nR + gend);
                }
                if (uq2) otx[ur2] = ((uint32_t)(k2 >> 8) - 1) >> 1;
                if (v2) ok2t[nR + (uint32_t)(k2 & 0xFF)] = (int32_t)ur2;
            }
        }
    };
    for (uint32_t it = it0;;)
    {
        if (it >= n_items) break;
        step(it, PA, PB);
        it += nw;
        if (it >= n_items) break;
        step(it, PB, PA);
        it += nw;
    }
    dflush();
    if (WIDE && PASS == 1 && nwide && lane == 0) atomicAdd(&b.ctl->n_wide1, (unsigned long long)nwide);
}

template <uint32_t RPW, bool RNG, bool WIDE, int PASS>
static hipError_t launch_lean(const DevSnapshot& s, const BatchBufs& b, hipStream_t st)
{
    static int per_cu = 0;
    if (!per_cu)
    {
        int nb = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_resolve_lean<RPW, RNG, WIDE, PASS>, 64 * LEAN_WAVES, 0) != hipSuccess ||
            nb <= 0)
            nb = 2;
        per_cu = std::min(nb, lean_occ<RNG, WIDE>());     // measured: more resident waves only add memory contention
    }
    const uint64_t need = ((b.n_txns + RPW - 1) / RPW + LEAN_WAVES - 1) / LEAN_WAVES;
    const unsigned grid = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(need, (uint64_t)device_cu_count() * per_cu));
    k_resolve_lean<RPW, RNG, WIDE, PASS><<<grid, 64 * LEAN_WAVES, 0, st>>>(s, b);
    return hipGetLastError();
}

// pass 1: every request, two per wave -> D1; pass 2: D1, two per wave with two emissions per lane
// (one per wave with range commands; up to 64 emissions) -> D2
hipError_t run_resolve_lean(const DevSnapshot& s, const BatchBufs& b, int pass, uint32_t rpw1, bool wide1, hipStream_t st)
{
    if (!b.n_txns) return hipSuccess;
    if (pass == 1)
    {
        if (!b.p_slot) return hipErrorInvalidValue;     // k_prepare writes the probes' lines
        if (rpw1 == 8) return s.n_rent ? launch_lean<8, true, false, 1>(s, b, st) : launch_lean<8, false, false, 1>(s, b, st);
        if (rpw1 == 4) return s.n_rent ? launch_lean<4, true, false, 1>(s, b, st) : launch_lean<4, false, false, 1>(s, b, st);
        if (wide1 && !s.n_rent) return launch_lean<2, false, true, 1>(s, b, st);
        return s.n_rent ? launch_lean<2, true, false, 1>(s, b, st) : launch_lean<2, false, false, 1>(s, b, st);
    }
    // pass 2 (requests with 33..64 raw emissions): two per wave, two emissions per lane; with range commands
    // one per wave after a pass 1 of two per wave, two per wave (up to 32) after one of four
    if (s.n_rent) return rpw1 == 4 ? launch_lean<2, true, false, 2>(s, b, st) : launch_lean<1, true, false, 2>(s, b, st);
    return launch_lean<2, false, true, 2>(s, b, st);
}


}  // namespace adx
