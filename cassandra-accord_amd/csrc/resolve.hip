// resolve.hip — the fused per-request kernel of the dependency-resolution path (gfx950).
//
// One wave resolves one PreAccept.calculatePartialDeps request end to end (PreAccept.java:245-267):
//   encode    executeAt/txnId -> dictionary ranks (64-ary wave search), keys -> CommandsForKey
//             index (open-addressing hash, one probe)
//   K1        CommandsForKey.mapReduceActive (CommandsForKey.java:910-968) for up to 8 keys at
//             once: lanes 8g..8g+7 serve key g (8-ary searches, 64-ary max-tree descent with
//             8 nodes per lane, ballot/prefix compaction into LDS)
//   K4        mapReduceRangesInternal (InMemoryCommandStore.java:884-1017) + RedundantBefore
//             .collectDeps (RedundantBefore.java:183-192), same group scheme
//   K2        Deps.AbstractBuilder.add / RelationMultiMap build / PartialDeps.with as the LDS
//             multi-list union of kernels.hip, written to a chunk-allocated region
// Requests with more than 8 keys or with a per-key output beyond the LDS staging are deferred
// to the general split kernels (kernels.hip), which handle any size.
#include <hip/hip_runtime.h>

#include "common.hpp"
#include "kernels.hpp"
#include "wave.hpp"

namespace adx {

constexpr int FMAXP = 8;        // keys per request on the fused path (one 8-lane group each)
constexpr int FCAP0 = 64;       // keyDeps txnIds staged per key
constexpr int FCAP1 = 16;       // directKeyDeps txnIds staged per key
constexpr int FCAPR = 32;       // range-command pairs staged per key (+1 slot: redundant pair)
constexpr int FWAVES = 4;       // waves per workgroup
#ifndef FUSED_WPE
#define FUSED_WPE 4          // waves per SIMD the general kernel's register budget is sized for
#endif
constexpr uint32_t F_REGION_CHUNK = 1u << 14;   // region bytes per refill (small: the arena stays dense)

struct FusedLds {
    uint32_t st0[FMAXP][FCAP0];
    uint32_t st1[FMAXP][FCAP1];
    uint64_t rs[FMAXP][FCAPR + 1];
    uint64_t stk[FMAXP][2 * MAX_LEVELS];
    int64_t key[FMAXP];
};

// ascending bitonic sort of one u64 key per lane over lanes [0, KMAX) (and independently over
// each further block of KMAX lanes): lanes >= n hold ~0, so sorting only the first 16 or 32 lanes
// when n fits saves stages
template <uint32_t KMAX>
__device__ __forceinline__ void bitonic_lanes(uint64_t& key)
{
    const uint32_t l = lane_id();
#pragma unroll
    for (uint32_t k = 2; k <= KMAX; k <<= 1)
#pragma unroll
        for (uint32_t j = k >> 1; j > 0; j >>= 1)
        {
            const uint64_t ok = __shfl_xor(key, (int)j, 64);
            const bool up = (l & k) == 0;
            const bool lower = (l & j) == 0;
            const bool take = lower ? (up ? ok < key : ok > key) : (up ? ok > key : ok < key);
            if (take) key = ok;
        }
}

template <uint32_t KMAX>
__device__ __forceinline__ void bitonic_lanes32(uint32_t& key)
{
    const uint32_t l = lane_id();
#pragma unroll
    for (uint32_t k = 2; k <= KMAX; k <<= 1)
#pragma unroll
        for (uint32_t j = k >> 1; j > 0; j >>= 1)
        {
            const uint32_t ok = __shfl_xor(key, (int)j, 64);
            const bool up = (l & k) == 0;
            const bool lower = (l & j) == 0;
            key = (lower == up) ? min(key, ok) : max(key, ok);
        }
}

__device__ __forceinline__ void wave_bitonic32(uint32_t& key, uint32_t n)
{
    if (n <= 16) bitonic_lanes32<16>(key);
    else if (n <= 32) bitonic_lanes32<32>(key);
    else bitonic_lanes32<64>(key);
}

// sort the n (wave-uniform) live keys held in lanes [0, n); the other lanes hold ~0
__device__ __forceinline__ void wave_bitonic64(uint64_t& key, uint32_t n)
{
    if (n <= 16) bitonic_lanes<16>(key);
    else if (n <= 32) bitonic_lanes<32>(key);
    else bitonic_lanes<64>(key);
}

__device__ __forceinline__ void set_error_f(BatchCtl* ctl, unsigned code) { atomicCAS(&ctl->error, 0u, code); }

// ---- group (8-lane) helpers --------------------------------------------------------------
__device__ __forceinline__ uint32_t grp_bits(uint64_t m, uint32_t g) { return (uint32_t)(m >> (8 * g)) & 0xFFu; }

__device__ __forceinline__ uint32_t grp_incl_scan(uint32_t v)
{
    const uint32_t j = lane_id() & 7;
#pragma unroll
    for (int d = 1; d < 8; d <<= 1)
    {
        const uint32_t t = __shfl_up(v, d, 8);
        if (j >= (uint32_t)d) v += t;
    }
    return v;
}

__device__ __forceinline__ uint32_t grp_sum(uint32_t v)
{
    v += __shfl_xor(v, 1, 64);
    v += __shfl_xor(v, 2, 64);
    v += __shfl_xor(v, 4, 64);
    return v;
}

__device__ __forceinline__ uint64_t grp_or64(uint64_t v)
{
    v |= __shfl_xor(v, 1, 64);
    v |= __shfl_xor(v, 2, 64);
    v |= __shfl_xor(v, 4, 64);
    return v;
}

// lower_bound over key(i), i in [lo, hi), by the 8 lanes of each active group (8-ary rounds);
// groups proceed independently, the wave loops until every group is done
template <class KeyAt, class Less>
__device__ __forceinline__ uint64_t grp_lower_bound(bool active, uint64_t lo, uint64_t hi, KeyAt key, Less less)
{
    const uint32_t j = lane_id() & 7, g = lane_id() >> 3;
    while (ballot(active && hi - lo > 8))
    {
        if (active && hi - lo > 8)
        {
            const uint64_t n = hi - lo;
            const uint64_t p = lo + (((uint64_t)(j + 1) * n) >> 3) - 1;
            const bool lt = less(key(p));
            const uint32_t c = __popc(grp_bits(ballot(lt), g));
            if (c == 8) lo = hi;
            else
            {
                const uint64_t pc = lo + (((uint64_t)(c + 1) * n) >> 3) - 1;
                const uint64_t nlo = c == 0 ? lo : lo + (((uint64_t)c * n) >> 3);
                lo = nlo;
                hi = pc;
            }
        }
    }
    const uint64_t i = lo + j;
    const bool v = active && i < hi && less(key(i));
    return lo + __popc(grp_bits(ballot(v), g));
}

// Two lower_bounds of one threshold (key(i) < x) by the same 8-lane groups, advanced in lockstep:
// both rounds' loads are in flight together, so the pair costs one search's chain of round trips
template <class KeyA, class KeyB>
__device__ __forceinline__ void grp_lower_bound2(bool act_a, uint64_t lo_a, uint64_t hi_a, KeyA key_a, bool act_b,
                                                 uint64_t lo_b, uint64_t hi_b, KeyB key_b, uint32_t x,
                                                 uint64_t& out_a, uint64_t& out_b)
{
    const uint32_t j = lane_id() & 7, g = lane_id() >> 3;
    auto step = [&](bool on, bool lt, uint64_t& lo, uint64_t& hi) {
        const uint32_t c = __popc(grp_bits(ballot(lt), g));
        if (!on) return;
        const uint64_t n = hi - lo;
        if (c == 8) lo = hi;
        else
        {
            const uint64_t pc = lo + (((uint64_t)(c + 1) * n) >> 3) - 1;
            lo = c == 0 ? lo : lo + (((uint64_t)c * n) >> 3);
            hi = pc;
        }
    };
    // one galloping round from the tail first: lane j probes hi - 8^(j+1), so an answer within 8^k of the end
    // (a late PreAccept's insertPos, an Accept's last committed Write) is left in a window of 8^k after one
    // round trip, k more rounds to go -- instead of the log8 of the key's whole segment
    auto gallop = [&](bool on, bool lt, uint64_t p_lane, uint64_t& lo, uint64_t& hi) {
        const uint32_t bits = grp_bits(ballot(lt), g);      // ascending j = descending position: 1...10...0 (lt)
        const uint32_t c = __popc(~bits & 0xFFu);           // probes at or above x (nearest the tail)
        const uint32_t gl = lane_id() & ~7u;
        const uint64_t p_lt = __shfl(p_lane, gl + (c < 8 ? c : 7u), 64);          // nearest probe below x
        const uint64_t p_ge = __shfl(p_lane, gl + (c > 0 ? c - 1 : 0u), 64);      // farthest probe at or above x
        if (!on) return;
        if (c < 8) lo = p_lt + 1;
        if (c > 0) hi = p_ge;
    };
    {
        const bool ga = act_a && hi_a - lo_a > 64, gb = act_b && hi_b - lo_b > 64;
        if (ballot(ga || gb))
        {
            const uint64_t sp = 1ull << (3 * (j + 1));
            const uint64_t pa = ga ? hi_a - (sp < hi_a - lo_a ? sp : hi_a - lo_a) : 0;
            const uint64_t pb = gb ? hi_b - (sp < hi_b - lo_b ? sp : hi_b - lo_b) : 0;
            const uint32_t va = ga ? key_a(pa) : 0u, vb = gb ? key_b(pb) : 0u;
            gallop(ga, ga && va < x, pa, lo_a, hi_a);
            gallop(gb, gb && vb < x, pb, lo_b, hi_b);
        }
    }
    while (ballot((act_a && hi_a - lo_a > 8) || (act_b && hi_b - lo_b > 8)))
    {
        const bool sa = act_a && hi_a - lo_a > 8, sb = act_b && hi_b - lo_b > 8;
        const uint64_t pa = sa ? lo_a + (((uint64_t)(j + 1) * (hi_a - lo_a)) >> 3) - 1 : 0;
        const uint64_t pb = sb ? lo_b + (((uint64_t)(j + 1) * (hi_b - lo_b)) >> 3) - 1 : 0;
        const uint32_t va = sa ? key_a(pa) : 0u, vb = sb ? key_b(pb) : 0u;
        step(sa, sa && va < x, lo_a, hi_a);
        step(sb, sb && vb < x, lo_b, hi_b);
    }
    const uint64_t ia = lo_a + j, ib = lo_b + j;
    const bool la = act_a && ia < hi_a, lb = act_b && ib < hi_b;
    const uint32_t va = la ? key_a(ia) : 0u, vb = lb ? key_b(ib) : 0u;
    out_a = lo_a + __popc(grp_bits(ballot(la && va < x), g));
    out_b = lo_b + __popc(grp_bits(ballot(lb && vb < x), g));
}

// Group-parallel max-tree descent: like wave_descent, but each 8-lane group walks its own
// range [lo, end) and every lane evaluates 8 consecutive nodes (leaves) of a 64-wide frame.
//   node_bits(lv, n0, nlo, nhi) -> 8-bit want mask of nodes n0..n0+7 (within [nlo, nhi])
//   leaf(n0)                    -> emission for leaves n0..n0+7 (group-collective)
template <class NodeBits, class Leaf>
__device__ __forceinline__ void grp_descent(bool active, uint64_t lo, uint64_t end, int n_levels, NodeBits node_bits,
                                            Leaf leaf, uint64_t* stk)
{
    const uint32_t j = lane_id() & 7;
    bool done = !active || end <= lo;
    int k = 0;
    // start at the lowest level whose aligned 64-node frame holds the whole range
    if (!done)
        while (k + 1 < n_levels && (lo >> (6 * (k + 1))) != ((end - 1) >> (6 * (k + 1)))) ++k;
    int lv = k;
    uint64_t base = done ? 0 : (lo >> (6 * k)) & ~63ull;
    uint64_t mask = 0;
    bool eval = !done;
    while (ballot(!done))
    {
        if (!done)
        {
            if (eval)
            {
                eval = false;
                const uint64_t n0 = base + 8 * j;
                if (lv == 0)
                {
                    leaf(n0);
                    mask = 0;
                }
                else
                {
                    const uint64_t nlo = lo >> (6 * lv), nhi = (end - 1) >> (6 * lv);
                    const uint32_t bits = node_bits(lv, n0, nlo, nhi);
                    mask = grp_or64((uint64_t)bits << (8 * j));
                }
            }
            else if (mask == 0)
            {
                if (lv == k) done = true;
                else
                {
                    ++lv;
                    base = stk[2 * lv];
                    mask = stk[2 * lv + 1];
                }
            }
            else
            {
                const int b = __ffsll((unsigned long long)mask) - 1;
                mask &= mask - 1;
                stk[2 * lv] = base;
                stk[2 * lv + 1] = mask;
                base = (base + b) << 6;
                --lv;
                eval = true;
            }
        }
    }
}

// 64-ary wave search of the dictionary: rank of an arbitrary id (member i -> 2i+1, else 2*lb)
__device__ __forceinline__ uint32_t wave_dict_rank(const DevSnapshot& s, uint64_t msb, uint64_t lsb, int32_t node)
{
    const NormTid x = norm_tid(msb, lsb, node);
    auto key = [&](uint64_t i) { return NormTid{s.dict_hi[i], s.dict_lo[i], s.dict_node[i]}; };
    if (s.n_dict == 0) return 0;
    const NormTid last{s.dict_last_hi, s.dict_last_lo, s.dict_last_node};
    if (norm_cmp(last, x) < 0) return (uint32_t)(2 * s.n_dict);   // newer than every id (new txns): no load
    const uint64_t lb = wave_lower_bound(0, s.n_dict, key, [&](const NormTid& v) { return norm_cmp(v, x) < 0; });
    bool eq = false;
    if (lb < s.n_dict) eq = norm_cmp(key(lb), x) == 0;
    return (uint32_t)(2 * lb + (eq ? 1 : 0));
}

// ---- LDS multi-list union with 2-D list addressing ------------------------------------------





// cell of key x in the range stabbing index: #endpoints < x (EndInclusive) or <= x (StartInclusive)
__device__ __forceinline__ uint32_t cell_search(const DevSnapshot& s, int64_t x)
{
    if (!s.cell_off) return NO_CELL;
    uint64_t lo = 0, hi = s.n_cell_E;
    while (lo < hi)
    {
        const uint64_t mid = (lo + hi) >> 1;
        const int64_t v = s.cell_E[mid];
        if (s.start_inclusive ? v <= x : v < x) lo = mid + 1;
        else hi = mid;
    }
    return (uint32_t)lo;
}

__device__ __forceinline__ uint64_t fregion_bytes(uint32_t nk, uint32_t U, uint32_t pairs)
{
    return ((uint64_t)nk * 8 + (uint64_t)U * 4 + (uint64_t)(nk + pairs) * 4 + 7) & ~7ull;
}

struct FChunk {
    uint64_t cur = 0, end = 0;
    __device__ __forceinline__ uint64_t take(BatchCtl* ctl, uint64_t n)
    {
        if (n > end - cur)
        {
            const uint64_t sz = n > F_REGION_CHUNK ? n : F_REGION_CHUNK;
            unsigned long long base = 0;
            if (lane_id() == 0) base = atomicAdd(&ctl->reg_top, (unsigned long long)sz);
            base = uniform64(base);
            if (base + sz > ctl->reg_cap && lane_id() == 0) atomicOr(&ctl->overflow, 8u);
            cur = base;
            end = base + sz;
        }
        const uint64_t r = cur;
        cur += n;
        return r;
    }
};

// a Range-domain request the split kernels must resolve (see k_prepare)
__device__ __forceinline__ bool range_split(const DevSnapshot& s, const BatchBufs& b, uint64_t k0, uint64_t np)
{
    return b.p_kind && np && b.p_kind[k0] != PK_KEY && (s.n_rent || s.n_rb);
}

__global__ __launch_bounds__(64 * FWAVES) __attribute__((amdgpu_waves_per_eu(FUSED_WPE))) void k_resolve(DevSnapshot s, BatchBufs b)
{
    __shared__ FusedLds lds_all[FWAVES];
    FusedLds& L = lds_all[threadIdx.x >> 6];
    const uint32_t lane = lane_id(), g = lane >> 3, j = lane & 7;
    const uint64_t n = b.n_txns;
    const uint64_t nw = (uint64_t)gridDim.x * FWAVES;
    FChunk ralloc;
    const bool incl = s.start_inclusive != 0;
    const uint64_t reg_cap = uniform64(b.ctl->reg_cap);     // set by the host before the launch

    // Software pipeline over this wave's requests t0, t0 + nw, ...: key offsets two requests
    // ahead, ids / keys / slots one ahead (issued at the top of an iteration), the KeyEntry quarters
    // one ahead (issued once the current request's lists are staged), so a request's dependent
    // chain key_off -> slot -> KeyEntry -> lists is mostly hidden behind the previous request.
    // iteration index ii -> request: all requests, or those the lean kernel deferred
    const uint64_t n_iter = b.req_list ? uniform64(*b.req_count) : n;
    auto tof = [&](uint64_t ii) -> uint64_t { return b.req_list ? (uint64_t)b.req_list[ii] : ii; };
    auto st1 = [&](uint64_t ii, uint64_t& k0o, uint32_t& npo) {
        const uint64_t tt = ii < n_iter ? tof(ii) : (uint64_t)DEFER_HOLE;
        if (tt != DEFER_HOLE)
        {
            k0o = b.q_key_off[tt];
            npo = (uint32_t)(b.q_key_off[tt + 1] - k0o);
        }
        else { k0o = 0; npo = 0; }
    };
    struct Ids { uint64_t tm, tl, em, el; int32_t tn, en; };
    auto ids = [&](uint64_t ii) -> Ids {
        Ids r{0, 0, 0, 0, 0, 0};
        const uint64_t tt = ii < n_iter ? tof(ii) : (uint64_t)DEFER_HOLE;
        if (tt != DEFER_HOLE)
        {
            r.tm = b.q_txn_msb[tt]; r.tl = b.q_txn_lsb[tt]; r.tn = b.q_txn_node[tt];
            r.em = b.q_exec_msb[tt]; r.el = b.q_exec_lsb[tt]; r.en = b.q_exec_node[tt];
        }
        return r;
    };
    auto st2 = [&](uint64_t k0i, uint32_t npi, int64_t& keyo) {
        const bool a = g < npi && npi <= FMAXP;
        keyo = a ? b.q_keys[k0i + g] : 0;
    };
    // key -> (KeyEntry / KeyRec index | in-slice bit, stabbing cell): the slice test
    // (InMemoryCommandStore.java:280) and an open-addressing probe of the KeySlot table by the
    // group's 8 lanes at once (8 consecutive 16-byte slots = one line per round)
    auto probe = [&](uint64_t iix, uint32_t npi, int64_t key, uint32_t& pso, uint32_t& pco) {
        bool a = g < npi && npi <= FMAXP;
        // the request's slice (its slice set when the batch names them; iteration iix's request)
        const bool in_slice = a && slice_has(s.start_inclusive,
                                             b.q_slice_set ? request_slice(s, b.q_slice_set, tof(iix))
                                                           : SliceView{s.slice_start, s.slice_end, s.n_slices, s.n_slices == 0},
                                             key);
        uint32_t slot = SLOT_NONE, cell = NO_CELL;
        bool look = a && in_slice && s.n_keys != 0;
        uint64_t h = key_hash(key) & s.khash_mask;
        while (ballot(look))
        {
            const uint4 q = look ? reinterpret_cast<const uint4*>(s.khash + ((h + j) & s.khash_mask))[0] : make_uint4(0, 0, 0, 0);
            const bool hit = look && q.z != KEY_EMPTY && (int64_t)(((uint64_t)q.y << 32) | q.x) == key;
            const bool emp = look && q.z == KEY_EMPTY;
            const uint32_t hm = grp_bits(ballot(hit), g), em = grp_bits(ballot(emp), g);
            const uint32_t fh = hm ? (uint32_t)(__ffs(hm) - 1) : 8u, fe = em ? (uint32_t)(__ffs(em) - 1) : 8u;
            const uint32_t zs = __shfl(q.z, (lane & ~7u) | (fh & 7u), 64);      // every lane shuffles
            const uint32_t ws = __shfl(q.w, (lane & ~7u) | (fh & 7u), 64);
            if (look && fh < fe)
            {
                slot = zs;
                cell = ws;
            }
            if (look && (fh < 8 || fe < 8)) look = false;
            h += 8;
        }
        if (a && in_slice && slot == SLOT_NONE && s.cell_off) cell = cell_search(s, key);
        pso = !a ? SLOT_NONE : (in_slice ? (slot | SLOT_IN_SLICE) : SLOT_NONE);
        pco = (a && in_slice) ? cell : NO_CELL;
    };
    auto st3 = [&](uint32_t psi, uint4& kqo) {
        const uint32_t sl = psi & ~SLOT_IN_SLICE;
        // lanes 0-3: the KeyEntry (64 B); lanes 4-5: the KeyRec (32 B)
        kqo = make_uint4(0, 0, 0, 0);
        if (sl != SLOT_NONE && j < 4) kqo = reinterpret_cast<const uint4*>(s.kent + sl)[j];
        if (sl != SLOT_NONE && (j == 4 || j == 5)) kqo = reinterpret_cast<const uint4*>(s.krec + sl)[j - 4];
    };
    const uint64_t t0 = uniform64((uint64_t)blockIdx.x * FWAVES + (threadIdx.x >> 6));
    uint64_t k0c, k0n;
    uint32_t npc, npn;
    st1(t0, k0c, npc);
    st1(t0 + nw, k0n, npn);
    Ids idc = ids(t0);
    int64_t keyc;
    uint32_t psc, pcc;
    st2(k0c, npc, keyc);
    probe(t0, npc, keyc, psc, pcc);
    uint4 kqc;
    st3(psc, kqc);
    for (uint64_t ii = t0; ii < n_iter; ii += nw)
    {
        const uint64_t t = tof(ii);
        uint64_t k0nn;
        uint32_t npnn;
        st1(ii + 2 * nw, k0nn, npnn);
        const Ids idn = ids(ii + nw);
        int64_t keyn;
        uint32_t psn = SLOT_NONE, pcn = NO_CELL;
        st2(k0n, npn, keyn);
        uint4 kqn = make_uint4(0, 0, 0, 0);
        bool pf3 = false;
        do {
        if (t == DEFER_HOLE) break;                // unused slot of a lean wave's deferral chunk
        const uint64_t k0 = k0c;
        (void)k0;
        const uint32_t np = npc;
        // more than 8 keys, or a Range-domain request (expanded probes: sliced parts and unsliced ranges, which
        // only the split kernels resolve): the split kernels' list
        if (np > FMAXP || range_split(s, b, k0c, np))
        {
            if (lane == 0) b.deferred[atomicAdd(&b.ctl->n_deferred, 1ull)] = (uint32_t)t;
            break;   // next request (pipeline rotation below)
        }
        // ---- encode the request (PreAccept.java:251-261)
        const uint64_t tm = idc.tm, tl = idc.tl;
        const int32_t tn = idc.tn;
        const uint64_t em = idc.em, el = idc.el;
        const int32_t en = idc.en;
        const uint32_t kinds = kind_witnesses((uint32_t)((tl >> 1) & 7));
        if (kinds == 0)
        {
            if (lane == 0) set_error_f(b.ctl, ERR_INVAL);
            break;   // next request (pipeline rotation below)
        }
        const int cls = kinds_class(kinds);
        const bool same = em == tm && ((el ^ tl) & 0xFFFFFFFFFFFF001EULL) == 0 && en == tn;
        (void)same;
        const uint4 rec = b.q_rec[t];              // ranks of S and self (k_prepare)
        const uint32_t S = rec.y;
        const uint32_t self = rec.w;
        const int64_t epoch = (int64_t)(em >> 15);
        const int64_t mine = b.q_min_epoch ? b.q_min_epoch[t] : 0;

        // ---- per key g (8-lane group g < np): the KeyEntry and KeyRec of the key's CommandsForKey,
        // found by k_prepare (lane j of the group loads quarter j)
        const bool gact = g < np;
        const uint32_t gb = lane & ~7u;
        const int64_t key = keyc;
        const uint32_t pslot = psc;
        const bool in_slice = (pslot & SLOT_IN_SLICE) != 0;
        const uint32_t slot = pslot & ~SLOT_IN_SLICE;
        if (gact && j == 0) L.key[g] = key;
        uint4 kq = kqc;
        const uint32_t ki = slot != SLOT_NONE ? slot : NO_KEY;
        KeyRec kr;     // lanes 4/5: KeyRec; lane 0: newest fields; lane 1 + cls: the class lists
        kr.seg_lo = __shfl(kq.x, gb + 4, 64);
        kr.seg_hi = __shfl(kq.y, gb + 4, 64);
        kr.w_lo = __shfl(kq.z, gb + 4, 64);
        kr.w_hi = __shfl(kq.w, gb + 4, 64);
        kr.last_txn = __shfl(kq.x, gb + 5, 64);
        kr.last_wexec = __shfl(kq.y, gb + 5, 64);
        kr.pruned = __shfl(kq.z, gb + 5, 64);
        kr.maw = (int32_t)__shfl(kq.w, gb + 5, 64);
        const uint32_t last_w_txn = __shfl(kq.z, gb, 64);
        const uint32_t cq = gb + 1 + (uint32_t)cls;
        const uint32_t cand_lo = __shfl(kq.x, cq, 64), cand_hi = __shfl(kq.y, cq, 64);
        const uint32_t cwr_tail = __shfl(kq.z, cq, 64), cwr_hi = __shfl(kq.w, cq, 64);
        const bool has_cfk = gact && ki != NO_KEY;

        // ---- K1: end = insertPos(S), M = maxCommittedWriteBefore (CommandsForKey.java:912-928)
        const uint64_t lo = kr.seg_lo, hi = kr.seg_hi;
        const bool tail = !has_cfk || hi == lo || kr.last_txn < S;
        const uint64_t wlo = kr.w_lo, whi = kr.w_hi;
        const bool wtail = !has_cfk || whi == wlo || kr.last_wexec < S;
        // S above the key's last committed Write (M is the newest one) and above prunedBefore: the emissions are
        // the newest probe's two precomputed lists (KeyEntry) less the entries at or above S -- insertPos(S) is the
        // element filter rank < S, no search and no descent (as the lean passes' newest test; a late PreAccept or an
        // Accept whose S sits below some newer txnIds lands here)
        const bool listp = has_cfk && s.elide && wtail && (tail || kr.pruned == 0 || S > kr.pruned);
        // insertPos(S) in byId and the committed Writes' executeAt search, in lockstep
        uint64_t end, wsearch;
        grp_lower_bound2(has_cfk && !tail && !listp, lo, hi, [&](uint64_t i) { return s.ent[i].y & RANK_MASK; },
                         has_cfk && !wtail, wlo, whi, [&](uint64_t i) { return s.w[i].x; }, S, end, wsearch);
        const uint64_t end_g = tail ? hi : end;
        const uint64_t wpos = !has_cfk ? wlo : (whi == wlo ? wlo : (kr.last_wexec < S ? whi : wsearch));
        uint32_t wprev = 0;
        if (has_cfk && wpos > wlo) wprev = (wpos == whi) ? kr.last_wexec : s.w[wpos - 1].x;
        const uint32_t M = (s.elide && has_cfk && wpos > wlo) ? wprev : 1u;

        // prunedBefore substitute (:952-965)
        uint32_t extra = 0;
        if (has_cfk && kr.pruned != 0 && S <= kr.pruned)
        {
            // no applied Write: binarySearch(committedByExecuteAt, 0, -1, S) = -1, the walk starts
            // at the first committed entry (:955-962); no committed Write at all throws
            if (kr.maw < 0 && whi == wlo) { if (j == 0) set_error_f(b.ctl, ERR_STATE); }
            else
            {
                const uint64_t idx = kr.maw < 0 ? wlo : (wpos <= (uint64_t)kr.maw ? wpos : (uint64_t)kr.maw);
                extra = s.w[idx].y;
                if (extra == self) extra = 0;
            }
        }

        uint32_t c0 = 0, c1 = 0, nlt = 0;
        bool ovf = false, dup = false;
        // emission of 8 consecutive byId entries n0..n0+7 held in q (mapReduceActive loop body,
        // CommandsForKey.java:930-950): group-collective, staged in entry order into LDS
        auto stage8 = [&](uint64_t n0, const uint4 (&q)[4], bool on) {
            uint32_t w0 = 0, w1 = 0, lt = 0, eq = 0;
#pragma unroll
            for (int i = 0; i < 8; ++i)
            {
                const uint32_t tau = (i & 1) ? q[i >> 1].z : q[i >> 1].x;
                const uint32_t txw = (i & 1) ? q[i >> 1].w : q[i >> 1].y;
                const uint64_t e = n0 + i;
                const uint32_t r = txw & RANK_MASK, kd = txw >> RANK_BITS;
                const bool want = on && e >= lo && e < end_g && tau >= M && ((kinds >> kd) & 1) && r != self;
                const bool is1 = ((KINDS_RS_OR_WS >> kd) & 1) == 0;   // !managesExecution -> directKeyDeps
                w0 |= (want && !is1) ? (1u << i) : 0u;
                w1 |= (want && is1) ? (1u << i) : 0u;
                lt += (want && !is1 && r < extra) ? 1u : 0u;
                eq |= (want && r == extra) ? 1u : 0u;
            }
            const uint32_t n0c = __popc(w0), n1c = __popc(w1);
            const uint32_t i0 = grp_incl_scan(n0c), i1 = grp_incl_scan(n1c);
            const uint32_t t0 = __shfl(i0, (lane & ~7u) | 7u, 64), t1 = __shfl(i1, (lane & ~7u) | 7u, 64);
            if (c0 + t0 <= FCAP0 && c1 + t1 <= FCAP1)
            {
                uint32_t p0 = c0 + i0 - n0c, p1 = c1 + i1 - n1c;
#pragma unroll
                for (int i = 0; i < 8; ++i)
                {
                    const uint32_t r = ((i & 1) ? q[i >> 1].w : q[i >> 1].y) & RANK_MASK;
                    if (w0 & (1u << i)) L.st0[g][p0++] = r;
                    if (w1 & (1u << i)) L.st1[g][p1++] = r;
                }
            }
            else ovf = true;
            c0 += t0;
            c1 += t1;
            if (extra)
            {
                nlt += grp_sum(lt);
                dup = dup || grp_sum(eq) != 0;
            }
        };
        auto node_bits = [&](int lv, uint64_t n0, uint64_t nlo, uint64_t nhi) -> uint32_t {
            const uint4* p4 = reinterpret_cast<const uint4*>(s.lvl[cls][lv] + n0);
            const uint4 a = p4[0], c = p4[1];
            const uint32_t v[8] = {a.x, a.y, a.z, a.w, c.x, c.y, c.z, c.w};
            uint32_t bits = 0;
#pragma unroll
            for (int i = 0; i < 8; ++i)
                if (n0 + i >= nlo && n0 + i <= nhi && v[i] >= M) bits |= 1u << i;
            return bits;
        };
        auto leaf = [&](uint64_t n0) {
            const uint4* p4 = reinterpret_cast<const uint4*>(s.ent + n0);
            uint4 q[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) q[i] = p4[i];
            stage8(n0, q, true);
        };

        // Newest probe (S above every committed Write's executeAt of the key and above prunedBefore, elision on):
        // the emissions are the two precomputed contiguous lists (KeyEntry, common.hpp) filtered by rank < S;
        // otherwise the class max tree prunes byId[lo, end) (output-sensitive descent).
        const bool newest = listp;
        if (ballot(newest))
        {
            const uint32_t n1 = newest ? cand_hi - cand_lo : 0u;
            const uint32_t n2 = !newest ? 0u : (cls == 0 ? (last_w_txn != 0 ? 1u : 0u) : cwr_hi - cwr_tail);
            const uint32_t nn = n1 + n2;
            for (uint32_t o = 0; ballot(o < nn); o += 8)
            {
                const uint32_t i = o + j;
                bool want = i < nn;
                uint32_t txw = 0;
                if (want)
                    txw = i < n1 ? s.cand[cand_lo + i]
                                 : (cls == 0 ? (last_w_txn | (1u << RANK_BITS)) : s.cwr[cwr_tail + (i - n1)]);
                const uint32_t r = txw & RANK_MASK, kd = txw >> RANK_BITS;
                want = want && r != self && r < S;
                const bool is1 = ((KINDS_RS_OR_WS >> kd) & 1) == 0;   // !managesExecution -> directKeyDeps
                const uint32_t w0 = (want && !is1) ? 1u : 0u, w1 = (want && is1) ? 1u : 0u;
                const uint32_t i0 = grp_incl_scan(w0), i1 = grp_incl_scan(w1);
                const uint32_t t0 = __shfl(i0, gb | 7u, 64), t1 = __shfl(i1, gb | 7u, 64);
                if (c0 + t0 <= FCAP0 && c1 + t1 <= FCAP1)
                {
                    if (w0) L.st0[g][c0 + i0 - 1] = r;
                    if (w1) L.st1[g][c1 + i1 - 1] = r;
                }
                else ovf = true;
                c0 += t0;
                c1 += t1;
            }
        }
        const bool treep = has_cfk && !newest;
        if (ballot(treep)) grp_descent(treep, lo, end_g, s.n_levels, node_bits, leaf, L.stk[g]);

        // ---- K4: range commands containing the key + the redundant-before entry
        uint32_t rc = 0;
        uint64_t rbv = NO_RB;
        if (s.n_rb)
        {
            const uint64_t c = grp_lower_bound(gact, 0, s.n_rb, [&](uint64_t i) { return s.rb_start[i]; },
                                               [&](int64_t v) { return incl ? v <= key : v < key; });
            if (gact && c > 0)
            {
                const uint64_t e = c - 1;
                if (range_contains(s.start_inclusive, s.rb_start[e], s.rb_end[e], key))
                {
                    const uint32_t wm = s.rb_wm[e];
                    if (!(epoch < s.rb_e0[e] || mine >= s.rb_e1[e]) && wm != 0) rbv = ((uint64_t)s.rb_rid[e] << 32) | wm;
                }
            }
        }
        const uint32_t pcell = gact ? pcc : NO_CELL;
        if (s.n_rent && s.cell_off)
        {
            // stabbing index: the key's cell lists every range entry containing it, in (range,
            // txnId) order; keep those the reference's filter keeps (InMemoryCommandStore.java:906-956)
            const bool ract = gact && in_slice && pcell != NO_CELL;
            const uint32_t clo = ract ? s.cell_off[pcell] : 0u, chi = ract ? s.cell_off[pcell + 1] : 0u;
            const uint32_t nn = chi - clo;
            for (uint32_t o = 0; ballot(o < nn); o += 8)
            {
                const uint32_t i = o + j;
                const uint64_t ce = i < nn ? s.cell_ent[clo + i] : 0ull;
                const uint32_t txw = (uint32_t)ce, r = txw & RANK_MASK, kd = txw >> RANK_BITS;
                const bool want = i < nn && r < S && ((kinds >> kd) & 1) && r != self;
                const uint32_t w1 = want ? 1u : 0u;
                const uint32_t inc = grp_incl_scan(w1);
                const uint32_t tot = __shfl(inc, (lane & ~7u) | 7u, 64);
                if (rc + tot <= FCAPR)
                {
                    if (want) L.rs[g][rc + inc - 1] = (ce & 0xFFFFFFFF00000000ull) | r;
                }
                else ovf = true;
                rc += tot;
            }
        }
        else if (s.n_rent)
        {
            const bool ract = gact && in_slice;
            const uint64_t rhi = grp_lower_bound(ract, 0, s.n_rent, [&](uint64_t i) { return s.r_start[i]; },
                                                 [&](int64_t v) { return incl ? v <= key : v < key; });
            auto end_ok = [&](int64_t e) { return incl ? e > key : e >= key; };
            auto rnode_bits = [&](int lv, uint64_t n0, uint64_t nlo, uint64_t nhi) -> uint32_t {
                const int64_t* pv = s.rlvl[cls][lv] + n0;
                uint32_t bits = 0;
#pragma unroll
                for (int i = 0; i < 8; ++i)
                    if (n0 + i >= nlo && n0 + i <= nhi && end_ok(pv[i])) bits |= 1u << i;
                return bits;
            };
            auto rleaf = [&](uint64_t n0) {
                uint32_t wbits = 0;
#pragma unroll
                for (int i = 0; i < 8; ++i)
                {
                    const uint64_t e = n0 + i;
                    const uint32_t txw = s.r_txw[e];
                    const uint32_t r = txw & RANK_MASK, kd = txw >> RANK_BITS;
                    // STARTED_BEFORE, testKind, contains key, self (InMemoryCommandStore.java:906-956)
                    if (e < rhi && end_ok(s.r_end[e]) && r < S && ((kinds >> kd) & 1) && r != self) wbits |= 1u << i;
                }
                const uint32_t nc = __popc(wbits);
                const uint32_t inc = grp_incl_scan(nc);
                const uint32_t tot = __shfl(inc, (lane & ~7u) | 7u, 64);
                if (rc + tot <= FCAPR)
                {
                    uint32_t pos = rc + inc - nc;
                    for (int i = 0; i < 8; ++i)
                        if (wbits & (1u << i))
                            L.rs[g][pos++] = ((uint64_t)s.r_rid[n0 + i] << 32) | (s.r_txw[n0 + i] & RANK_MASK);
                }
                else ovf = true;
                rc += tot;
            };
            grp_descent(ract, 0, rhi, s.n_rlevels, rnode_bits, rleaf, L.stk[g]);
        }
        if (gact && j == 0) L.rs[g][FCAPR] = rbv;

        // lists staged: the next request's key probe and KeyEntry loads go out now, behind this
        // one's build
        probe(ii + nw, npn, keyn, psn, pcn);
        st3(psn, kqn);
        pf3 = true;

        // any key overflowing its staging -> defer the whole request to the split kernels
        if (ballot(ovf))
        {
            if (lane == 0) b.deferred[atomicAdd(&b.ctl->n_deferred, 1ull)] = (uint32_t)t;
            break;   // next request (pipeline rotation below)
        }
        const bool has_extra = extra != 0 && !dup;
        // insert the prunedBefore substitute at its sorted position (class 0 list)
        if (ballot(has_extra && gact))
        {
            wave_lds_sync();
            uint32_t vals[FCAP0 / 8];
#pragma unroll
            for (int i = 0; i < FCAP0 / 8; ++i)
            {
                const uint32_t idx = j + 8 * i;
                vals[i] = (has_extra && gact && idx >= nlt && idx < c0) ? L.st0[g][idx] : 0u;
            }
            wave_lds_sync();
            if (has_extra && gact)
            {
                if (c0 + 1 > FCAP0) ovf = true;
                else
                {
#pragma unroll
                    for (int i = 0; i < FCAP0 / 8; ++i)
                    {
                        const uint32_t idx = j + 8 * i;
                        if (idx >= nlt && idx < c0) L.st0[g][idx + 1] = vals[i];
                    }
                    if (j == 0) L.st0[g][nlt] = extra;
                }
            }
            if (ballot(ovf))
            {
                if (lane == 0) b.deferred[atomicAdd(&b.ctl->n_deferred, 1ull)] = (uint32_t)t;
                break;   // next request (pipeline rotation below)
            }
        }
        const uint32_t cnt0 = c0 + (has_extra ? 1u : 0u);

        // ---- K2: build the three maps in registers (lane = element, <= 64 per map)
        const uint32_t q0 = __shfl(cnt0, lane * 8, 64), q1 = __shfl(c1, lane * 8, 64), qr = __shfl(rc, lane * 8, 64);
        const uint64_t qrb = __shfl(rbv, lane * 8, 64);
        const uint32_t sh_qr = __shfl(qr, lane >> 1, 64);
        const uint64_t sh_rb = __shfl(qrb, lane >> 1, 64);
        const uint32_t rl = lane < 2 * np ? ((lane & 1) ? (sh_rb != NO_RB ? 1u : 0u) : sh_qr) : 0u;
        const uint32_t tot0 = uniform(wave_sum(lane < np ? q0 : 0u));
        const uint32_t tot1 = uniform(wave_sum(lane < np ? q1 : 0u));
        const uint32_t totR = uniform(wave_sum(rl));
        if (tot0 > 64 || tot1 > 64 || totR > 64)
        {
            if (lane == 0) b.deferred[atomicAdd(&b.ctl->n_deferred, 1ull)] = (uint32_t)t;
            break;   // next request (pipeline rotation below)
        }
        wave_lds_sync();
        // keyDeps (class 0) and directKeyDeps (class 1): lists = keys in request order
        for (int c = 0; c < 2; ++c)
        {
            const int m = c == 0 ? 0 : 2;
            const uint32_t tot = c == 0 ? tot0 : tot1;
            const uint32_t cnt_l = c == 0 ? q0 : q1;               // lane p < np: length of key p's list
            const uint32_t inc = wave_incl_scan(lane < np ? cnt_l : 0u);
            const uint32_t start_l = inc - (lane < np ? cnt_l : 0u);
            if (tot == 0)
            {
                if (lane == 0) { b.sz[(3 * m) * n + t] = 0; b.sz[(3 * m + 1) * n + t] = 0; b.sz[(3 * m + 2) * n + t] = 0; }
                continue;
            }
            // element e = lane: its key a and value
            uint32_t a = 0, a_start = 0;
            for (uint32_t pp = 1; pp < np; ++pp)
            {
                const uint32_t sp = __shfl(start_l, pp, 64);
                if (lane >= sp) { a = pp; a_start = sp; }
            }
            const bool live = lane < tot;
            const uint32_t x = live ? (c == 0 ? L.st0[a][lane - a_start] : L.st1[a][lane - a_start]) : 0u;
            // sort (rank, key) ascending -- rank < 2^29, key < 8: one u32; dedup ranks -> values; a
            // key's body lists the unique-rank index of each of its values in ascending order
            // (staging order is free)
            uint32_t key = live ? ((x << 3) | a) : 0xFFFFFFFFu;
            wave_bitonic32(key, tot);
            const uint32_t xr = key >> 3;
            const uint32_t prevk = __shfl_up(key, 1, 64);
            const bool valid = live;                     // the tot live keys end in lanes [0, tot)
            const bool uniq = valid && (lane == 0 || (prevk >> 3) != xr);
            const uint32_t ka = key & 7u;
            uint64_t same_key = ballot(valid);
#pragma unroll
            for (int bit = 0; bit < 3; ++bit)
            {
                const uint64_t bb = ballot((ka >> bit) & 1u);
                same_key &= ((ka >> bit) & 1u) ? bb : ~bb;
            }
            const uint32_t kstart = __shfl(start_l, ka, 64);
            const uint32_t kpos = kstart + __popcll(same_key & ((1ull << lane) - 1));
            const uint64_t um = ballot(uniq);
            const uint32_t U = __popcll(um);
            const uint32_t ur = __popcll(um & ((2ull << lane) - 1)) - 1;     // rank among distinct values
            const uint64_t nem = ballot(lane < np && cnt_l > 0);
            const uint32_t nk = __popcll(nem);
            const uint64_t bytes = fregion_bytes(nk, U, tot);
            const uint64_t ro = ralloc.take(b.ctl, bytes);
            const bool fits = ro + bytes <= reg_cap;
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
                if (lane < np && cnt_l > 0)
                {
                    const uint32_t kk = mbcnt(nem);
                    okeys[kk] = L.key[lane];
                    ok2t[kk] = (int32_t)(nk + start_l + cnt_l);      // absolute end offset (RelationMultiMap.java:245-257)
                }
                if (uniq) otx[ur] = (xr - 1) >> 1;
                if (valid) ok2t[nk + kpos] = (int32_t)ur;
            }
        }

        if (totR == 0)
        {
            if (lane == 0) { b.sz[3 * n + t] = 0; b.sz[4 * n + t] = 0; b.sz[5 * n + t] = 0; }
            break;   // next request (pipeline rotation below)
        }
        {
            // rangeDeps: element e = lane: per key [command pairs] then [redundant pair]
            const uint32_t inc = wave_incl_scan(rl);
            const uint32_t start_l = inc - rl;
            uint32_t a = 0, a_start = 0;
            for (uint32_t pp = 1; pp < 2 * np; ++pp)
            {
                const uint32_t sp = __shfl(start_l, pp, 64);
                if (lane >= sp) { a = pp; a_start = sp; }
            }
            const bool live = lane < totR;
            const uint64_t pr = live ? ((a & 1) ? L.rs[a >> 1][FCAPR] : L.rs[a >> 1][lane - a_start]) : ~0ull;
            // unique (range, txnId) pairs in (Range.compare, TxnId.compareTo) order
            uint64_t key = pr;
            wave_bitonic64(key, totR);
            const uint64_t prevk = __shfl_up(key, 1, 64);
            const bool valid = key != ~0ull;
            const bool uniq = valid && (lane == 0 || prevk != key);
            const uint64_t um = ballot(uniq);
            const uint32_t UPn = __popcll(um);
            // compact the unique pairs to lanes 0..UPn-1 through LDS (the staging is consumed)
            wave_lds_sync();
            uint64_t* cbuf = &L.rs[0][0];
            if (uniq) cbuf[mbcnt(um)] = key;
            wave_lds_sync();
            const uint64_t upair = lane < UPn ? cbuf[lane] : ~0ull;
            wave_lds_sync();
            const bool uplive = lane < UPn;
            const uint32_t rid = (uint32_t)(upair >> 32), rk = (uint32_t)upair;
            const uint32_t prid = __shfl_up(rid, 1, 64);
            const bool gfirst = uplive && (lane == 0 || prid != rid);
            const uint64_t gm = ballot(gfirst);
            const uint32_t nR = __popcll(gm);
            // group end offsets: the next group's first index (or UPn)
            // distinct txnIds: sort (rank, pair position)
            uint64_t k2 = uplive ? (((uint64_t)rk << 8) | lane) : ~0ull;
            wave_bitonic64(k2, UPn);
            const uint64_t prev2 = __shfl_up(k2, 1, 64);
            const bool v2 = k2 != ~0ull;
            const bool uq2 = v2 && (lane == 0 || (uint32_t)(prev2 >> 8) != (uint32_t)(k2 >> 8));
            const uint64_t um2 = ballot(uq2);
            const uint32_t UR = __popcll(um2);
            const uint32_t ur2 = __popcll(um2 & ((2ull << lane) - 1)) - 1;
            const uint64_t bytes = fregion_bytes(nR, UR, UPn);
            const uint64_t ro = ralloc.take(b.ctl, bytes);
            const bool fits = ro + bytes <= reg_cap;
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
                if (gfirst)
                {
                    const uint32_t gi = mbcnt(gm);
                    // end of this group = start of the next group (or UPn)
                    const uint64_t later = gm & ~((2ull << lane) - 1);
                    const uint32_t gend = later ? (uint32_t)(__ffsll((unsigned long long)later) - 1) : UPn;
                    okeys[gi] = (int64_t)rid;
                    ok2t[gi] = (int32_t)(nR + gend);
                }
                if (uq2) otx[ur2] = ((uint32_t)(k2 >> 8) - 1) >> 1;
                if (v2) ok2t[nR + (uint32_t)(k2 & 0xFF)] = (int32_t)ur2;
            }
        }
        } while (false);
        if (!pf3)
        {
            probe(ii + nw, npn, keyn, psn, pcn);
            st3(psn, kqn);
        }
        k0c = k0n; npc = npn;
        k0n = k0nn; npn = npnn;
        idc = idn;
        keyc = keyn; psc = psn; pcc = pcn;
        kqc = kqn;
    }
}

// Per-request preparation, one thread per request (PreAccept.java:251-261 and the key lookups of
// InMemoryCommandStore.mapReduceForKey, :280): the request record the lean kernel reads instead
// of the raw ids, and the key index (KeyEntry / krec position) of every (request, key) probe (open
// addressing, linear probing in the 16-byte KeySlot table).
// Keeping the dependent key -> slot probing here leaves the per-request kernels one load shorter;
// one thread per probe (the first n_txns threads also write the request records).

// SLOTS: the same launch also gives every probe its KeyLine for the lean passes (one thread per
// probe: the slice test, then the perfect hash; 0xFFFFFFFF outside the slices)
// PREP_PPT probes per thread (block-strided: probe blockIdx.x * 256 * PREP_PPT + j * 256 + tid, each j a
// coalesced pass), their key and displacement loads issued together
#ifndef PREP_PPT
#define PREP_PPT 2
#endif
template <bool SLOTS>
__global__ __launch_bounds__(256) void k_prepare(DevSnapshot s, BatchBufs b)
{
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b.ctl_init && blockIdx.x == 0 && threadIdx.x < sizeof(BatchCtl) / 8)
    {
        const uint32_t i = threadIdx.x;
        reinterpret_cast<uint64_t*>(b.ctl)[i] = (i & 1) && i < 8 ? b.init_cap[i >> 1] : 0ull;
    }
    if (SLOTS)
    {
        const uint64_t p0 = (uint64_t)blockIdx.x * blockDim.x * PREP_PPT + threadIdx.x;
        int64_t key[PREP_PPT];
        bool in[PREP_PPT];
        uint32_t d[PREP_PPT];
#pragma unroll
        for (int j = 0; j < PREP_PPT; ++j)
        {
            const uint64_t p = p0 + (uint64_t)j * blockDim.x;
            key[j] = b.q_keys[p < b.n_probes ? p : 0];
        }
#pragma unroll
        for (int j = 0; j < PREP_PPT; ++j)
        {
            bool x;
            if (b.q_slice_set)
            {
                // per-request slices: the probe's request by a search of the key offsets (batches that name slice
                // sets only; a probe-major thread does not know its request otherwise)
                const uint64_t p = p0 + (uint64_t)j * blockDim.x;
                uint64_t lo = 0, hi = b.n_txns;
                while (lo + 1 < hi)
                {
                    const uint64_t mid = (lo + hi) >> 1;
                    if (b.q_key_off[mid] <= p) lo = mid;
                    else hi = mid;
                }
                x = p < b.n_probes && slice_has(s.start_inclusive, request_slice(s, b.q_slice_set, lo), key[j]);
            }
            else
                x = slice_has(s.start_inclusive, SliceView{s.slice_start, s.slice_end, s.n_slices, s.n_slices == 0}, key[j]);
            in[j] = x;
            d[j] = 0;
            if (x) d[j] = s.kl_disp[kl_bucket(key_hash(key[j]), s.kl_buckets)];
        }
#pragma unroll
        for (int j = 0; j < PREP_PPT; ++j)
        {
            const uint64_t p = p0 + (uint64_t)j * blockDim.x;
            if (p < b.n_probes) b.p_slot[p] = in[j] ? (uint32_t)kl_index(key_hash2(key[j]), d[j], s.kl_lines) : 0xFFFFFFFFu;
        }
    }
    if (t >= b.n_txns) return;
    if (b.q_slice_set && b.q_slice_set[t] != SLICE_STORE && b.q_slice_set[t] >= s.n_ssets) set_error_f(b.ctl, ERR_SLICE);
    // request t's record
    const uint64_t k0 = b.q_key_off[t], k1 = b.q_key_off[t + 1];
    const uint64_t tm = b.q_txn_msb[t], tl = b.q_txn_lsb[t], em = b.q_exec_msb[t], el = b.q_exec_lsb[t];
    const int32_t tn = b.q_txn_node[t], en = b.q_exec_node[t];
    const uint32_t kinds = kind_witnesses((uint32_t)((tl >> 1) & 7));
    const uint32_t cls = kinds ? (uint32_t)kinds_class(kinds) : 0u;
    // S = executeAt, self = txnId unless it equals executeAt (PreAccept.java:251-261), as ranks:
    // no load for ids newer than the store (fresh PreAccepts), else a search of the sampled
    // dictionary (Accepts: S is a proposed executeAt, self a txnId the store holds)
    const bool same = em == tm && ((el ^ tl) & 0xFFFFFFFFFFFF001EULL) == 0 && en == tn;
    // both searches advance in lockstep (one chain of round trips for an Accept's two ids)
    const NormTid ids2[2] = {norm_tid(em, el, en), norm_tid(tm, tl, tn)};
    const bool want2[2] = {true, !same};
    uint32_t rk2[2];
    dict_rank_sampled_n<2>(s, ids2, want2, rk2);
    const uint32_t S = rk2[0], self = rk2[1];
    const uint64_t np = k1 - k0;
    // a Range-domain request (its probes expanded by k_range_fill; the first is not a key's) on a store with range
    // commands or redundant-before entries -- whose sliced parts (PK_RANGE) and unsliced ranges (PK_RANGE_RB) only
    // the split kernels resolve -- leaves the lean and general kernels for the split kernels' list. On a store
    // with neither its probes are the CommandsForKey keys inside its sliced ranges (PK_RANGE_KEY), ascending:
    // mapReduceActive over each as for a key-domain request (InMemoryCommandStore.java:289-304), so it stays.
    const bool rreq = range_split(s, b, k0, np);
    // lean path: at most 8 keys, a valid kind, key offsets within 32 bits, key-domain
    const bool fast = kinds != 0 && np <= 8 && k1 <= 0xFFFFFFFFull && !rreq;
    b.q_rec[t] = make_uint4((uint32_t)k0, S,
                            (uint32_t)(np < 0xFFFFu ? np : 0xFFFFu) | (cls << 16) | (fast ? REC_FAST : 0u) | (rreq ? REC_SPLIT : 0u),
                            self);
}

hipError_t run_prepare(const DevSnapshot& s, const BatchBufs& b, hipStream_t st)
{
    if (b.p_slot)
    {
        const uint64_t m = std::max<uint64_t>(b.n_txns, (b.n_probes + PREP_PPT - 1) / PREP_PPT);
        if (m) k_prepare<true><<<(unsigned)((m + 255) / 256), 256, 0, st>>>(s, b);
    }
    else if (b.n_txns)
        k_prepare<false><<<(unsigned)((b.n_txns + 255) / 256), 256, 0, st>>>(s, b);
    return hipGetLastError();
}

hipError_t run_resolve(const DevSnapshot& s, const BatchBufs& b, hipStream_t st)
{
    if (!b.n_txns) return hipSuccess;
    // one resident generation of waves (grid-stride over requests): blocks per CU from the
    // occupancy query (4 waves/SIMD at <= 128 VGPRs), never more than the requests need
    static int per_cu = 0;
    if (!per_cu)
    {
        int nb = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_resolve, 64 * FWAVES, 0) != hipSuccess || nb <= 0) nb = 2;
        per_cu = std::min(nb, 8);
    }
    const uint64_t need = (b.n_txns + FWAVES - 1) / FWAVES;
    const unsigned grid = (unsigned)std::min<uint64_t>(need, (uint64_t)device_cu_count() * per_cu);
    k_resolve<<<grid, 64 * FWAVES, 0, st>>>(s, b);
    return hipGetLastError();
}

// ---- deferred requests -> sub-batch for the split kernels, and back -------------------------
__global__ void k_defer_counts(BatchBufs b, const uint32_t* deferred, uint64_t nd, uint32_t* cnt)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nd) return;
    const uint32_t t = deferred[i];
    cnt[i] = (uint32_t)(b.q_key_off[t + 1] - b.q_key_off[t]);
}

__global__ void k_defer_gather(BatchBufs b, const uint32_t* deferred, uint64_t nd, const uint64_t* sub_off, BatchBufs sub,
                               uint64_t* o_tm, uint64_t* o_tl, int32_t* o_tn, uint64_t* o_em, uint64_t* o_el, int32_t* o_en,
                               int64_t* o_me, uint64_t* o_ko, int64_t* o_k, int64_t* o_khi, uint8_t* o_kind, uint32_t* o_ss)
{
    const uint64_t i = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (i >= nd) return;
    const uint32_t t = deferred[i];
    const uint32_t lane = lane_id();
    if (lane == 0)
    {
        o_tm[i] = b.q_txn_msb[t]; o_tl[i] = b.q_txn_lsb[t]; o_tn[i] = b.q_txn_node[t];
        o_em[i] = b.q_exec_msb[t]; o_el[i] = b.q_exec_lsb[t]; o_en[i] = b.q_exec_node[t];
        if (b.q_min_epoch) o_me[i] = b.q_min_epoch[t];
        if (b.q_slice_set) o_ss[i] = b.q_slice_set[t];
        if (o_ko != sub_off)
        {
            o_ko[i] = sub_off[i];
            if (i == nd - 1) o_ko[nd] = sub_off[nd];
        }
    }
    const uint64_t s0 = b.q_key_off[t], len = b.q_key_off[t + 1] - s0, d0 = sub_off[i];
    for (uint64_t k = lane; k < len; k += 64) o_k[d0 + k] = b.q_keys[s0 + k];
    // a batch with Range-domain requests: each probe's kind and range end (k_range_fill)
    if (b.p_kind)
        for (uint64_t k = lane; k < len; k += 64)
        {
            o_khi[d0 + k] = b.q_keys_hi[s0 + k];
            o_kind[d0 + k] = b.p_kind[s0 + k];
        }
}

__global__ void k_defer_scatter(BatchBufs b, const uint32_t* deferred, uint64_t nd, const uint32_t* sub_sz,
                                const uint64_t* sub_reg)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nd) return;
    const uint64_t t = deferred[i], n = b.n_txns;
    for (int a = 0; a < 9; ++a) b.sz[(uint64_t)a * n + t] = sub_sz[(uint64_t)a * nd + i];
    for (int m = 0; m < 3; ++m) b.t_reg[(uint64_t)m * n + t] = sub_reg[(uint64_t)m * nd + i];
}

hipError_t run_defer_counts(const BatchBufs& b, const uint32_t* deferred, uint64_t nd, uint32_t* cnt, hipStream_t st)
{
    if (!nd) return hipSuccess;
    k_defer_counts<<<(unsigned)((nd + 255) / 256), 256, 0, st>>>(b, deferred, nd, cnt);
    return hipGetLastError();
}

hipError_t run_defer_gather(const BatchBufs& b, const uint32_t* deferred, uint64_t nd, const uint64_t* sub_off,
                            const BatchBufs& sub, uint64_t* o_tm, uint64_t* o_tl, int32_t* o_tn, uint64_t* o_em,
                            uint64_t* o_el, int32_t* o_en, int64_t* o_me, uint64_t* o_ko, int64_t* o_k, int64_t* o_khi,
                            uint8_t* o_kind, uint32_t* o_ss, hipStream_t st)
{
    if (!nd) return hipSuccess;
    if (b.p_kind && (!o_khi || !o_kind || !b.q_keys_hi)) return hipErrorInvalidValue;
    if (b.q_slice_set && !o_ss) return hipErrorInvalidValue;
    k_defer_gather<<<(unsigned)((nd + 3) / 4), 256, 0, st>>>(b, deferred, nd, sub_off, sub, o_tm, o_tl, o_tn, o_em, o_el,
                                                             o_en, o_me, o_ko, o_k, o_khi, o_kind, o_ss);
    return hipGetLastError();
}

hipError_t run_defer_scatter(const BatchBufs& b, const uint32_t* deferred, uint64_t nd, const uint32_t* sub_sz,
                             const uint64_t* sub_reg, hipStream_t st)
{
    if (!nd) return hipSuccess;
    k_defer_scatter<<<(unsigned)((nd + 255) / 256), 256, 0, st>>>(b, deferred, nd, sub_sz, sub_reg);
    return hipGetLastError();
}

}  // namespace adx
