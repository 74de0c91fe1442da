// lean.hip — the lean fused kernel: the common case of PreAccept.calculatePartialDeps
// (PreAccept.java:245-267) on a CommandStore without range commands or RedundantBefore entries,
// for requests newer than everything the store holds. Two requests per wave (lanes 0-31 and
// 32-63), no LDS, no trees:
//
//   * executeAt (and txnId) newer than every dictionary id: S = 2 * n_dict without a search
//   * every key newest (S above its last txnId and its last committed Write's executeAt): the
//     mapReduceActive emissions (CommandsForKey.java:930-950) are exactly the key's two
//     precomputed lists (KeyEntry, common.hpp), loaded one element per lane
//   * Deps.AbstractBuilder.add routing (Deps.java:80-106) and the RelationMultiMap build
//     (RelationMultiMap.java:147-260): a 32-lane bitonic sort of (rank, key) per map
//
// Anything else (more than 8 keys, more than 32 emissions, a key needing the tree, an older id)
// is appended to the deferred list and resolved by the general fused kernel (resolve.hip).
#include <hip/hip_runtime.h>

#include "common.hpp"
#include "kernels.hpp"
#include "wave.hpp"

namespace adx {

constexpr int LEAN_WAVES = 4;
constexpr uint32_t LEAN_MAXP = 8;      // keys per request
constexpr uint32_t LEAN_MAXE = 32;     // raw emissions per request (one lane each)
constexpr uint32_t LEAN_CHUNK = 1u << 16;

// ascending bitonic sort within each 32-lane half (lane bit 5 never selects a direction)
template <uint32_t KMAX>
__device__ __forceinline__ void half_bitonic(uint32_t& key)
{
    const uint32_t l = lane_id() & 31u;
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

__device__ __forceinline__ uint32_t half_bits(uint64_t m, uint32_t h) { return (uint32_t)(m >> (32 * h)); }

struct LeanChunk {
    uint64_t cur = 0, end = 0;
    // wave-uniform bump allocation from the region arena
    __device__ __forceinline__ uint64_t take(BatchCtl* ctl, uint64_t nbytes, uint64_t cap)
    {
        if (nbytes > end - cur)
        {
            const uint64_t sz = nbytes > LEAN_CHUNK ? nbytes : LEAN_CHUNK;
            unsigned long long base = 0;
            if (lane_id() == 0) base = atomicAdd(&ctl->reg_top, (unsigned long long)sz);
            base = uniform64(base);
            if (base + sz > cap && lane_id() == 0) atomicOr(&ctl->overflow, 8u);
            cur = base;
            end = base + sz;
        }
        const uint64_t r = cur;
        cur += nbytes;
        return r;
    }
};

__global__ __launch_bounds__(64 * LEAN_WAVES) void k_resolve_lean(DevSnapshot s, BatchBufs b)
{
    const uint32_t lane = lane_id(), h = lane >> 5, hl = lane & 31u;
    const uint32_t below = (1u << hl) - 1u;                     // lanes below this one in its half
    const uint64_t n = b.n_txns;
    const uint64_t npairs = (n + 1) / 2;
    const uint64_t nw = (uint64_t)gridDim.x * LEAN_WAVES;
    const uint64_t reg_cap = uniform64(b.ctl->reg_cap);
    const NormTid last{s.dict_last_hi, s.dict_last_lo, s.dict_last_node};
    const uint32_t S_new = (uint32_t)(2 * s.n_dict);            // rank of an id above every member
    LeanChunk ralloc;

    for (uint64_t pr = uniform64((uint64_t)blockIdx.x * LEAN_WAVES + (threadIdx.x >> 6)); pr < npairs; pr += nw)
    {
        const uint64_t t = 2 * pr + h;
        bool act = t < n;
        // ---- request (PreAccept.java:251-261): ids, witness class, S / self by the newest fast path
        uint64_t k0 = 0;
        uint32_t np = 0;
        uint32_t kinds = 0, S = 0, self = 0;
        int cls = 0;
        bool defer = false;
        if (act)
        {
            k0 = b.q_key_off[t];
            np = (uint32_t)(b.q_key_off[t + 1] - k0);
            const uint64_t tm = b.q_txn_msb[t], tl = b.q_txn_lsb[t], em = b.q_exec_msb[t], el = b.q_exec_lsb[t];
            const int32_t tn = b.q_txn_node[t], en = b.q_exec_node[t];
            kinds = kind_witnesses((uint32_t)((tl >> 1) & 7));
            cls = kinds_class(kinds);
            const bool same = em == tm && ((el ^ tl) & 0xFFFFFFFFFFFF001EULL) == 0 && en == tn;
            const bool s_new = s.n_dict == 0 || norm_cmp(last, norm_tid(em, el, en)) < 0;
            const bool t_new = same || s.n_dict == 0 || norm_cmp(last, norm_tid(tm, tl, tn)) < 0;
            S = s.n_dict ? S_new : 0u;
            self = 0;          // same: none; else a non-member rank (even): never equal to an emission
            defer = np > LEAN_MAXP || kinds == 0 || !s_new || !t_new;
        }
        // ---- per key p = hl < np: its KeyEntry (first 64 bytes)
        const bool kact = act && !defer && hl < np;
        int64_t key = 0;
        uint32_t slot = SLOT_NONE;
        if (kact)
        {
            key = b.q_keys[k0 + hl];
            slot = b.p_slot[k0 + hl] & ~SLOT_IN_SLICE;
        }
        uint4 q0 = make_uint4(0, 0, 0, 0), q1 = q0, q2 = q0, q3 = q0;
        if (slot != SLOT_NONE)
        {
            const uint4* e = reinterpret_cast<const uint4*>(s.kent + slot);
            q0 = e[0];
            q1 = e[1];
            q2 = e[2];
            q3 = e[3];
        }
        const bool has_cfk = slot != SLOT_NONE;
        // newest: end = byId.length (last txnId < S) and M = the last committed Write's executeAt
        // (it executes before S), CommandsForKey.java:912-928
        const bool newest = !has_cfk || (q1.x < S && q1.y < S);
        const uint32_t cand_lo = cls == 0 ? q2.x : (cls == 1 ? q2.y : q2.z);
        const uint32_t cand_hi = cls == 0 ? q3.x : (cls == 1 ? q3.y : q3.z);
        const uint32_t n1 = has_cfk ? cand_hi - cand_lo : 0u;
        const uint32_t n2 = !has_cfk ? 0u : (cls == 0 ? (q0.w != 0 ? 1u : 0u) : q1.w - q1.z);
        const uint32_t nn = kact ? n1 + n2 : 0u;
        // exclusive prefix of nn over the 8 key lanes of each half
        uint32_t inc = nn;
#pragma unroll
        for (uint32_t d = 1; d < 8; d <<= 1)
        {
            const uint32_t v = __shfl_up(inc, d, 8);
            if ((hl & 7) >= d) inc += v;
        }
        const uint32_t start = inc - nn;
        const uint32_t T = __shfl(inc, (lane & 32u) | 7u, 64);
        defer = defer || half_bits(ballot(kact && !newest), h) != 0 || T > LEAN_MAXE;
        if (act && defer && hl == 0) b.deferred1[atomicAdd(&b.ctl->n_deferred1, 1ull)] = (uint32_t)t;
        act = act && !defer;

        // ---- one raw emission per lane: element e = hl of key a
        uint32_t a = 0;
#pragma unroll
        for (uint32_t p = 1; p < LEAN_MAXP; ++p)
        {
            const uint32_t sp = __shfl(start, (lane & 32u) | p, 64);
            if (p < np && hl >= sp) a = p;
        }
        const uint32_t src = (lane & 32u) | a;
        const uint32_t a_start = __shfl(start, src, 64), a_n1 = __shfl(n1, src, 64);
        const uint32_t a_clo = __shfl(cand_lo, src, 64), a_ct = __shfl(q1.z, src, 64), a_lw = __shfl(q0.w, src, 64);
        const bool live = act && hl < T;
        uint32_t txw = 0;
        if (live)
        {
            const uint32_t i = hl - a_start;
            txw = i < a_n1 ? s.cand[a_clo + i] : (cls == 0 ? (a_lw | (1u << RANK_BITS)) : s.cwr[a_ct + (i - a_n1)]);
        }
        const uint32_t r = txw & RANK_MASK, kd = txw >> RANK_BITS;
        const bool want = live && r != self;
        const bool is1 = ((KINDS_RS_OR_WS >> kd) & 1) == 0;       // !managesExecution -> directKeyDeps

        // ---- keyDeps (m = 0) and directKeyDeps (m = 2)
        for (int m = 0; m < 3; m += 2)
        {
            const bool mine = want && (m == 0 ? !is1 : is1);
            const uint64_t mb = ballot(mine);
            const uint32_t tot = __popc(half_bits(mb, h));
            if (mb == 0)
            {
                if (act && hl == 0)
                {
                    b.sz[(3 * m) * n + t] = 0;
                    b.sz[(3 * m + 1) * n + t] = 0;
                    b.sz[(3 * m + 2) * n + t] = 0;
                }
                continue;
            }
            // sort (rank, key) per half; dedup -> txnIds; body = unique-rank index per key, ascending
            uint32_t k = mine ? ((r << 3) | a) : 0xFFFFFFFFu;
            const uint32_t kmax = uniform(max(__shfl(tot, 0, 64), __shfl(tot, 32, 64)));
            if (kmax <= 8) half_bitonic<8>(k);
            else if (kmax <= 16) half_bitonic<16>(k);
            else half_bitonic<32>(k);
            const bool valid = hl < tot;
            const uint32_t xr = k >> 3, ka = k & 7u;
            const uint32_t prev = __shfl_up(k, 1, 32);
            const bool uniq = valid && (hl == 0 || (prev >> 3) != xr);
            // index of this lane's value among the distinct values: uniques up to and including this
            // lane, minus one (equal values sit in adjacent lanes)
            const uint64_t um = ballot(uniq);
            const uint32_t U = __popc(half_bits(um, h));
            const uint32_t ur = __popc(half_bits(um, h) & below) + (uniq ? 1u : 0u) - 1u;
            uint64_t same = ballot(valid);
#pragma unroll
            for (int bit = 0; bit < 3; ++bit)
            {
                const uint64_t bb = ballot((ka >> bit) & 1u);
                same &= ((ka >> bit) & 1u) ? bb : ~bb;
            }
            const uint32_t pos_in_key = __popc(half_bits(same, h) & below);
            // per key p (lanes hl < 8): its number of values, then body starts and heads
            uint32_t cnt = 0;
#pragma unroll
            for (uint32_t p = 0; p < LEAN_MAXP; ++p)
            {
                const uint32_t c = __popc(half_bits(ballot(valid && ka == p), h));
                if ((hl & 7) == p) cnt = c;
            }
            if (hl >= 8) cnt = 0;
            uint32_t cinc = cnt;
#pragma unroll
            for (uint32_t d = 1; d < 8; d <<= 1)
            {
                const uint32_t v = __shfl_up(cinc, d, 8);
                if ((hl & 7) >= d) cinc += v;
            }
            const uint32_t kstart_l = cinc - cnt;
            const uint64_t nem = ballot(hl < 8 && cnt > 0);
            const uint32_t nk = __popc(half_bits(nem, h));
            const uint32_t kk = __popc(half_bits(nem, h) & below);
            const uint32_t kstart = __shfl(kstart_l, (lane & 32u) | ka, 64);
            // regions of both halves from one wave-uniform allocation
            const uint64_t bytes = act && tot ? (((uint64_t)nk * 8 + (uint64_t)U * 4 + (uint64_t)(nk + tot) * 4 + 7) & ~7ull) : 0;
            const uint64_t bA = uniform64(__shfl(bytes, 0, 64)), bB = uniform64(__shfl(bytes, 32, 64));
            const uint64_t base = ralloc.take(b.ctl, bA + bB, reg_cap);
            const uint64_t ro = h ? base + bA : base;
            const bool fits = base + bA + bB <= reg_cap;
            if (act && hl == 0)
            {
                b.sz[(3 * m) * n + t] = fits ? nk : 0;
                b.sz[(3 * m + 1) * n + t] = fits ? U : 0;
                b.sz[(3 * m + 2) * n + t] = fits ? nk + tot : 0;
                b.t_reg[(uint64_t)m * n + t] = ro;
            }
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
        if (act && hl == 0)
        {
            b.sz[3 * n + t] = 0;      // rangeDeps: no range commands / redundant entries on this path
            b.sz[4 * n + t] = 0;
            b.sz[5 * n + t] = 0;
        }
    }
}

hipError_t run_resolve_lean(const DevSnapshot& s, const BatchBufs& b, hipStream_t st)
{
    if (!b.n_txns) return hipSuccess;
    static int per_cu = 0;
    if (!per_cu)
    {
        int nb = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_resolve_lean, 64 * LEAN_WAVES, 0) != hipSuccess || nb <= 0)
            nb = 2;
        per_cu = std::min(nb, 8);
    }
    const uint64_t need = ((b.n_txns + 1) / 2 + LEAN_WAVES - 1) / LEAN_WAVES;
    const unsigned grid = (unsigned)std::min<uint64_t>(need, (uint64_t)device_cu_count() * per_cu);
    k_resolve_lean<<<grid, 64 * LEAN_WAVES, 0, st>>>(s, b);
    return hipGetLastError();
}

}  // namespace adx
