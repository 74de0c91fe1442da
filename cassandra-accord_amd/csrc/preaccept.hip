// preaccept.hip — the timestamp proposal of a PreAccept batch:
// CommandStore.preaccept (CommandStore.java:322-347) without the node clock. Per request:
//   * rejectBefore.foldl(keys, ...) (CommandStore.java:328-329): rejected if an interval holding
//     one of its keys carries an id above txnId;
//   * ExclusiveSyncPoint: witnessedAt = txnId (markExclusiveSyncPoint stays on the host);
//   * minNonConflicting = maxConflicts.get(keys) (MaxConflicts.java:46-50): the Timestamp::max fold
//     of the intervals holding its keys (ReducingRangeMap.foldl, ReducingRangeMap.java:123-157),
//     fold(value, accumulator) keeping the value on ties; fast path iff permitted, txnId >=
//     minNonConflicting and txnId's epoch >= the node's.
// 8 lanes per request; a key's values from a per-key table of the snapshot's keys (one KeySlot probe,
// one 64-byte line), or by binary search over the map's starts.
#include <hip/hip_runtime.h>

#include "../../include/accord_deps.h"
#include "common.hpp"
#include "kernels.hpp"

namespace adx {

namespace {

// interval of key x: #starts <= x (or < x with inclusive ends) minus one; -1 / n = outside
__device__ __forceinline__ int64_t interval_of(const DevRangeMap& m, int64_t x)
{
    uint64_t lo = 0, hi = m.n + 1;
    while (lo < hi)
    {
        const uint64_t mid = (lo + hi) >> 1;
        const int64_t s = m.starts[mid];
        if (m.inclusive_ends ? s < x : s <= x) lo = mid + 1;
        else hi = mid;
    }
    return (int64_t)lo - 1;
}

__device__ __forceinline__ bool value_at(const DevRangeMap& m, int64_t x, uint64_t& i)
{
    if (m.n == 0) return false;
    const int64_t v = interval_of(m, x);
    if (v < 0 || v >= (int64_t)m.n) return false;
    i = (uint64_t)v;
    return !m.present || m.present[i];
}

__device__ __forceinline__ PaValue value_of(const DevRangeMap& m, int64_t x)
{
    uint64_t i;
    PaValue v{0, 0, 0, 0, 0};
    if (value_at(m, x, i))
    {
        v.msb = m.msb[i];
        v.lsb = m.lsb[i];
        v.node = m.node[i];
        v.present = 1;
    }
    return v;
}

// the snapshot key index of x (KeySlot open addressing, as k_prepare), or KEY_EMPTY
__device__ __forceinline__ uint32_t key_index(const PreacceptArgs& a, int64_t x)
{
    if (!a.khash) return KEY_EMPTY;
    uint64_t h = key_hash(x) & a.khash_mask;
    while (true)
    {
        const KeySlot ks = a.khash[h];
        if (ks.idx == KEY_EMPTY || ks.key == x) return ks.idx;
        h = (h + 1) & a.khash_mask;
    }
}

__global__ void k_key_values(DevRangeMap mc, DevRangeMap rb, const int64_t* keys, uint64_t n_keys, PaValue* key_val)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_keys) return;
    const int64_t x = keys[i];
    key_val[2 * i] = value_of(mc, x);
    key_val[2 * i + 1] = value_of(rb, x);
}

// 8 lanes per request: lane j searches keys j, j+8, ...; the group reduces (rejected: any;
// max: the largest value, on ties the one of the later key, as the ascending fold keeps it)
constexpr uint32_t PA_LANES = 8;

__device__ __forceinline__ bool later_max(const NormTid& v, uint32_t kv, const NormTid& w, uint32_t kw)
{
    const int c = norm_cmp(v, w);
    return c > 0 || (c == 0 && kv > kw);
}

__global__ __launch_bounds__(256) void k_preaccept(PreacceptArgs a)
{
    const uint64_t t = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / PA_LANES;
    const uint32_t j = threadIdx.x % PA_LANES;
    const bool on = t < a.n;                              // every lane stays for the shuffles
    const uint64_t tt = on ? t : 0;
    const uint64_t tm = a.txn_msb[tt], tl = a.txn_lsb[tt];
    const int32_t tn = a.txn_node[tt];
    const NormTid txn = norm_tid(tm, tl, tn);
    const uint64_t k0 = on ? a.key_off[tt] : 0, k1 = on ? a.key_off[tt + 1] : 0;
    const bool esp = ((tl >> 1) & 7) == AD_KIND_EXCLUSIVE_SYNC_POINT;
    bool rejected = false;
    NormTid acc{0, 0, 0};                                 // Timestamp.NONE
    uint64_t om = 0, ol = 0;
    int32_t on_ = 0;
    uint32_t kbest = 0;                                   // key position of the held value (+1; 0 = NONE)
    for (uint64_t k = k0 + j; k < k1; k += PA_LANES)
    {
        const int64_t x = a.keys[k];
        // the key's values: precomputed for snapshot keys, else by search
        const uint32_t ki = key_index(a, x);
        PaValue vmc, vrb;
        if (ki != KEY_EMPTY)
        {
            vmc = a.key_val[2 * (uint64_t)ki];
            vrb = a.key_val[2 * (uint64_t)ki + 1];
        }
        else
        {
            vmc = value_of(a.mc, x);
            vrb = value_of(a.rb, x);
        }
        if (vrb.present) rejected = rejected || norm_cmp(norm_tid(vrb.msb, vrb.lsb, vrb.node), txn) > 0;
        if (esp || !vmc.present) continue;
        const uint64_t vm = vmc.msb, vl = vmc.lsb;
        const int32_t vn = vmc.node;
        const NormTid v = norm_tid(vm, vl, vn);
        const uint32_t kp = (uint32_t)(k - k0) + 1;
        if (later_max(v, kp, acc, kbest) || kbest == 0)
        {
            if (kbest == 0 && norm_cmp(v, acc) < 0) continue;   // below NONE: never taken (NONE is the minimum)
            acc = v; om = vm; ol = vl; on_ = vn; kbest = kp;
        }
    }
#pragma unroll
    for (uint32_t d = 1; d < PA_LANES; d <<= 1)
    {
        const uint64_t hm = __shfl_xor(acc.hi, (int)d, PA_LANES), lm = __shfl_xor(acc.lo, (int)d, PA_LANES);
        const int32_t nm = __shfl_xor(acc.node, (int)d, PA_LANES);
        const uint64_t rm = __shfl_xor(om, (int)d, PA_LANES), rl = __shfl_xor(ol, (int)d, PA_LANES);
        const int32_t rn = __shfl_xor(on_, (int)d, PA_LANES);
        const uint32_t kb = __shfl_xor(kbest, (int)d, PA_LANES);
        const int rj = __shfl_xor(rejected ? 1 : 0, (int)d, PA_LANES);
        rejected = rejected || rj;
        const NormTid o{hm, lm, nm};
        if (kb != 0 && (kbest == 0 || later_max(o, kb, acc, kbest)))
        {
            acc = o; om = rm; ol = rl; on_ = rn; kbest = kb;
        }
    }
    if (!on || j != 0) return;
    uint8_t flags = 0;
    if (rejected) { flags = AD_PA_REJECTED; om = ol = 0; on_ = 0; }
    else if (esp) flags = AD_PA_ESP;
    else if (a.permit_fast_path && norm_cmp(txn, acc) >= 0 && (tm >> 15) >= a.node_epoch) flags = AD_PA_FAST;
    a.out_msb[t] = om;
    a.out_lsb[t] = ol;
    a.out_node[t] = on_;
    a.out_flags[t] = flags;
}

}  // namespace

hipError_t run_preaccept_key_values(const DevRangeMap& mc, const DevRangeMap& rb, const int64_t* keys, uint64_t n_keys,
                                    PaValue* key_val, hipStream_t st)
{
    if (n_keys) k_key_values<<<(unsigned)((n_keys + 255) / 256), 256, 0, st>>>(mc, rb, keys, n_keys, key_val);
    return hipGetLastError();
}

hipError_t run_preaccept(const PreacceptArgs& a, hipStream_t st)
{
    if (a.n) k_preaccept<<<(unsigned)((a.n * PA_LANES + 255) / 256), 256, 0, st>>>(a);
    return hipGetLastError();
}

}  // namespace adx
