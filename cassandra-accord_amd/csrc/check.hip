// check.hip — debug invariant checks on the device (SURVEY §5 "debug aids"): the structural
// invariants the reference asserts on the structures this library produces and maintains, checked
// in place in HBM so a caller (or a test) can validate a batch without copying it back.
//
//   * results (ad_check_result_device): for every request and map the RelationMultiMap invariants
//     (RelationMultiMap.checkValid, RelationMultiMap.java:1074-1097, and the builder's layout,
//     :147-260): keys strictly ascending (Deps keys / Range.compare order = range id order), txnIds
//     strictly ascending and inside the dictionary, keysToTxnIds = nKeys strictly increasing absolute
//     end offsets starting above nKeys and ending at its length, each key's values strictly
//     ascending (no duplicate value for a key) and below nTxnIds, every TxnId used by some key,
//     and the CSR offsets monotone;
//   * the snapshot (ad_check_snapshot): keys strictly ascending, every key's byId segment strictly
//     increasing by TxnId (CommandsForKey.java:1438) with member ranks of the dictionary, the key's
//     cached last txnId, its committed Writes by executeAt strictly increasing (no two committed
//     entries share an executeAt, :1439), and the id dictionary strictly ascending
//     (Timestamp.compareTo, Timestamp.java:208-217).
//
// A violation is counted (atomicAdd) and the smallest failing item recorded (atomicMin); nothing is
// corrected. Integer work, one wave per item, no LDS beyond a per-wave bitmap.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/accord_deps.h"
#include "check.hpp"
#include "common.hpp"
#include "wave.hpp"

namespace adx {

constexpr uint32_t CHK_WAVES = 4;
constexpr uint32_t CHK_BITS = 4096;           // txnIds a wave's bitmap covers per pass

struct CheckOut {
    unsigned long long n_bad;
    unsigned long long first;
};

__device__ __forceinline__ void chk_fail(CheckOut* o, uint64_t item)
{
    if (lane_id() == 0)
    {
        atomicAdd(&o->n_bad, 1ull);
        atomicMin(&o->first, (unsigned long long)item);
    }
}

// one wave per (request, map): item = request * 3 + map
__global__ __launch_bounds__(64 * CHK_WAVES) void k_check_result(ad_deps_result r, uint64_t n_dict, CheckOut* o)
{
    __shared__ uint32_t bits_all[CHK_WAVES][CHK_BITS / 32];
    uint32_t* bits = bits_all[threadIdx.x >> 6];
    const uint32_t lane = lane_id();
    const uint64_t n = r.n_txns;
    const uint64_t nw = (uint64_t)gridDim.x * CHK_WAVES;
    for (uint64_t item = (uint64_t)blockIdx.x * CHK_WAVES + (threadIdx.x >> 6); item < 3 * n; item += nw)
    {
        const uint64_t t = item / 3;
        const int m = (int)(item % 3);
        const uint64_t k0 = r.keys_off[m][t], k1 = r.keys_off[m][t + 1];
        const uint64_t x0 = r.txn_off[m][t], x1 = r.txn_off[m][t + 1];
        const uint64_t p0 = r.k2t_off[m][t], p1 = r.k2t_off[m][t + 1];
        if (k1 < k0 || x1 < x0 || p1 < p0)
        {
            chk_fail(o, item);
            continue;
        }
        const uint64_t nk = k1 - k0, nt = x1 - x0, np = p1 - p0;
        // an empty map has no keys, no ids and no keysToTxnIds; otherwise every key has a value
        // and every id a key: nKeys <= pairs, nTxnIds <= pairs
        if ((nk == 0) != (np == 0) || (nk == 0 && nt != 0) || (nk != 0 && (np < 2 * nk || nt == 0 || np - nk < nt)))
        {
            chk_fail(o, item);
            continue;
        }
        if (nk == 0) continue;
        const int64_t* keys = r.keys[m] + k0;
        const uint32_t* txns = r.txns[m] + x0;
        const int32_t* k2t = r.k2t[m] + p0;
        bool bad = false;
        // keys strictly ascending; txnIds strictly ascending and in the dictionary
        for (uint64_t i = lane; i < nk; i += 64)
            if (i + 1 < nk && !(keys[i] < keys[i + 1])) bad = true;
        for (uint64_t i = lane; i < nt; i += 64)
        {
            if (txns[i] >= n_dict) bad = true;
            if (i + 1 < nt && !(txns[i] < txns[i + 1])) bad = true;
        }
        // end offsets: strictly increasing, from above nKeys to the array's length
        for (uint64_t i = lane; i < nk; i += 64)
        {
            const int64_t e = k2t[i];
            const int64_t prev = i == 0 ? (int64_t)nk : (int64_t)k2t[i - 1];
            if (!(e > prev) || e > (int64_t)np) bad = true;
            if (i + 1 == nk && e != (int64_t)np) bad = true;
        }
        if (ballot(bad))
        {
            chk_fail(o, item);
            continue;
        }
        // values: per key strictly ascending, below nTxnIds (RelationMultiMap.checkValid)
        for (uint64_t j = nk + lane; j < np; j += 64)
        {
            const int32_t v = k2t[j];
            if (v < 0 || (uint64_t)v >= nt) bad = true;
            // j is a key's first value iff it is nKeys or some key's end offset: the binary search
            // finds the key of j, then compares with the previous value of the same key
            uint64_t lo = 0, hi = nk;       // first key whose end > j
            while (lo < hi)
            {
                const uint64_t mid = (lo + hi) >> 1;
                if ((uint64_t)k2t[mid] > j) hi = mid;
                else lo = mid + 1;
            }
            const uint64_t start = lo == 0 ? nk : (uint64_t)k2t[lo - 1];
            if (j > start && !(k2t[j - 1] < v)) bad = true;
        }
        // every TxnId is some key's value: one bitmap pass per CHK_BITS ids
        for (uint64_t b0 = 0; b0 < nt && !ballot(bad); b0 += CHK_BITS)
        {
            for (uint32_t i = lane; i < CHK_BITS / 32; i += 64) bits[i] = 0;
            wave_lds_sync();
            for (uint64_t j = nk + lane; j < np; j += 64)
            {
                const uint64_t v = (uint64_t)(uint32_t)k2t[j];
                if (v >= b0 && v < b0 + CHK_BITS) atomicOr(&bits[(v - b0) >> 5], 1u << ((v - b0) & 31));
            }
            wave_lds_sync();
            const uint64_t span = nt - b0 < CHK_BITS ? nt - b0 : CHK_BITS;
            for (uint64_t i = lane; i < span; i += 64)
                if (!((bits[i >> 5] >> (i & 31)) & 1u)) bad = true;
            wave_lds_sync();
        }
        if (ballot(bad)) chk_fail(o, item);
    }
}

// one wave per key: item = key index; the dictionary's order is item n_keys + i (pair i, i + 1)
__global__ __launch_bounds__(64 * CHK_WAVES) void k_check_snapshot(DevSnapshot s, CheckOut* o)
{
    const uint32_t lane = lane_id();
    const uint64_t nw = (uint64_t)gridDim.x * CHK_WAVES;
    const uint64_t w0 = (uint64_t)blockIdx.x * CHK_WAVES + (threadIdx.x >> 6);
    const uint32_t max_rank = (uint32_t)(2 * s.n_dict + 1);
    for (uint64_t k = w0; k < s.n_keys; k += nw)
    {
        const KeyRec kr = s.krec[k];
        bool bad = k + 1 < s.n_keys && !(s.keys[k] < s.keys[k + 1]);
        if (kr.seg_lo > kr.seg_hi || kr.seg_hi > s.n_ent || (k + 1 < s.n_keys && kr.seg_hi > s.krec[k + 1].seg_lo))
            bad = true;
        if (!ballot(bad))
        {
            // byId strictly increasing, odd (member) ranks inside the dictionary
            for (uint64_t e = kr.seg_lo + lane; e < kr.seg_hi; e += 64)
            {
                const uint32_t rk = s.ent[e].y & RANK_MASK;
                if (!(rk & 1u) || rk >= max_rank) bad = true;
                if (e + 1 < kr.seg_hi && !(rk < (s.ent[e + 1].y & RANK_MASK))) bad = true;
            }
            const uint32_t last = kr.seg_hi > kr.seg_lo ? (s.ent[kr.seg_hi - 1].y & RANK_MASK) : 0u;
            if (lane == 0 && kr.last_txn != last) bad = true;
            // committed Writes by executeAt: strictly increasing executeAt (no duplicates)
            for (uint64_t i = kr.w_lo + lane; i + 1 < kr.w_hi; i += 64)
                if (!(s.w[i].x < s.w[i + 1].x)) bad = true;
        }
        if (ballot(bad)) chk_fail(o, k);
    }
    // the dictionary: strictly ascending under Timestamp.compareTo
    const uint64_t t0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, nt = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = t0; i + 1 < s.n_dict; i += nt)
    {
        const NormTid a{s.dict_hi[i], s.dict_lo[i], s.dict_node[i]};
        const NormTid b{s.dict_hi[i + 1], s.dict_lo[i + 1], s.dict_node[i + 1]};
        if (norm_cmp(a, b) >= 0)
        {
            atomicAdd(&o->n_bad, 1ull);
            atomicMin(&o->first, (unsigned long long)(s.n_keys + i));
        }
    }
}

static unsigned check_grid(uint64_t items)
{
    const uint64_t blocks = (items + CHK_WAVES - 1) / CHK_WAVES;
    const uint64_t cap = (uint64_t)device_cu_count() * 8;
    return (unsigned)(blocks < 1 ? 1 : (blocks < cap ? blocks : cap));
}

hipError_t run_check_result(const ad_deps_result& r, uint64_t n_dict, void* out_dev, hipStream_t st)
{
    CheckOut* o = static_cast<CheckOut*>(out_dev);
    if (r.n_txns == 0) return hipSuccess;
    k_check_result<<<check_grid(3 * r.n_txns), 64 * CHK_WAVES, 0, st>>>(r, n_dict, o);
    return hipGetLastError();
}

hipError_t run_check_snapshot(const DevSnapshot& s, void* out_dev, hipStream_t st)
{
    CheckOut* o = static_cast<CheckOut*>(out_dev);
    const uint64_t items = s.n_keys > s.n_dict / 64 ? s.n_keys : s.n_dict / 64;
    k_check_snapshot<<<check_grid(items + 1), 64 * CHK_WAVES, 0, st>>>(s, o);
    return hipGetLastError();
}

}  // namespace adx
