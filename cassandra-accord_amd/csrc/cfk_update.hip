// cfk_update.hip — SURVEY §8 f1: CommandsForKey.update (CommandsForKey.java:972-1042) applied to
// the device-resident snapshot, so a store's steady stream of status transitions does not re-run
// the host ingest and re-upload the snapshot.
//
// An update (key, txnId, InternalStatus, executeAt) raises an entry already in the key's byId:
// the Java's update branch (:1009-1036) replaces the entry iff the new status is above the current
// one (equal status with a higher ballot is not carried by the ABI and counts as "not above").
// Within a batch, updates of one entry apply in order, so the entry ends at the first update of the
// highest status (if above its current status). Entries keep their place in byId; what the
// status/executeAt change moves is re-derived on the device from the per-entry state:
//   * ent[e] = {tau, txw}                         (elision key, common.hpp)
//   * committedByExecuteAt per key (:651-672)      -> stable compaction + LSD radix sort by
//                                                    (key index, executeAt rank)
//   * w (committed Writes by executeAt), maxAppliedWriteByExecuteAt (:660-672), krec
//   * the newest-probe emission lists cand / cwr and KeyEntry
//   * the 64-ary max trees over tau (build_cfk_trees).
// Insertion (:1002-1007): an absent txnId is inserted at its byId position (-1 - binarySearch; the
// per-entry arrays are rewritten once per batch with every key's new entries spliced in). Ids the
// dictionary does not hold (txnIds and executeAts) join it first: appended when newer than all of
// it (no rank changes), otherwise merged, which remaps every stored rank in place (monotone, so all
// rank-sorted arrays stay sorted) before the batch is located. A failed batch leaves the store's
// content unchanged (a merged dictionary stays: it adds ids, changes no answer).
// Pruning (run_cfk_prune, end of file): Pruning.maybePrune / pruneBefore for a list of keys, the
// removed entries compacted out of the per-entry arrays and the derived arrays rebuilt.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>

#include "../../include/accord_deps.h"
#include "cfk_update.hpp"
#include "devmem.hpp"
#include "kernels.hpp"
#include "levels.hpp"

namespace adx {

namespace {

enum : uint32_t {
    UE_KEY = 1,          // key not in the snapshot
    UE_STATUS = 2,       // status > 7
    UE_ABSENT = 3,       // txnId not in the key's byId (insert)
    UE_NEW_EXEC = 4,     // executeAt not in the id dictionary
    UE_FLAGS = 5,        // equal ids differing in flag bits
    UE_DOMAIN = 6,       // live range-domain id in a CommandsForKey
    UE_DUP_EXEC = 7,     // two committed entries of a key with one executeAt (:1439)
    UE_UNWITNESSED = 8,  // a dep the txn's kind does not witness, inside byId, absent, not an ExclusiveSyncPoint
};

struct UpdCtl {
    uint32_t err, err_idx;
    unsigned long long applied;
    uint64_t tot[4];          // cand per class, committed entries
    uint64_t tot2[2];         // new dictionary ids (unique), inserted entries (groups)
    uint64_t tot3[2];         // insertion updates, present updates (ballot fold)
    uint32_t n_new, n_ins;    // ids the dictionary does not hold, insertion updates
    unsigned long long diff[3];   // OR of (word ^ reference) over the new ids: node, lo, hi (sort digits)
    uint32_t older, pad;      // a new id is older than the newest dictionary id (dictionary merge)
    uint64_t cm[2];           // incremental committed order: entries kept from the last one, changed committed entries
    uint32_t n_newk, pad2;    // update keys without a CommandsForKey (with repeats)
    unsigned long long kdiff; // OR of (key ^ the batch's first key) over them, sign-flipped (sort digits)
};
constexpr uint32_t LOC_NONE = 0xFFFFFFFFu;

__device__ inline void upd_fail(UpdCtl* c, uint32_t code, uint32_t idx)
{
    if (atomicCAS(&c->err, 0u, code) == 0u) c->err_idx = idx;
}

// Every SAMP-th dictionary id, rebuilt per batch (a few 10^4 ids: cache-resident), so a search
// touches HBM only inside one SAMP-id window.
constexpr uint64_t SAMP = 256;
struct DictSample { const uint64_t* hi; const uint64_t* lo; const int32_t* node; uint64_t n; };

__global__ void k_dict_sample(DevSnapshot s, uint64_t* hi, uint64_t* lo, int32_t* node, uint64_t n)
{
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    hi[j] = s.dict_hi[j * SAMP];
    lo[j] = s.dict_lo[j * SAMP];
    node[j] = s.dict_node[j * SAMP];
}

// lower bound of t in the dictionary: member i -> 2i+1, else 0 (with *pos = i)
__device__ inline uint32_t dict_member_rank(const DevSnapshot& s, const DictSample& ds, const NormTid& t, uint64_t* pos)
{
    // last sample <= t bounds the window [j * SAMP, (j + 1) * SAMP]
    uint64_t a = 0, b = ds.n;
    while (a < b)
    {
        const uint64_t m = (a + b) >> 1;
        const NormTid d{ds.hi[m], ds.lo[m], ds.node[m]};
        if (norm_cmp(d, t) <= 0) a = m + 1;
        else b = m;
    }
    uint64_t lo = a ? (a - 1) * SAMP : 0, hi = a < ds.n ? a * SAMP : s.n_dict;
    while (lo < hi)
    {
        const uint64_t m = (lo + hi) >> 1;
        const NormTid d{s.dict_hi[m], s.dict_lo[m], s.dict_node[m]};
        if (norm_cmp(d, t) < 0) lo = m + 1;
        else hi = m;
    }
    *pos = lo;
    if (lo < s.n_dict)
    {
        const NormTid d{s.dict_hi[lo], s.dict_lo[lo], s.dict_node[lo]};
        if (norm_cmp(d, t) == 0) return (uint32_t)(2 * lo + 1);
    }
    return 0;
}

__device__ inline uint32_t tau_of(uint32_t st, uint32_t kind, uint32_t xr)
{
    if (st == AD_ST_TRANSITIVELY_KNOWN || st == AD_ST_INVALID_OR_TRUNCATED_OR_UNMANAGED_COMMITTED) return 0;
    if (st >= AD_ST_COMMITTED && ((KINDS_RS_OR_WS >> kind) & 1u)) return xr;
    return TAU_NEVER_ELIDED;
}

// InternalStatus flags (CommandsForKey.java:495-538)
__device__ inline bool st_has_exec(uint32_t st) { return st >= AD_ST_ACCEPTED && st <= AD_ST_APPLIED; }
__device__ inline bool st_has_ballot(uint32_t st)
{
    return st >= AD_ST_PREACCEPTED_OR_ACCEPTED_INVALIDATE && st <= AD_ST_COMMITTED;
}
__device__ inline bool st_has_info(uint32_t st)
{
    return st >= AD_ST_PREACCEPTED_OR_ACCEPTED_INVALIDATE && st <= AD_ST_APPLIED;
}
__device__ inline Bal upd_ballot(const CfkUpdIn& u, uint64_t i)
{
    if (!u.bal_msb) return Bal{0, 0, 0, 0};
    return Bal{u.bal_msb[i], u.bal_lsb[i], u.bal_node[i], 0};
}
__device__ inline int bal_cmp(const Bal& a, const Bal& b)
{
    return norm_cmp(norm_tid(a.msb, a.lsb, a.node), norm_tid(b.msb, b.lsb, b.node));
}
// does an update (status st, the command's ballot b) replace an entry (cur, cb)? (:1018-1034)
__device__ inline bool replaces(uint32_t st, uint32_t cur, const Bal& b, const Bal& cb)
{
    if (st > cur) return true;
    if (st < cur)   // an invalidation outbidding an Accept
        return st == AD_ST_PREACCEPTED_OR_ACCEPTED_INVALIDATE && cur == AD_ST_ACCEPTED && bal_cmp(b, cb) > 0;
    return st_has_info(st) && bal_cmp(b, cb) > 0;
}
// the ballot a replacing TxnInfo keeps (TxnInfo.create :254-262)
__device__ inline Bal kept_ballot(uint32_t st, const Bal& b) { return st_has_ballot(st) ? b : Bal{0, 0, 0, 0}; }

// thread per update: key index, entry position, executeAt rank (the txnId's own rank unless the
// status has an executeAt, TxnInfo.create :254-262). Without ballots the entry is claimed for the
// first update of the highest status (packed u64 max: status, then the lowest update index); with
// ballots the updates of an entry are folded in batch order by k_fold_present. Insertions are
// flagged (ordered compaction by a scan).
__device__ inline uint32_t remap_rank(uint32_t r, const uint64_t* pos, uint64_t U);

// the rank k_ins_collect found for an id (0: not in the dictionary then -- search it now), moved by
// a merge since
__device__ inline uint32_t known_rank(const DevSnapshot& s, const DictSample& ds, uint32_t r, const uint64_t* mpos, uint64_t U,
                                      const NormTid& t, uint64_t* p)
{
    if (!r) return dict_member_rank(s, ds, t, p);
    if (U) r = remap_rank(r, mpos, U);
    *p = (r - 1) >> 1;
    return r;
}

__global__ __launch_bounds__(256) void k_upd_locate(DevSnapshot s, DictSample ds, CfkDevState d, CfkUpdIn u, uint32_t* loc,
                                                    uint32_t* xr_out, unsigned long long* word, uint64_t* ins_key,
                                                    uint32_t* flags, const uint32_t* rk, const uint64_t* mpos, uint64_t U,
                                                    UpdCtl* ctl, int fold, uint32_t* trk)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= u.n) return;
    loc[i] = 0xFFFFFFFFu;
    flags[i] = 0;                 // insertion
    flags[u.n + i] = 0;           // present (ballot fold)
    const int64_t key = u.keys[i];
    uint32_t k = KEY_EMPTY;
    if (s.n_keys)
    {
        uint64_t h = key_hash(key) & s.khash_mask;
        for (;;)
        {
            const KeySlot sl = s.khash[h];
            if (sl.idx == KEY_EMPTY) break;
            if (sl.key == key) { k = sl.idx; break; }
            h = (h + 1) & s.khash_mask;
        }
    }
    if (k == KEY_EMPTY) { upd_fail(ctl, UE_KEY, (uint32_t)i); return; }
    const uint32_t st = u.status[i];
    if (st > 7) { upd_fail(ctl, UE_STATUS, (uint32_t)i); return; }
    const uint64_t tl = u.txn_lsb[i];
    uint64_t p;
    const uint32_t r = known_rank(s, ds, rk[2 * i], mpos, U, norm_tid(u.txn_msb[i], tl, u.txn_node[i]), &p);
    if (!r) { upd_fail(ctl, UE_ABSENT, (uint32_t)i); return; }
    if (d.dict_lsb_raw[p] != tl) { upd_fail(ctl, UE_FLAGS, (uint32_t)i); return; }
    const KeyRec kr = s.krec[k];
    uint32_t lo = kr.seg_lo, hi = kr.seg_hi;
    while (lo < hi)
    {
        const uint32_t m = (lo + hi) >> 1;
        if ((s.ent[m].y & RANK_MASK) < r) lo = m + 1;
        else hi = m;
    }
    // absent: inserted at -1 - binarySearch (:1002-1007), placed by insert_entries
    const bool present = lo < kr.seg_hi && (s.ent[lo].y & RANK_MASK) == r;
    uint32_t xr = r;
    if (st_has_exec(st))
    {
        const uint64_t el = u.exec_lsb[i];
        xr = known_rank(s, ds, rk[2 * i + 1], mpos, U, norm_tid(u.exec_msb[i], el, u.exec_node[i]), &p);
        if (!xr) { upd_fail(ctl, UE_NEW_EXEC, (uint32_t)i); return; }
        if (d.dict_lsb_raw[p] != el) { upd_fail(ctl, UE_FLAGS, (uint32_t)i); return; }
    }
    if ((tl & 1) && tau_of(st, (uint32_t)((tl >> 1) & 7), xr) != 0) { upd_fail(ctl, UE_DOMAIN, (uint32_t)i); return; }
    xr_out[i] = xr;
    if (trk)
    {
        // for the additions past byId's end (k_past_*): key index, the key's last txnId before the
        // batch, this update's txnId
        trk[3 * i + 0] = k;
        trk[3 * i + 1] = kr.last_txn;
        trk[3 * i + 2] = r;
    }
    if (!present)
    {
        ins_key[i] = ((uint64_t)k << 32) | r;
        flags[i] = 1;
        return;
    }
    loc[i] = lo;
    if (fold) flags[u.n + i] = 1;
    else atomicMax(word + lo, ((unsigned long long)st << 32) | (0xFFFFFFFFull - i));
}

// ---- TxnInfo.missing() and deps-derived additions (Updating.java:99-470, Utils.java:68-352) ----
__device__ inline bool newer_than_dict(const DevSnapshot& s, const NormTid& t);

// the update of dep j (dep_off ascending)
__device__ inline uint64_t dep_owner(const CfkUpdIn& u, uint64_t j)
{
    uint64_t lo = 0, hi = u.n;            // last i with dep_off[i] <= j
    while (hi - lo > 1)
    {
        const uint64_t m = (lo + hi) >> 1;
        if (u.dep_off[m] <= j) lo = m;
        else hi = m;
    }
    return lo;
}

// deps of updates with a deps status join the dictionary with the batch's ids (a superset of the
// additions: an id nothing refers to changes no answer), so the additions batch never grows it
__global__ __launch_bounds__(256) void k_dep_collect(DevSnapshot s, DictSample ds, CfkUpdIn u, uint64_t ndep, uint64_t* nw,
                                                     uint64_t cap, UpdCtl* ctl)
{
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= ndep) return;
    if (!st_has_exec(u.status[dep_owner(u, j)])) return;
    const NormTid ref = norm_tid(u.txn_msb[0], u.txn_lsb[0], u.txn_node[0]);
    const uint64_t l = u.dep_lsb[j];
    const NormTid t = norm_tid(u.dep_msb[j], l, u.dep_node[j]);
    if (!newer_than_dict(s, t))
    {
        uint64_t p;
        if (dict_member_rank(s, ds, t, &p)) return;
        ctl->older = 1u;
    }
    const uint32_t k = atomicAdd(&ctl->n_new, 1u);
    nw[k] = (uint64_t)((uint32_t)t.node ^ 0x80000000u);
    nw[cap + k] = t.lo;
    nw[2 * cap + k] = t.hi;
    nw[3 * cap + k] = l;
    atomicOr(&ctl->diff[0], (unsigned long long)((uint32_t)t.node ^ (uint32_t)ref.node));
    atomicOr(&ctl->diff[1], (unsigned long long)(t.lo ^ ref.lo));
    atomicOr(&ctl->diff[2], (unsigned long long)(t.hi ^ ref.hi));
}

__device__ inline uint32_t key_index_of(const DevSnapshot& s, int64_t key)
{
    if (!s.n_keys) return KEY_EMPTY;
    uint64_t h = key_hash(key) & s.khash_mask;
    for (;;)
    {
        const KeySlot sl = s.khash[h];
        if (sl.idx == KEY_EMPTY) return KEY_EMPTY;
        if (sl.key == key) return sl.idx;
        h = (h + 1) & s.khash_mask;
    }
}

// entry of rank r in key k's byId, or LOC_NONE
__device__ inline uint32_t seg_find(const DevSnapshot& s, const KeyRec& kr, uint32_t r)
{
    uint32_t lo = kr.seg_lo, hi = kr.seg_hi;
    while (lo < hi)
    {
        const uint32_t m = (lo + hi) >> 1;
        if ((s.ent[m].y & RANK_MASK) < r) lo = m + 1;
        else hi = m;
    }
    return (lo < kr.seg_hi && (s.ent[lo].y & RANK_MASK) == r) ? lo : LOC_NONE;
}

// rank of every dep: a member's odd rank, else the even rank of its gap
__global__ void k_dep_rank(DevSnapshot s, DictSample ds, CfkUpdIn u, uint64_t ndep, uint32_t* drank)
{
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= ndep) return;
    uint64_t p;
    const uint32_t r = dict_member_rank(s, ds, norm_tid(u.dep_msb[j], u.dep_lsb[j], u.dep_node[j]), &p);
    drank[j] = r ? r : (uint32_t)(2 * p);
}

// Does update i derive its entry's missing() from its deps (computeInfoAndAdditions, :174-188)? It
// was applied, its status has deps, and its txnId is a key-domain one (a live range-domain id is
// refused by the locate).
__device__ inline bool upd_with_deps(const CfkUpdIn& u, const uint8_t* uapp, uint64_t i)
{
    return (uapp[i] & 1) && st_has_exec(u.status[i]) && !(u.txn_lsb[i] & 1);
}

// The key's last txnId in byId as update i sees it in the sequential Java (Updating.java:210-263 walks
// byId as it stands when update i runs): the last before the batch, raised by every earlier update of
// the batch on the key -- its txnId (now in byId) and, for an applied update with deps, its largest dep
// (a dep above the last id is added, :253-262). Per update: sort key (key index << 32 | batch index),
// value v_i; an exclusive max-scan of (key index << 32 | v) over that order is a segmented max-scan
// (segments ascend), so its low word is the max of v over the earlier updates of the same key.
__global__ void k_past_keys(CfkUpdIn u, const uint8_t* uapp, const uint32_t* trk, const uint32_t* drank, uint64_t* sk,
                            uint32_t* sv, uint32_t* vv)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= u.n) return;
    uint32_t v = trk[3 * i + 2];
    if (upd_with_deps(u, uapp, i))
        for (uint64_t j = u.dep_off[i]; j < u.dep_off[i + 1]; ++j) v = max(v, drank[j]);
    sk[i] = ((uint64_t)trk[3 * i] << 32) | i;
    sv[i] = (uint32_t)i;
    vv[i] = v;
}

__global__ void k_past_words(uint64_t n, const uint64_t* sk, const uint32_t* sv, const uint32_t* vv, uint64_t* wd)
{
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p < n) wd[p] = (sk[p] & 0xFFFFFFFF00000000ull) | vv[sv[p]];
}

__global__ void k_past_last(uint64_t n, const uint64_t* sk, const uint32_t* sv, const uint64_t* ex, const uint32_t* trk,
                            uint32_t* last, uint32_t* pos)
{
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const uint32_t i = sv[p];
    const uint32_t earlier = (ex[p] >> 32) == (sk[p] >> 32) ? (uint32_t)ex[p] : 0u;
    last[i] = max(trk[3 * (uint64_t)i + 1], earlier);
    pos[i] = (uint32_t)p;          // the update's place in (key, batch index) order
}

// Updating.computeInfoAndAdditions (:239-249): a dep that falls between byId entries (not past the
// key's last id as the update sees it), is absent from byId and is not witnessed by the txn's kind must
// be an ExclusiveSyncPoint -- the Java's Invariants.checkState, here AD_E_INVAL. A dep an earlier update
// of the batch on the same key added (witnessed by it, or past its last id) is in the Java's byId when
// this update runs, so it passes. (Not distinguished: a dep only a later update of the batch inserts.)
__global__ void k_dep_check(DevSnapshot s, CfkUpdIn u, const uint8_t* uapp, const uint32_t* drank, const uint32_t* last,
                            const uint64_t* sk, const uint32_t* sv, const uint32_t* pos, UpdCtl* ctl)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= u.n || !upd_with_deps(u, uapp, i)) return;
    const uint32_t k = key_index_of(s, u.keys[i]);
    if (k == KEY_EMPTY) return;
    const KeyRec kr = s.krec[k];
    const uint32_t wk = kind_witnesses((uint32_t)((u.txn_lsb[i] >> 1) & 7));
    const uint32_t lst = last[i];
    for (uint64_t j = u.dep_off[i]; j < u.dep_off[i + 1]; ++j)
    {
        const uint32_t r = drank[j], kd = (uint32_t)((u.dep_lsb[j] >> 1) & 7);
        if (((wk >> kd) & 1u) || r > lst || kd == 4u /* ExclusiveSyncPoint */) continue;
        if (seg_find(s, kr, r) != LOC_NONE) continue;
        bool added = false;
        const uint64_t p = pos[i];
        for (uint64_t q = p; q-- > 0 && !added && (sk[q] >> 32) == (sk[p] >> 32);)
        {
            const uint32_t jj = sv[q];
            if (!upd_with_deps(u, uapp, jj)) continue;
            const uint32_t wj = kind_witnesses((uint32_t)((u.txn_lsb[jj] >> 1) & 7));
            for (uint64_t d = u.dep_off[jj]; d < u.dep_off[jj + 1] && !added; ++d)
                added = drank[d] == r && (((wj >> kd) & 1u) || r > last[jj]);
        }
        if (!added)
        {
            upd_fail(ctl, UE_UNWITNESSED, (uint32_t)i);
            return;
        }
    }
}

// exclusive prefix max of u64 words (identity 0): per-1024 maxima, their scan (one block), the apply
__global__ __launch_bounds__(256) void k_maxscan_blocks(const uint64_t* in, uint64_t n, uint64_t* bmax)
{
    __shared__ uint64_t red[256];
    const uint64_t b0 = (uint64_t)blockIdx.x * 1024;
    uint64_t m = 0;
    for (uint32_t k = threadIdx.x; k < 1024; k += 256)
        if (b0 + k < n) m = max(m, in[b0 + k]);
    red[threadIdx.x] = m;
    __syncthreads();
    for (uint32_t w = 128; w; w >>= 1)
    {
        if (threadIdx.x < w) red[threadIdx.x] = max(red[threadIdx.x], red[threadIdx.x + w]);
        __syncthreads();
    }
    if (!threadIdx.x) bmax[blockIdx.x] = red[0];
}

__device__ inline uint64_t block_excl_max256(uint64_t v, uint64_t* sh)
{
    sh[threadIdx.x] = v;
    __syncthreads();
    for (uint32_t d = 1; d < 256; d <<= 1)
    {
        const uint64_t o = threadIdx.x >= d ? sh[threadIdx.x - d] : 0;
        __syncthreads();
        sh[threadIdx.x] = max(sh[threadIdx.x], o);
        __syncthreads();
    }
    const uint64_t ex = threadIdx.x ? sh[threadIdx.x - 1] : 0;
    __syncthreads();
    return ex;
}

__global__ __launch_bounds__(256) void k_maxscan_top(uint64_t* bmax, uint64_t nb)
{
    __shared__ uint64_t sh[256];
    uint64_t carry = 0;
    for (uint64_t c = 0; c < nb; c += 256)
    {
        const uint64_t i = c + threadIdx.x;
        const uint64_t v = i < nb ? bmax[i] : 0;
        const uint64_t ex = max(carry, block_excl_max256(v, sh));
        if (i < nb) bmax[i] = ex;
        sh[threadIdx.x] = max(ex, v);
        __syncthreads();
        carry = sh[255];
        __syncthreads();
    }
}

__global__ __launch_bounds__(256) void k_maxscan_apply(const uint64_t* in, uint64_t n, const uint64_t* bex, uint64_t* out)
{
    __shared__ uint64_t sh[256];
    const uint64_t b0 = (uint64_t)blockIdx.x * 1024 + 4ull * threadIdx.x;
    uint64_t v[4], run = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k)
    {
        v[k] = b0 + k < n ? in[b0 + k] : 0;
        run = max(run, v[k]);
    }
    uint64_t ex = max(bex[blockIdx.x], block_excl_max256(run, sh));
#pragma unroll
    for (int k = 0; k < 4; ++k)
    {
        if (b0 + k < n) out[b0 + k] = ex;
        ex = max(ex, v[k]);
    }
}

// additions (:210-263): the deps of applied updates with deps statuses -- those their kind witnesses,
// and every dep above the key's last txnId as the update sees it (`last`, :253-262: past byId's end the
// Java adds without the witness test) -- that are not in byId after the batch -> TRANSITIVELY_KNOWN
// insertions. Additions below the key's prunedBefore are dropped (removePrunedAdditions,
// Utils.java:229-246) and handed back as LoadPruned (Updating.java:111-117,171: Pruning.loadPruned).
// Pass 0 counts both per update, pass 1 writes.
struct AddOut {
    uint32_t* cnt; const uint64_t* off; int64_t* k; uint64_t* tm; uint64_t* tl; int32_t* tn;
    uint32_t* pcnt; const uint64_t* poff; int64_t* pk; uint64_t* ptm; uint64_t* ptl; int32_t* ptn; uint64_t* pidx;
};

template <int WRITE>
__global__ __launch_bounds__(256) void k_add_deps(DevSnapshot s, CfkUpdIn u, const uint8_t* uapp, const uint32_t* drank,
                                                  const uint32_t* last, AddOut o)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= u.n) return;
    uint32_t c = 0, pc = 0;
    if (upd_with_deps(u, uapp, i))
    {
        const uint32_t k = key_index_of(s, u.keys[i]);
        if (k != KEY_EMPTY)
        {
            const KeyRec kr = s.krec[k];
            const uint32_t wk = kind_witnesses((uint32_t)((u.txn_lsb[i] >> 1) & 7));
            const uint32_t lst = last[i];
            uint64_t a = WRITE ? o.off[i] : 0, b = WRITE ? o.poff[i] : 0;
            for (uint64_t j = u.dep_off[i]; j < u.dep_off[i + 1]; ++j)
            {
                const uint32_t r = drank[j];
                if (!((wk >> (uint32_t)((u.dep_lsb[j] >> 1) & 7)) & 1u) && r <= lst) continue;
                if (seg_find(s, kr, r) != LOC_NONE) continue;
                if (kr.pruned && r < kr.pruned)
                {
                    if (WRITE)
                    {
                        o.pk[b] = u.keys[i];
                        o.ptm[b] = u.dep_msb[j];
                        o.ptl[b] = u.dep_lsb[j];
                        o.ptn[b] = u.dep_node[j];
                        o.pidx[b] = i;
                        ++b;
                    }
                    ++pc;
                    continue;
                }
                if (WRITE)
                {
                    o.k[a] = u.keys[i];
                    o.tm[a] = u.dep_msb[j];
                    o.tl[a] = u.dep_lsb[j];
                    o.tn[a] = u.dep_node[j];
                    ++a;
                }
                ++c;
            }
        }
    }
    if (!WRITE)
    {
        o.cnt[i] = c;
        o.pcnt[i] = pc;
    }
}

// the entry whose TxnInfo an applied update with deps made (its last applied update): dsrc[e] = i
__global__ void k_miss_src(DevSnapshot s, DictSample ds, CfkUpdIn u, const uint8_t* uapp, uint32_t* dsrc)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= u.n || uapp[i] != 3 || !upd_with_deps(u, uapp, i)) return;
    const uint32_t k = key_index_of(s, u.keys[i]);
    if (k == KEY_EMPTY) return;
    uint64_t p;
    const uint32_t r = dict_member_rank(s, ds, norm_tid(u.txn_msb[i], u.txn_lsb[i], u.txn_node[i]), &p);
    const uint32_t e = r ? seg_find(s, s.krec[k], r) : LOC_NONE;
    if (e != LOC_NONE) dsrc[e] = (uint32_t)i;
}

// per entry: below COMMITTED (a candidate for others' missing()), and that and inserted by this batch
__global__ void k_miss_flags(uint64_t ne, CfkDevState d, uint32_t* f)
{
    const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= ne) return;
    const bool pend = d.status[e] < AD_ST_COMMITTED;
    f[e] = pend ? 1u : 0u;
    f[ne + e] = (pend && d.mref[e] == MREF_BORN) ? 1u : 0u;
}

__global__ void k_miss_scatter(uint64_t ne, const uint32_t* f, const uint64_t* pp, uint32_t* pend)
{
    const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= ne) return;
    if (f[e]) pend[pp[e]] = (uint32_t)e;
    if (f[ne + e]) pend[pp[ne] + pp[ne + 1 + e]] = (uint32_t)e;     // the born list after the pending one
}

// Every entry's missing() after the batch (thread per entry; pass 0 counts, pass 1 writes ranks
// ascending):
//   * statuses without deps: NO_TXNIDS (TxnInfo.create :254-262);
//   * an entry its batch update derived (dsrc): computeInfoAndAdditions' list (:194-287) -- the
//     key's entries below COMMITTED, below its depsKnownBefore (:561-580), its kind witnesses, other
//     than itself, not in its deps;
//   * any other entry with deps: its list less the ids now COMMITTED or later / INVALID
//     (removeFromMissingArrays / removeSelfMissing) merged with this batch's insertions below
//     COMMITTED under its depsKnownBefore that its kind witnesses (addToMissingArrays /
//     insertOrUpdateWithAdditions' missingSource).
template <int WRITE>
__global__ __launch_bounds__(256) void k_miss_build(DevSnapshot s, CfkDevState d, CfkUpdIn u, const uint32_t* dsrc,
                                                    const uint32_t* drank, const uint64_t* pp, const uint32_t* pend,
                                                    const uint64_t* ooff, const uint32_t* oids, uint32_t* cnt,
                                                    const uint64_t* noff, uint32_t* nids)
{
    const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t ne = s.n_ent;
    if (e >= ne) return;
    const uint32_t st = d.status[e];
    uint64_t c = 0, o = WRITE ? noff[e] : 0;
    auto emit = [&](uint32_t r) {
        if (WRITE) nids[o++] = r;
        ++c;
    };
    if (st_has_exec(st))
    {
        const uint32_t k = d.ekey[e];
        const KeyRec kr = s.krec[k];
        const uint32_t y = s.ent[e].y, self = y & RANK_MASK;
        const uint32_t wk = kind_witnesses(y >> RANK_BITS);
        const uint32_t dkb = st == AD_ST_ACCEPTED ? self : d.xrank[e];
        const uint64_t n_pend = pp[ne];
        const uint32_t i = dsrc[e];
        if (i != LOC_NONE)
        {
            // depsKnownBeforePos is searched from the txn's own byId position (:202-208): the entries
            // below its txnId count even when executeAt is below it
            const uint32_t bound = max(dkb, self);
            uint64_t jd = u.dep_off[i];
            const uint64_t jd1 = u.dep_off[i + 1];
            for (uint64_t q = pp[kr.seg_lo]; q < pp[kr.seg_hi]; ++q)
            {
                const uint32_t p = pend[q];
                const uint32_t yp = s.ent[p].y, rp = yp & RANK_MASK;
                if (rp >= bound) break;
                if (p == e || !((wk >> (yp >> RANK_BITS)) & 1u)) continue;
                while (jd < jd1 && drank[jd] < rp) ++jd;
                if (jd < jd1 && drank[jd] == rp) continue;
                emit(rp);
            }
        }
        else
        {
            const uint32_t L = d.mref[e];
            uint64_t a = 0, a1 = 0;
            if (L != MREF_NONE && L != MREF_BORN)
            {
                a = ooff[L];
                a1 = ooff[L + 1];
            }
            const uint64_t* bp = pp + (ne + 1);
            uint64_t b = bp[kr.seg_lo], b1 = bp[kr.seg_hi];
            const uint32_t* born = pend + n_pend;
            // the old ids still below COMMITTED, merged with the born candidates (both ascending)
            uint32_t ra = 0;
            bool ha = false;
            auto next_a = [&]() {
                ha = false;
                while (a < a1)
                {
                    const uint32_t r = oids[a++];
                    const uint32_t pe = seg_find(s, kr, r);
                    if (pe != LOC_NONE && d.status[pe] < AD_ST_COMMITTED) { ra = r; ha = true; return; }
                }
            };
            uint32_t rb = 0;
            bool hb = false;
            auto next_b = [&]() {
                hb = false;
                while (b < b1)
                {
                    const uint32_t p = born[b++];
                    const uint32_t yp = s.ent[p].y, rp = yp & RANK_MASK;
                    if (rp >= dkb) { b = b1; return; }
                    if (p == e || !((wk >> (yp >> RANK_BITS)) & 1u)) continue;
                    rb = rp;
                    hb = true;
                    return;
                }
            };
            next_a();
            next_b();
            while (ha || hb)
            {
                if (ha && (!hb || ra < rb)) { emit(ra); next_a(); }
                else if (hb && (!ha || rb < ra)) { emit(rb); next_b(); }
                else { emit(ra); next_a(); next_b(); }
            }
        }
    }
    if (!WRITE) cnt[e] = (uint32_t)c;
}

__global__ void k_mref_identity(uint64_t ne, uint32_t* mref)
{
    const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e < ne) mref[e] = (uint32_t)e;
}

// ---- insertion ------------------------------------------------------------------------------
__device__ inline bool newer_than_dict(const DevSnapshot& s, const NormTid& t)
{
    if (s.n_dict == 0) return true;
    const NormTid l{s.dict_last_hi, s.dict_last_lo, s.dict_last_node};
    return norm_cmp(t, l) > 0;
}

// ids the dictionary does not hold (txnIds and executeAts): words for the LSD sort + raw lsb;
// ctl->older is set when one of them is older than the newest dictionary id (a merge, not an append)
__global__ __launch_bounds__(256) void k_ins_collect(DevSnapshot s, DictSample ds, CfkUpdIn u, uint64_t* nw, uint64_t cap,
                                                     uint32_t* rk, UpdCtl* ctl)
{
    __shared__ unsigned long long red[3];
    if (threadIdx.x < 3) red[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    // digits that vary among the new ids: relative to the batch's first txnId (any fixed id works)
    const NormTid ref = norm_tid(u.txn_msb[0], u.txn_lsb[0], u.txn_node[0]);
    unsigned long long d0 = 0, d1 = 0, d2 = 0;
    for (int side = 0; side < 2 && i < u.n; ++side)
    {
        rk[2 * i + side] = 0;
        if (side && !st_has_exec(u.status[i])) break;      // executeAt = txnId (TxnInfo.create)
        const uint64_t m = side ? u.exec_msb[i] : u.txn_msb[i], l = side ? u.exec_lsb[i] : u.txn_lsb[i];
        const int32_t nd = side ? u.exec_node[i] : u.txn_node[i];
        const NormTid t = norm_tid(m, l, nd);
        if (!newer_than_dict(s, t))
        {
            uint64_t p;
            const uint32_t r = dict_member_rank(s, ds, t, &p);
            rk[2 * i + side] = r;              // locate takes it from here
            if (r) continue;
            ctl->older = 1u;
        }
        const uint32_t j = atomicAdd(&ctl->n_new, 1u);
        nw[j] = (uint64_t)((uint32_t)t.node ^ 0x80000000u);
        nw[cap + j] = t.lo;
        nw[2 * cap + j] = t.hi;
        nw[3 * cap + j] = l;
        d0 |= (uint64_t)((uint32_t)t.node ^ (uint32_t)ref.node);
        d1 |= t.lo ^ ref.lo;
        d2 |= t.hi ^ ref.hi;
    }
    if (d0) atomicOr(&red[0], d0);
    if (d1) atomicOr(&red[1], d1);
    if (d2) atomicOr(&red[2], d2);
    __syncthreads();
    if (threadIdx.x < 3 && red[threadIdx.x]) atomicOr(&ctl->diff[threadIdx.x], red[threadIdx.x]);
}

static uint32_t digits_that_vary(uint64_t diff)
{
    uint32_t m = 0;
    for (int d = 0; d < 8; ++d)
        if ((diff >> (8 * d)) & 0xFF) m |= 1u << d;
    return m;
}

__global__ void k_iota(uint32_t* v, uint64_t n)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) v[i] = (uint32_t)i;
}

__global__ void k_gather64(const uint64_t* src, const uint32_t* idx, uint64_t n, uint64_t* out)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = src[idx[i]];
}

// sorted new ids: first of each equal run; equal ids must carry equal flag bits
__global__ void k_ins_unique(const uint32_t* order, uint64_t m, const uint64_t* nw, uint64_t cap, uint32_t* flag, UpdCtl* ctl)
{
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= m) return;
    const uint32_t a = order[r];
    bool first = r == 0;
    if (!first)
    {
        const uint32_t b = order[r - 1];
        first = nw[a] != nw[b] || nw[cap + a] != nw[cap + b] || nw[2 * cap + a] != nw[2 * cap + b];
        if (!first && nw[3 * cap + a] != nw[3 * cap + b]) upd_fail(ctl, UE_FLAGS, 0);
    }
    flag[r] = first ? 1u : 0u;
}

__global__ void k_ins_append(const uint32_t* order, uint64_t m, const uint64_t* nw, uint64_t cap, const uint32_t* flag,
                             const uint64_t* pos, uint64_t n_dict, uint64_t* dh, uint64_t* dl, int32_t* dn, uint64_t* draw)
{
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= m || !flag[r]) return;
    const uint32_t a = order[r];
    const uint64_t p = n_dict + pos[r];
    dn[p] = (int32_t)((uint32_t)nw[a] ^ 0x80000000u);
    dl[p] = nw[cap + a];
    dh[p] = nw[2 * cap + a];
    draw[p] = nw[3 * cap + a];
}

// ---- dictionary merge: new ids older than the newest dictionary id ---------------------------
// Every rank moves: old id i -> i + #{new ids below it}, new id j (sorted) -> pos[j] + j where pos[j]
// = its lower bound among the old ids. The rank order is kept, so every rank-keyed array stays
// sorted; the ranks stored in the per-entry state, krec and the range arrays are rewritten in
// place and the derived arrays rebuilt from them.
__global__ void k_merge_pos(DevSnapshot s, DictSample ds, uint64_t U, const uint64_t* uh, const uint64_t* ul,
                            const int32_t* un, uint64_t* pos)
{
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= U) return;
    const NormTid t{uh[j], ul[j], un[j]};
    uint64_t p;
    (void)dict_member_rank(s, ds, t, &p);
    pos[j] = p;
}

// #{j : pos[j] <= i} over the sorted merge positions (U is small: cache-resident)
__device__ inline uint64_t merged_before(const uint64_t* pos, uint64_t U, uint64_t i)
{
    uint64_t lo = 0, hi = U;
    while (lo < hi)
    {
        const uint64_t m = (lo + hi) >> 1;
        if (pos[m] <= i) lo = m + 1;
        else hi = m;
    }
    return lo;
}

__device__ inline uint32_t remap_rank(uint32_t r, const uint64_t* pos, uint64_t U)
{
    if (r == 0) return 0;                       // NONE
    const uint64_t i = (r - 1) >> 1;            // every stored rank is a member rank
    return (uint32_t)(2 * (i + merged_before(pos, U, i)) + 1);
}

struct DictArrays { uint64_t* hi; uint64_t* lo; int32_t* node; uint64_t* raw; };

__global__ __launch_bounds__(256) void k_merge_old(DevSnapshot s, const uint64_t* raw, const uint64_t* pos, uint64_t U, DictArrays nd)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= s.n_dict) return;
    const uint64_t p = i + merged_before(pos, U, i);
    nd.hi[p] = s.dict_hi[i];
    nd.lo[p] = s.dict_lo[i];
    nd.node[p] = s.dict_node[i];
    nd.raw[p] = raw[i];
}

__global__ void k_merge_new(uint64_t U, const uint64_t* uh, const uint64_t* ul, const int32_t* un, const uint64_t* uraw,
                            const uint64_t* pos, DictArrays nd)
{
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= U) return;
    const uint64_t p = pos[j] + j;
    nd.hi[p] = uh[j];
    nd.lo[p] = ul[j];
    nd.node[p] = un[j];
    nd.raw[p] = uraw[j];
}

__global__ __launch_bounds__(256) void k_remap_entries(uint64_t ne, uint2* ent, uint32_t* xrank, const uint64_t* pos, uint64_t U)
{
    const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= ne) return;
    const uint32_t y = ent[e].y;
    ent[e].y = (y & ~RANK_MASK) | remap_rank(y & RANK_MASK, pos, U);
    xrank[e] = remap_rank(xrank[e], pos, U);
}

__global__ void k_remap_krec(uint64_t nk, KeyRec* krec, const uint64_t* pos, uint64_t U)
{
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nk) return;
    KeyRec kr = krec[k];
    kr.last_txn = remap_rank(kr.last_txn, pos, U);
    kr.last_wexec = remap_rank(kr.last_wexec, pos, U);
    kr.pruned = remap_rank(kr.pruned, pos, U);
    krec[k] = kr;
}

// txw words (rank | kind << RANK_BITS) of the range entries and stabbing cells, watermark ranks
__global__ void k_remap_txw(uint64_t n, uint32_t* txw, const uint64_t* pos, uint64_t U)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t y = txw[i];
    txw[i] = (y & ~RANK_MASK) | remap_rank(y & RANK_MASK, pos, U);
}

__global__ void k_remap_cells(uint64_t n, uint64_t* cell, const uint64_t* pos, uint64_t U)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t v = cell[i];
    const uint32_t y = (uint32_t)v;
    cell[i] = (v & 0xFFFFFFFF00000000ull) | ((y & ~RANK_MASK) | remap_rank(y & RANK_MASK, pos, U));
}

// ---- keys without a CommandsForKey: the update creates one (an empty byId the insertion then
// fills). New keys are merged into the sorted key array; every key index moves up by the new keys
// below it (monotone: segments keep their order), the key hash is rebuilt.
__device__ inline uint32_t key_index(const DevSnapshot& s, int64_t key)
{
    if (!s.n_keys) return KEY_EMPTY;
    uint64_t h = key_hash(key) & s.khash_mask;
    for (;;)
    {
        const KeySlot sl = s.khash[h];
        if (sl.idx == KEY_EMPTY) return KEY_EMPTY;
        if (sl.key == key) return sl.idx;
        h = (h + 1) & s.khash_mask;
    }
}

__global__ void k_key_collect(DevSnapshot s, CfkUpdIn u, uint64_t* out, UpdCtl* ctl)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= u.n) return;
    const int64_t key = u.keys[i];
    if (key_index(s, key) != KEY_EMPTY) return;
    const uint64_t x = (uint64_t)key ^ 0x8000000000000000ull;     // unsigned sort order
    out[atomicAdd(&ctl->n_newk, 1u)] = x;
    const uint64_t d = x ^ ((uint64_t)u.keys[0] ^ 0x8000000000000000ull);
    if (d) atomicOr(&ctl->kdiff, (unsigned long long)d);
}

__global__ void k_key_unique(const uint64_t* ks, uint64_t m, uint32_t* flag)
{
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r < m) flag[r] = (r == 0 || ks[r] != ks[r - 1]) ? 1u : 0u;
}

// the unique new keys (sorted) and their lower bounds among the old keys
__global__ void k_key_place(DevSnapshot s, const uint64_t* ks, uint64_t m, const uint32_t* flag, const uint64_t* pos_in,
                            int64_t* nkeys, uint64_t* kpos)
{
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= m || !flag[r]) return;
    const int64_t key = (int64_t)(ks[r] ^ 0x8000000000000000ull);
    uint64_t lo = 0, hi = s.n_keys;
    while (lo < hi)
    {
        const uint64_t mid = (lo + hi) >> 1;
        if (s.keys[mid] < key) lo = mid + 1;
        else hi = mid;
    }
    nkeys[pos_in[r]] = key;
    kpos[pos_in[r]] = lo;
}

__global__ __launch_bounds__(256) void k_key_move(DevSnapshot s, const uint32_t* kcell, const uint64_t* kpos, uint64_t U,
                                                  KeyBufs nb, uint32_t* kmap)
{
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= s.n_keys) return;
    const uint64_t p = k + merged_before(kpos, U, k);
    kmap[k] = (uint32_t)p;
    nb.keys[p] = s.keys[k];
    nb.krec[p] = s.krec[k];
    nb.kcell[p] = kcell ? kcell[k] : NO_CELL;
}

__global__ void k_key_new(DevSnapshot s, const int64_t* nkeys, const uint64_t* kpos, uint64_t U, KeyBufs nb)
{
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= U) return;
    const uint64_t p = kpos[j] + j;
    const int64_t key = nkeys[j];
    const uint32_t at = kpos[j] < s.n_keys ? s.krec[kpos[j]].seg_lo : (uint32_t)s.n_ent;
    KeyRec r;
    r.seg_lo = r.seg_hi = at;
    r.w_lo = r.w_hi = 0;
    r.last_txn = r.last_wexec = r.pruned = 0;
    r.maw = -1;
    nb.keys[p] = key;
    nb.krec[p] = r;
    uint32_t cell = NO_CELL;
    if (s.cell_off)
    {
        // the key's cell of the range stabbing index (as the ingest places it)
        uint64_t lo = 0, hi = s.n_cell_E;
        while (lo < hi)
        {
            const uint64_t mid = (lo + hi) >> 1;
            const int64_t v = s.cell_E[mid];
            if (s.start_inclusive ? v <= key : v < key) lo = mid + 1;
            else hi = mid;
        }
        cell = (uint32_t)lo;
    }
    nb.kcell[p] = cell;
}

// entries' key indices through the old -> new key index map k_key_move wrote (one gather per entry, not a
// search of the new keys' positions)
__global__ __launch_bounds__(256) void k_ekey_remap(uint64_t ne, uint32_t* ekey, const uint32_t* kmap)
{
    const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e < ne) ekey[e] = kmap[ekey[e]];
}

__global__ void k_khash_clear(KeySlot* h, uint64_t n)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) h[i] = KeySlot{0, KEY_EMPTY, NO_CELL};
}

__global__ void k_khash_fill(uint64_t nk, KeyBufs nb)
{
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nk) return;
    const int64_t key = nb.keys[k];
    const uint64_t mask = nb.hcap - 1;
    uint64_t h = key_hash(key) & mask;
    while (atomicCAS(&nb.khash[h].idx, KEY_EMPTY, (uint32_t)k) != KEY_EMPTY) h = (h + 1) & mask;
    nb.khash[h].key = key;
    nb.khash[h].cell = nb.kcell[k];
}

// insertion updates sorted by (key index, txn rank): group starts
__global__ void k_ins_gflags(const uint64_t* ks, uint64_t q, uint32_t* gflag)
{
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j < q) gflag[j] = (j == 0 || ks[j] != ks[j - 1]) ? 1u : 0u;
}

// ordered compaction of the flagged updates (flags[i], exclusive prefix pos[i]): key, update index
__global__ void k_compact(uint64_t n, const uint32_t* flags, const uint64_t* pos, const uint64_t* key, const uint32_t* loc,
                          uint64_t* ks, uint32_t* vs)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || !flags[i]) return;
    ks[pos[i]] = key ? key[i] : (uint64_t)loc[i];
    vs[pos[i]] = (uint32_t)i;
}

// with ballots: the updates of one present entry (sorted by entry, batch order within) fold in
// order through CommandsForKey.update's replacement test; the entry's old state is kept at its
// first update's index for a rollback
// uapp (non-null): per update 1 = applied (replaced the entry when its turn came), 2 = the last
// applied update of its entry (the entry's TxnInfo comes from it). Without ballots anywhere
// (d.ballot null) every ballot is Ballot.ZERO.
__global__ void k_fold_present(uint64_t m, const uint64_t* ks, const uint32_t* vs, CfkUpdIn u, const uint32_t* xr,
                               CfkDevState d, uint2* bk, Bal* bkb, uint8_t* chg, UpdCtl* ctl, uint8_t* uapp)
{
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= m || (j > 0 && ks[j - 1] == ks[j])) return;
    const uint32_t e = (uint32_t)ks[j];
    uint32_t st = d.status[e], x = d.xrank[e];
    Bal b = d.ballot ? d.ballot[e] : Bal{0, 0, 0, 0};
    unsigned long long cnt = 0;
    uint32_t last = 0xFFFFFFFFu;
    for (uint64_t t = j; t < m && ks[t] == e; ++t)
    {
        const uint32_t i = vs[t], ns = u.status[i];
        const Bal nb = upd_ballot(u, i);
        if (uapp) uapp[i] = 0;
        if (!replaces(ns, st, nb, b)) continue;
        st = ns;
        x = xr[i];
        b = kept_ballot(ns, nb);
        ++cnt;
        if (uapp) uapp[i] = 1;
        last = i;
    }
    if (!cnt) return;
    if (uapp) uapp[last] = 3;
    const uint32_t i0 = vs[j];
    bk[i0] = make_uint2(d.status[e], d.xrank[e]);
    if (d.ballot) bkb[i0] = d.ballot[e];
    d.status[e] = (uint8_t)st;
    d.xrank[e] = x;
    if (d.ballot) d.ballot[e] = b;
    chg[e] = 1;
    atomicAdd(&ctl->applied, cnt);
}

// per group (one new entry), with ballots: the group's updates fold in batch order (the first
// inserts); gword = final status << 32 | ~(update index the entry takes executeAt and ballot from)
__global__ void k_ins_fold(const uint64_t* ks, const uint32_t* vs, uint64_t q, const uint32_t* gflag, const uint64_t* gs,
                           CfkUpdIn u, unsigned long long* gword, uint32_t* gkey, uint32_t* grank, UpdCtl* ctl, uint8_t* uapp)
{
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= q || !gflag[j]) return;
    const uint64_t g = gs[j];
    gkey[g] = (uint32_t)(ks[j] >> 32);
    grank[g] = (uint32_t)ks[j];
    uint32_t il = vs[j], st = u.status[il];
    Bal b = kept_ballot(st, upd_ballot(u, il));
    unsigned long long cnt = 0;
    if (uapp) uapp[il] = 1;                   // the insertion
    for (uint64_t t = j + 1; t < q && ks[t] == ks[j]; ++t)
    {
        const uint32_t i = vs[t], ns = u.status[i];
        const Bal nb = upd_ballot(u, i);
        if (uapp) uapp[i] = 0;
        if (!replaces(ns, st, nb, b)) continue;
        st = ns;
        il = i;
        b = kept_ballot(ns, nb);
        ++cnt;
        if (uapp) uapp[i] = 1;
    }
    if (uapp) uapp[il] = 3;
    gword[g] = ((unsigned long long)st << 32) | (0xFFFFFFFFull - il);
    if (cnt) atomicAdd(&ctl->applied, cnt);
}

// per group (one new entry): the first update of the highest status wins (batch order)
__global__ void k_ins_claim(const uint64_t* ks, const uint32_t* vs, uint64_t q, const uint32_t* gflag, const uint64_t* gs,
                            const uint8_t* status, unsigned long long* gword, uint32_t* gkey, uint32_t* grank)
{
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= q) return;
    const uint64_t g = gs[j] + gflag[j] - 1;
    if (gflag[j])
    {
        gkey[g] = (uint32_t)(ks[j] >> 32);
        grank[g] = (uint32_t)ks[j];
    }
    const uint32_t i = vs[j];
    atomicMax(gword + g, ((unsigned long long)status[i] << 32) | (0xFFFFFFFFull - i));
}

// ib[k] = new entries of keys below k (k <= n_keys)
__global__ void k_ins_before(uint64_t nk, const uint32_t* gkey, uint64_t G, uint32_t* ib)
{
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k > nk) return;
    uint64_t lo = 0, hi = G;
    while (lo < hi)
    {
        const uint64_t m = (lo + hi) >> 1;
        if (gkey[m] < k) lo = m + 1;
        else hi = m;
    }
    ib[k] = (uint32_t)lo;
}

struct EntArrays { uint2* ent; uint8_t* status; uint32_t* xrank; uint32_t* ekey; Bal* bal; uint8_t* chg; uint32_t* mref; };

// an old entry moves up by the new entries before it: those of lower keys, and those of its key
// with a lower rank (a mid-segment insert, :1002-1007)
__global__ __launch_bounds__(256) void k_ins_move_old(uint64_t ne, EntArrays a, const uint32_t* ib, const uint32_t* grank,
                                                      EntArrays b, uint32_t* mv)
{
    const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= ne) return;
    const uint32_t k = a.ekey[e];
    uint32_t lo = ib[k], hi = ib[k + 1];
    if (lo < hi)
    {
        const uint32_t r = a.ent[e].y & RANK_MASK;
        while (lo < hi)
        {
            const uint32_t m = (lo + hi) >> 1;
            if (grank[m] < r) lo = m + 1;
            else hi = m;
        }
    }
    const uint64_t p = e + lo;
    b.ent[p] = a.ent[e];
    b.status[p] = a.status[e];
    b.xrank[p] = a.xrank[e];
    b.ekey[p] = k;
    if (b.bal) b.bal[p] = a.bal[e];
    if (b.mref) b.mref[p] = a.mref[e];
    b.chg[p] = a.chg[e];
    mv[e] = (uint32_t)p;
}

// a new entry lands after the old entries below it (its insertPos, -1 - binarySearch) and the new
// entries before it (g)
__global__ void k_ins_place(uint64_t G, const uint32_t* gkey, const uint32_t* grank, const unsigned long long* gword,
                            const KeyRec* krec, const uint2* old_ent, CfkUpdIn u, const uint32_t* xr, EntArrays b)
{
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= G) return;
    const uint32_t k = gkey[g];
    const unsigned long long wd = gword[g];
    const uint32_t i = (uint32_t)(0xFFFFFFFFull - (uint32_t)wd);
    const KeyRec kr = krec[k];
    uint32_t lo = kr.seg_lo, hi = kr.seg_hi;
    if (kr.seg_hi > kr.seg_lo && grank[g] < kr.last_txn)
        while (lo < hi)
        {
            const uint32_t m = (lo + hi) >> 1;
            if ((old_ent[m].y & RANK_MASK) < grank[g]) lo = m + 1;
            else hi = m;
        }
    else lo = kr.seg_hi;
    const uint64_t p = (uint64_t)lo + g;
    const uint32_t kind = (uint32_t)((u.txn_lsb[i] >> 1) & 7);
    b.ent[p] = make_uint2(0u, grank[g] | (kind << RANK_BITS));
    b.status[p] = (uint8_t)(wd >> 32);
    b.xrank[p] = xr[i];
    b.ekey[p] = k;
    if (b.bal) b.bal[p] = kept_ballot((uint32_t)(wd >> 32), upd_ballot(u, i));
    if (b.mref) b.mref[p] = MREF_BORN;
    b.chg[p] = 1;
}

__global__ void k_ins_krec(uint64_t nk, const uint32_t* ib, const uint32_t* grank, KeyRec* krec)
{
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nk) return;
    KeyRec kr = krec[k];
    const uint32_t a = ib[k], b = ib[k + 1];
    kr.seg_lo += a;
    kr.seg_hi += b;
    if (b > a && grank[b - 1] > kr.last_txn) kr.last_txn = grank[b - 1];
    krec[k] = kr;
}

// after a failed locate: release every claimed entry
__global__ void k_upd_release(uint64_t n, const uint32_t* loc, unsigned long long* word)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && loc[i] != 0xFFFFFFFFu) word[loc[i]] = 0;
}

// the claiming update of each entry applies if its status is above the entry's; the entry's old
// state is kept in bk[i] for a rollback
__global__ void k_upd_apply(uint64_t n, const uint32_t* loc, const uint32_t* xr, unsigned long long* word,
                            CfkDevState d, uint2* bk, Bal* bkb, uint8_t* chg, UpdCtl* ctl)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t e = loc[i];
    if (e == LOC_NONE) return;                 // an insertion
    const unsigned long long wd = word[e];
    if ((uint32_t)wd != (uint32_t)(0xFFFFFFFFull - i)) return;
    word[e] = 0;
    const uint32_t st = (uint32_t)(wd >> 32);
    const uint32_t cur = d.status[e];
    if (st <= cur) return;
    bk[i] = make_uint2(cur, d.xrank[e]);
    d.status[e] = (uint8_t)st;
    d.xrank[e] = xr[i];
    chg[e] = 1;
    if (d.ballot)
    {
        // the batch carries Ballot.ZERO: the replacing TxnInfo has no ballot
        bkb[i] = d.ballot[e];
        d.ballot[e] = Bal{0, 0, 0, 0};
    }
    atomicAdd(&ctl->applied, 1ull);
}

__global__ void k_upd_rollback(uint64_t n, const uint32_t* loc, const uint2* bk, const Bal* bkb, CfkDevState d)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || bk[i].x == 0xFFFFFFFFu) return;
    d.status[loc[i]] = (uint8_t)bk[i].x;
    d.xrank[loc[i]] = bk[i].y;
    if (d.ballot) d.ballot[loc[i]] = bkb[i];
}

// ---- derivation (thread per entry): tau, never-elided class flags, committed flag
__global__ __launch_bounds__(256) void k_drv_flags(uint64_t ne, CfkDevState d, uint32_t* flags)
{
    const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= ne) return;
    const uint32_t st = d.status[e], y = d.ent[e].y, kind = y >> RANK_BITS;
    const uint32_t tau = tau_of(st, kind, d.xrank[e]);
    d.ent[e].x = tau;
    for (int cl = 0; cl < NCLASS; ++cl)
        flags[cl * ne + e] = tau == TAU_NEVER_ELIDED ? ((CLASS_KINDS[cl] >> kind) & 1u) : 0u;
    flags[3 * ne + e] = (st >= AD_ST_COMMITTED && st <= AD_ST_APPLIED) ? 1u : 0u;
}

__global__ void k_drv_totals(const uint64_t* fs, uint64_t n, int n_arrays, uint64_t* tot)
{
    if ((int)threadIdx.x < n_arrays) tot[threadIdx.x] = fs[threadIdx.x * (n + 1) + n];
}

// cand (class-major, byId order) and the committed entries keyed (key index, executeAt rank)
__global__ __launch_bounds__(256) void k_drv_scatter(uint64_t ne, CfkDevState d, const uint64_t* fs, const UpdCtl* ctl,
                                                     uint32_t* cand, uint64_t* ck, uint32_t* cv)
{
    const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= ne) return;
    const uint2 en = d.ent[e];
    const uint32_t kind = en.y >> RANK_BITS;
    if (en.x == TAU_NEVER_ELIDED)
    {
        uint64_t base = 0;
        for (int cl = 0; cl < NCLASS; ++cl)
        {
            if ((CLASS_KINDS[cl] >> kind) & 1u) cand[base + fs[cl * (ne + 1) + e]] = en.y;
            base += ctl->tot[cl];
        }
    }
    const uint32_t st = d.status[e];
    if (ck && st >= AD_ST_COMMITTED && st <= AD_ST_APPLIED)
    {
        const uint64_t j = fs[3 * (ne + 1) + e];
        ck[j] = ((uint64_t)d.ekey[e] << 32) | d.xrank[e];
        cv[j] = (uint32_t)e;
    }
}

// sorted committed entries: duplicate executeAt check, cwr (Read/Write) and w (Write) flags
__global__ __launch_bounds__(256) void k_drv_committed(uint64_t ncm, const uint64_t* ck, const uint32_t* cv,
                                                       CfkDevState d, uint32_t* f2, UpdCtl* ctl)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= ncm) return;
    if (i > 0 && ck[i - 1] == ck[i]) upd_fail(ctl, UE_DUP_EXEC, cv[i]);
    const uint32_t kind = d.ent[cv[i]].y >> RANK_BITS;
    f2[i] = (KINDS_RS_OR_WS >> kind) & 1u;
    f2[ncm + i] = kind == AD_KIND_WRITE ? 1u : 0u;
    f2[2 * ncm + i] = (kind == AD_KIND_WRITE && d.status[cv[i]] == AD_ST_APPLIED) ? 1u : 0u;
}

__global__ __launch_bounds__(256) void k_drv_emit(uint64_t ncm, uint64_t ne, const uint64_t* ck, const uint32_t* cv,
                                                  CfkDevState d, const uint64_t* fs, const uint64_t* s2,
                                                  uint32_t* cwr, uint2* w, int32_t* maw, uint32_t* wtail)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= ncm) return;
    const uint32_t e = cv[i];
    const uint32_t y = d.ent[e].y, kind = y >> RANK_BITS;
    if ((KINDS_RS_OR_WS >> kind) & 1u) cwr[s2[i]] = y;
    if (kind != AD_KIND_WRITE) return;
    const uint64_t p = s2[(ncm + 1) + i];
    const uint32_t k = (uint32_t)(ck[i] >> 32);
    w[p] = make_uint2((uint32_t)ck[i], y & RANK_MASK);
    const uint64_t cm_hi = fs[3 * (ne + 1) + d.krec[k].seg_hi];
    if (p + 1 == s2[(ncm + 1) + cm_hi]) wtail[k] = (uint32_t)s2[i];     // the key's last Write: its cwr index
    // maxAppliedWriteByExecuteAt: the key's last APPLIED Write (no atomics: hot keys hold ~10^6)
    if (d.status[e] == AD_ST_APPLIED && s2[2 * (ncm + 1) + i] + 1 == s2[2 * (ncm + 1) + cm_hi]) maw[k] = (int32_t)p;
}

__global__ __launch_bounds__(256) void k_drv_keys(uint64_t nk, uint64_t ne, uint64_t ncm, CfkDevState d, const uint64_t* fs,
                                                  const uint64_t* s2, const uint2* w, const int32_t* maw,
                                                  const uint32_t* wtail, const UpdCtl* ctl)
{
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nk) return;
    KeyRec kr = d.krec[k];
    const uint64_t cm_lo = fs[3 * (ne + 1) + kr.seg_lo], cm_hi = fs[3 * (ne + 1) + kr.seg_hi];
    const uint32_t cwr_lo = (uint32_t)s2[cm_lo], cwr_hi = (uint32_t)s2[cm_hi];
    const uint32_t w_lo = (uint32_t)s2[(ncm + 1) + cm_lo], w_hi = (uint32_t)s2[(ncm + 1) + cm_hi];
    const bool has_w = w_hi > w_lo;
    const uint2 lw = has_w ? w[w_hi - 1] : make_uint2(0u, 0u);
    kr.w_lo = w_lo;
    kr.w_hi = w_hi;
    kr.last_wexec = lw.x;
    kr.maw = maw[k];
    d.krec[k] = kr;
    KeyEntry ke;
    ke.last_txn = kr.last_txn;
    ke.last_wexec = lw.x;
    ke.last_w_txn = lw.y;
    ke.pad = 0;
    uint64_t base = 0;
    for (int cl = 0; cl < NCLASS; ++cl)
    {
        ke.cl[cl].cand_lo = (uint32_t)(base + fs[cl * (ne + 1) + kr.seg_lo]);
        ke.cl[cl].cand_hi = (uint32_t)(base + fs[cl * (ne + 1) + kr.seg_hi]);
        ke.cl[cl].cwr_tail = has_w ? wtail[k] : cwr_lo;
        ke.cl[cl].cwr_hi = cwr_hi;
        base += ctl->tot[cl];
    }
    d.kent[k] = ke;
}

// ---- incremental committedByExecuteAt (the (key index, executeAt rank) order of the committed
// entries): the last batch's order minus the entries this batch changed (moved by the insertion
// map), merged with the changed entries that are committed now (sorted on their own) -- linear
// passes instead of a radix sort of every committed entry.
__global__ void k_cm_keep(uint64_t m, const uint32_t* cm, const uint32_t* mv, const uint8_t* chg, uint32_t* f)
{
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= m) return;
    const uint32_t e = mv ? mv[cm[j]] : cm[j];
    f[j] = chg[e] ? 0u : 1u;
}

__global__ __launch_bounds__(256) void k_cm_changed(uint64_t ne, CfkDevState d, const uint8_t* chg, uint32_t* f)
{
    const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= ne) return;
    const uint32_t st = d.status[e];
    f[e] = (chg[e] && st >= AD_ST_COMMITTED && st <= AD_ST_APPLIED) ? 1u : 0u;
}

__global__ void k_cm_compact(uint64_t m, const uint32_t* src, const uint32_t* mv, const uint32_t* f, const uint64_t* pos,
                             CfkDevState d, uint64_t* ko, uint32_t* vo)
{
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= m || !f[j]) return;
    uint32_t e = src ? src[j] : (uint32_t)j;
    if (mv) e = mv[e];
    const uint64_t p = pos[j];
    ko[p] = ((uint64_t)d.ekey[e] << 32) | d.xrank[e];
    vo[p] = e;
}

// each block merges CM_TILE consecutive elements of one list into the output: the block's first and last
// element bound its window in the other list (two searches per block, ~20 dependent loads each -- one block
// per 256 elements, as before round 6, spent most of the merge on them), each thread then searches only that
// window, from its previous element's place on (its elements ascend)
constexpr uint32_t CM_ITEMS = 8, CM_TILE = 256 * CM_ITEMS;

__global__ __launch_bounds__(256) void k_cm_merge(uint64_t na, const uint64_t* ka, const uint32_t* va, uint64_t nb,
                                                  const uint64_t* kb, const uint32_t* vb, uint64_t* ko, uint32_t* vo)
{
    __shared__ uint64_t win[2];
    const uint64_t blocks_a = (na + CM_TILE - 1) / CM_TILE;
    const bool from_a = blockIdx.x < blocks_a;
    const uint64_t base = from_a ? (uint64_t)blockIdx.x * CM_TILE : ((uint64_t)blockIdx.x - blocks_a) * CM_TILE;
    const uint64_t nself = from_a ? na : nb, nother = from_a ? nb : na;
    const uint64_t* self = from_a ? ka : kb;
    const uint64_t* o = from_a ? kb : ka;
    // A before B on equal keys (a duplicate executeAt, reported by k_drv_committed)
    auto bound = [&](uint64_t x, uint64_t lo, uint64_t hi) {
        while (lo < hi)
        {
            const uint64_t mid = (lo + hi) >> 1;
            if (from_a ? o[mid] < x : o[mid] <= x) lo = mid + 1;
            else hi = mid;
        }
        return lo;
    };
    const uint64_t last = min(base + CM_TILE, nself) - 1;
    if (threadIdx.x == 0) win[0] = bound(self[base], 0, nother);
    if (threadIdx.x == 64) win[1] = bound(self[last], 0, nother);
    __syncthreads();
    uint64_t lo = win[0];
    const uint64_t hi = win[1];
#pragma unroll
    for (uint32_t j = 0; j < CM_ITEMS; ++j)
    {
        const uint64_t i = base + (uint64_t)j * 256 + threadIdx.x;
        if (i >= nself) break;
        const uint64_t x = self[i];
        lo = bound(x, lo, hi);
        const uint64_t p = i + lo;
        ko[p] = x;
        vo[p] = from_a ? va[i] : vb[i];
    }
}

unsigned blocks(uint64_t n, unsigned t = 256) { return (unsigned)std::max<uint64_t>(1, (n + t - 1) / t); }

// grows with slack (insertions raise the entry count every batch: no reallocation, and no re-zeroing
// of `word`, per batch); zero: the whole new allocation is zeroed
struct DBuf : DevBuf {
    bool ensure(size_t b, bool zero = false) { return grow(b, zero); }
};

}  // namespace

struct CfkUpdWork {
    DBuf ctl, loc, xr, word, bk, flags, fs, bsum, ck, cv, ck2, cv2, hist, hoff, f2, s2, maw, wtail, kmap;
    DBuf sm_hi, sm_lo, sm_node;
    DBuf nw, nk_a, nk_b, nv_a, nv_b, nflag, npos, ins_k, ins_v, gflag, gs, gword, gkey, grank, ib, krec_bk;
    DBuf mh, ml, mn, mraw, mpos;
    DBuf bkb, uflag, upos, rk;
    // missing() maintenance: per update applied flags, dep ranks, additions batch, derivation
    DBuf uapp, drank, acnt, aoff, a_k, a_tm, a_tl, a_tn, a_st, dsrc, mflag, mpp, mpend, mcnt, moff;
    // byId's last txnId as each update sees it (additions past the end) and the LoadPruned ids
    DBuf trk, pk, pv, pk2, pv2, pvv, pw, pe, pbm, plast, ppos, lcnt, loff, l_k, l_tm, l_tl, l_tn, l_i;
    DBuf kn_a, kn_b, kv_a, kv_b, kflag, kfpos, knew, kpos;   // new keys
    DBuf tpos, twm, ids_st, ids_rank;                          // RedundantBefore truncation / dictionary ensure
    // incremental committed order: the last derivation's order (entry indices), per-entry changed
    // flags (double-buffered with the entry arrays), the insertion's old -> new entry map
    DBuf cm, chg[2], mv, af, ap, bfl, bps, cka, cva, ckb, cvb, ckb2, cvb2;
    int chg_cur = 0;
    uint64_t cm_n = 0;
    bool cm_valid = false, moved = false;
    UpdCtl* h_ctl = nullptr;
    hipEvent_t ev[3] = {};
    ~CfkUpdWork()
    {
        if (h_ctl) (void)hipHostFree(h_ctl);
        for (auto& e : ev)
            if (e) (void)hipEventDestroy(e);
    }
};

CfkUpdWork* cfk_upd_work_create() { return new CfkUpdWork(); }
void cfk_upd_work_invalidate(CfkUpdWork* w)
{
    if (w) w->cm_valid = false;
}
void cfk_upd_work_destroy(CfkUpdWork* w) { delete w; }

static uint32_t bytes_of(uint64_t v)
{
    uint32_t b = 0;
    while (v) { ++b; v >>= 8; }
    return b;
}

#define UCHK(expr)                                                                                \
    do {                                                                                          \
        hipError_t _e = (expr);                                                                   \
        if (_e != hipSuccess) { *err = std::string(#expr) + ": " + hipGetErrorString(_e); return AD_E_DEVICE; } \
    } while (0)
#define UALLOC_V(buf, bytes)                                                                      \
    do {                                                                                          \
        if (!(buf).ensure((bytes), false)) return DictSample{nullptr, nullptr, nullptr, 0};       \
    } while (0)
#define UALLOC(buf, bytes, zero)                                                                  \
    do {                                                                                          \
        if (!(buf).ensure((bytes), (zero))) { *err = "device allocation (cfk update)"; return AD_E_NOMEM; } \
    } while (0)

static uint32_t key_rank_mask(uint64_t n_dict, uint64_t nk);

// Rebuild ent.tau, cand, cwr, w, krec, kent and the trees from the per-entry state (status,
// executeAt rank). A duplicate committed executeAt is reported in ctl->err.
static int cfk_derive(CfkUpdWork* w, DevSnapshot& s, const CfkDevState& dd, CfkDerivedBufs* bufs,
                      int (*need)(void*, uint64_t, uint64_t, uint64_t, CfkDerivedBufs*), void* need_ctx, hipStream_t st,
                      std::string* err, bool incr = false)
{
    const uint64_t ne = s.n_ent, nk = s.n_keys;
    UpdCtl* ctl = w->ctl.as<UpdCtl>();
    const uint64_t sb = (std::max<uint64_t>(ne, 1) + 1023) / 1024 + 8;
    UALLOC(w->flags, 4ull * 4 * std::max<uint64_t>(ne, 1), false);
    UALLOC(w->fs, 8ull * 4 * (ne + 1), false);
    UALLOC(w->bsum, 8ull * 4 * sb + 8 * (radix_hist_entries(ne) / 1024 + 8), false);
    if (ne)
    {
        k_drv_flags<<<blocks(ne), 256, 0, st>>>(ne, dd, w->flags.as<uint32_t>());
        UCHK(hipGetLastError());
    }
    UCHK(run_scan_arrays(w->flags.as<uint32_t>(), w->fs.as<uint64_t>(), ne, 4, w->bsum.as<uint64_t>(), st));
    k_drv_totals<<<1, 64, 0, st>>>(w->fs.as<uint64_t>(), ne, 4, ctl->tot);
    // incremental committed order: flags of the kept old entries and of the changed committed ones
    const bool inc = incr && w->cm_valid && ne;
    const uint64_t m0 = inc ? w->cm_n : 0;
    const uint8_t* chg = w->chg[w->chg_cur].as<uint8_t>();
    const uint32_t* mv = w->moved ? w->mv.as<uint32_t>() : nullptr;
    if (inc)
    {
        UALLOC(w->af, 4 * std::max<uint64_t>(m0, 1), false);
        UALLOC(w->ap, 8 * (m0 + 1), false);
        UALLOC(w->bfl, 4 * ne, false);
        UALLOC(w->bps, 8 * (ne + 1), false);
        if (m0) k_cm_keep<<<blocks(m0), 256, 0, st>>>(m0, w->cm.as<uint32_t>(), mv, chg, w->af.as<uint32_t>());
        UCHK(run_scan_arrays(w->af.as<uint32_t>(), w->ap.as<uint64_t>(), m0, 1, w->bsum.as<uint64_t>(), st));
        k_drv_totals<<<1, 64, 0, st>>>(w->ap.as<uint64_t>(), m0, 1, ctl->cm);
        k_cm_changed<<<blocks(ne), 256, 0, st>>>(ne, dd, chg, w->bfl.as<uint32_t>());
        UCHK(run_scan_arrays(w->bfl.as<uint32_t>(), w->bps.as<uint64_t>(), ne, 1, w->bsum.as<uint64_t>(), st));
        k_drv_totals<<<1, 64, 0, st>>>(w->bps.as<uint64_t>(), ne, 1, ctl->cm + 1);
        UCHK(hipGetLastError());
    }
    UCHK(d2h(w->h_ctl, ctl, sizeof(UpdCtl), st));
    UCHK(hipStreamSynchronize(st));
    const uint64_t n_cand = w->h_ctl->tot[0] + w->h_ctl->tot[1] + w->h_ctl->tot[2], ncm = w->h_ctl->tot[3];
    host_trace("derive: totals sync");
    const uint64_t nA = inc ? w->h_ctl->cm[0] : 0, nB = inc ? w->h_ctl->cm[1] : 0;
    const bool use_inc = inc && nA + nB == ncm;     // else (never expected) the full sort
    int rc = need(need_ctx, n_cand, ncm, ncm, bufs);
    if (rc) return rc;
    UALLOC(w->ck, 8 * std::max<uint64_t>(ncm, 1), false);
    UALLOC(w->cv, 4 * std::max<uint64_t>(ncm, 1), false);
    UALLOC(w->ck2, 8 * std::max<uint64_t>(ncm, 1), false);
    UALLOC(w->cv2, 4 * std::max<uint64_t>(ncm, 1), false);
    const uint64_t hist_n = radix_hist_entries(std::max<uint64_t>(ncm, 1));
    UALLOC(w->hist, 4 * hist_n, false);
    UALLOC(w->hoff, 8 * (hist_n + 1), false);
    UALLOC(w->f2, 4ull * 3 * std::max<uint64_t>(ncm, 1), false);
    UALLOC(w->s2, 8ull * 3 * (ncm + 1), false);
    UALLOC(w->maw, 4 * std::max<uint64_t>(nk, 1), false);
    UALLOC(w->wtail, 4 * std::max<uint64_t>(nk, 1), false);
    const uint64_t sb2 = (std::max<uint64_t>(std::max(ncm, hist_n), 1) + 1023) / 1024 + 8;
    UALLOC(w->bsum, 8ull * std::max<uint64_t>(4 * sb, 3 * sb2), false);
    if (ne)
        k_drv_scatter<<<blocks(ne), 256, 0, st>>>(ne, dd, w->fs.as<uint64_t>(), ctl, bufs->cand,
                                                  use_inc ? nullptr : w->ck.as<uint64_t>(), w->cv.as<uint32_t>());
    uint64_t* ks = w->ck.as<uint64_t>();
    uint32_t* vs = w->cv.as<uint32_t>();
    if (use_inc)
    {
        UALLOC(w->cka, 8 * std::max<uint64_t>(nA, 1), false);
        UALLOC(w->cva, 4 * std::max<uint64_t>(nA, 1), false);
        UALLOC(w->ckb, 8 * std::max<uint64_t>(nB, 1), false);
        UALLOC(w->cvb, 4 * std::max<uint64_t>(nB, 1), false);
        UALLOC(w->ckb2, 8 * std::max<uint64_t>(nB, 1), false);
        UALLOC(w->cvb2, 4 * std::max<uint64_t>(nB, 1), false);
        if (m0)
            k_cm_compact<<<blocks(m0), 256, 0, st>>>(m0, w->cm.as<uint32_t>(), mv, w->af.as<uint32_t>(), w->ap.as<uint64_t>(), dd,
                                                     w->cka.as<uint64_t>(), w->cva.as<uint32_t>());
        k_cm_compact<<<blocks(ne), 256, 0, st>>>(ne, nullptr, nullptr, w->bfl.as<uint32_t>(), w->bps.as<uint64_t>(), dd,
                                                 w->ckb.as<uint64_t>(), w->cvb.as<uint32_t>());
        uint64_t* kb = w->ckb.as<uint64_t>();
        uint32_t* vb = w->cvb.as<uint32_t>();
        if (nB > 1)
        {
            const uint64_t hb = radix_hist_entries(nB);
            UALLOC(w->hist, 4 * std::max(hist_n, hb), false);
            UALLOC(w->hoff, 8 * (std::max(hist_n, hb) + 1), false);
            UCHK(radix_sort_pairs(kb, vb, w->ckb2.as<uint64_t>(), w->cvb2.as<uint32_t>(), nB, key_rank_mask(s.n_dict, nk),
                                  w->hist.as<uint32_t>(), w->hoff.as<uint64_t>(), w->bsum.as<uint64_t>(), st, &kb, &vb));
        }
        if (ncm)
            k_cm_merge<<<(unsigned)((nA + CM_TILE - 1) / CM_TILE + (nB + CM_TILE - 1) / CM_TILE), 256, 0, st>>>(nA, w->cka.as<uint64_t>(),
                                                                                      w->cva.as<uint32_t>(), nB, kb, vb, ks, vs);
        UCHK(hipGetLastError());
    }
    else if (ncm > 1)
    {
        uint32_t mask = 0;
        const uint32_t xb = bytes_of(2 * s.n_dict + 1), kb = bytes_of(nk ? nk - 1 : 0);
        for (uint32_t b = 0; b < xb && b < 4; ++b) mask |= 1u << b;
        for (uint32_t b = 0; b < kb && b < 4; ++b) mask |= 1u << (4 + b);
        UCHK(radix_sort_pairs(ks, vs, w->ck2.as<uint64_t>(), w->cv2.as<uint32_t>(), ncm, mask, w->hist.as<uint32_t>(),
                              w->hoff.as<uint64_t>(), w->bsum.as<uint64_t>(), st, &ks, &vs));
    }
    if (ncm)
    {
        k_drv_committed<<<blocks(ncm), 256, 0, st>>>(ncm, ks, vs, dd, w->f2.as<uint32_t>(), ctl);
        UCHK(hipGetLastError());
    }
    UCHK(run_scan_arrays(w->f2.as<uint32_t>(), w->s2.as<uint64_t>(), ncm, 3, w->bsum.as<uint64_t>(), st));
    if (nk) UCHK(hipMemsetAsync(w->maw.p, 0xFF, 4 * nk, st));
    if (ncm)
        k_drv_emit<<<blocks(ncm), 256, 0, st>>>(ncm, ne, ks, vs, dd, w->fs.as<uint64_t>(), w->s2.as<uint64_t>(), bufs->cwr,
                                                bufs->w, w->maw.as<int32_t>(), w->wtail.as<uint32_t>());
    if (nk)
        k_drv_keys<<<blocks(nk), 256, 0, st>>>(nk, ne, ncm, dd, w->fs.as<uint64_t>(), w->s2.as<uint64_t>(), bufs->w,
                                               w->maw.as<int32_t>(), w->wtail.as<uint32_t>(), ctl);
    UCHK(hipGetLastError());
    // keep this committed order for the next batch's incremental derivation
    if (w->cm.cap < 4 * std::max<uint64_t>(ncm, 1))
    {
        UCHK(hipStreamSynchronize(st));       // the old order may still be read by queued kernels
        UALLOC(w->cm, 4 * std::max<uint64_t>(ncm, 1), false);
    }
    if (ncm) UCHK(hipMemcpyAsync(w->cm.p, vs, 4 * ncm, hipMemcpyDeviceToDevice, st));
    w->cm_n = ncm;
    w->cm_valid = true;
    s.cand = bufs->cand;
    s.cwr = bufs->cwr;
    s.w = bufs->w;
    UCHK(build_cfk_trees(s, st));
    host_trace("derive: queued");
    return AD_OK;
}

// the radix digits a (key index << 32 | rank) sort needs
static uint32_t key_rank_mask(uint64_t n_dict, uint64_t nk)
{
    uint32_t mask = 0;
    const uint32_t xb = bytes_of(2 * n_dict + 1), kb = bytes_of(nk ? nk - 1 : 0);
    for (uint32_t b = 0; b < xb && b < 4; ++b) mask |= 1u << b;
    for (uint32_t b = 0; b < kb && b < 4; ++b) mask |= 1u << (4 + b);
    return mask;
}

// Keys of the batch without a CommandsForKey: merged into the key arrays (spare buffers), entry key
// indices remapped, key hash rebuilt.
static int add_keys(CfkUpdWork* w, DevSnapshot& s, CfkDevState& d, const CfkUpdIn& u, const CfkGrow& grow, hipStream_t st,
                    CfkUpdOut* out, std::string* err)
{
    const uint64_t n = u.n, nk = s.n_keys, ne = s.n_ent;
    UpdCtl* ctl = w->ctl.as<UpdCtl>();
    UALLOC(w->kn_a, 8 * n, false);
    k_key_collect<<<blocks(n), 256, 0, st>>>(s, u, w->kn_a.as<uint64_t>(), ctl);
    UCHK(hipGetLastError());
    UCHK(d2h(w->h_ctl, ctl, sizeof(UpdCtl), st));
    UCHK(hipStreamSynchronize(st));
    const uint64_t m = w->h_ctl->n_newk;
    if (m == 0) return AD_OK;
    host_trace("add_keys: collect sync");
    UALLOC(w->kn_b, 8 * m, false);
    UALLOC(w->kv_a, 4 * m, false);
    UALLOC(w->kv_b, 4 * m, false);
    UALLOC(w->kflag, 4 * m, false);
    UALLOC(w->kfpos, 8 * (m + 1), false);
    const uint64_t hist_n = radix_hist_entries(m);
    UALLOC(w->hist, 4 * hist_n, false);
    UALLOC(w->hoff, 8 * (hist_n + 1), false);
    UALLOC(w->bsum, 8 * ((std::max(hist_n, m) + 1023) / 1024 + 8), false);
    uint64_t* ks = w->kn_a.as<uint64_t>();
    uint32_t* vs = w->kv_a.as<uint32_t>();
    k_iota<<<blocks(m), 256, 0, st>>>(vs, m);
    if (m > 1)
    {
        // only the bytes in which the keys differ (a key space of 2^20: three passes, not eight)
        uint32_t dm = 0;
        for (int dg = 0; dg < 8; ++dg)
            if ((w->h_ctl->kdiff >> (8 * dg)) & 0xFF) dm |= 1u << dg;
        UCHK(radix_sort_pairs(ks, vs, w->kn_b.as<uint64_t>(), w->kv_b.as<uint32_t>(), m, dm, w->hist.as<uint32_t>(),
                              w->hoff.as<uint64_t>(), w->bsum.as<uint64_t>(), st, &ks, &vs));
    }
    k_key_unique<<<blocks(m), 256, 0, st>>>(ks, m, w->kflag.as<uint32_t>());
    UCHK(run_scan_arrays(w->kflag.as<uint32_t>(), w->kfpos.as<uint64_t>(), m, 1, w->bsum.as<uint64_t>(), st));
    k_drv_totals<<<1, 64, 0, st>>>(w->kfpos.as<uint64_t>(), m, 1, &ctl->tot3[0]);
    UCHK(d2h(w->h_ctl, ctl, sizeof(UpdCtl), st));
    UCHK(hipStreamSynchronize(st));
    const uint64_t U = w->h_ctl->tot3[0];
    host_trace("add_keys: sort+unique sync");
    if (nk + U >= KEY_EMPTY) { *err = "more than 2^32-1 keys"; return AD_E_CAPACITY; }
    UALLOC(w->knew, 8 * U, false);
    UALLOC(w->kpos, 8 * U, false);
    k_key_place<<<blocks(m), 256, 0, st>>>(s, ks, m, w->kflag.as<uint32_t>(), w->kfpos.as<uint64_t>(), w->knew.as<int64_t>(),
                                           w->kpos.as<uint64_t>());
    KeyBufs nb{};
    if (int rc = grow.keys_spare(grow.ctx, nk + U, &nb)) { *err = "key arrays"; return rc; }
    host_trace("add_keys: keys_spare");
    const uint64_t* kpos = w->kpos.as<uint64_t>();
    UALLOC(w->kmap, 4 * std::max<uint64_t>(nk, 1), false);
    if (nk) k_key_move<<<blocks(nk), 256, 0, st>>>(s, grow.kcell, kpos, U, nb, w->kmap.as<uint32_t>());
    k_key_new<<<blocks(U), 256, 0, st>>>(s, w->knew.as<int64_t>(), kpos, U, nb);
    if (ne) k_ekey_remap<<<blocks(ne), 256, 0, st>>>(ne, d.ekey, w->kmap.as<uint32_t>());
    k_khash_clear<<<blocks(nb.hcap), 256, 0, st>>>(nb.khash, nb.hcap);
    k_khash_fill<<<blocks(nk + U), 256, 0, st>>>(nk + U, nb);
    UCHK(hipGetLastError());
    if (int rc = grow.keys_swap(grow.ctx, &nb)) { *err = "key arrays"; return rc; }
    UCHK(hipStreamSynchronize(st));
    host_trace("add_keys: move+swap sync");
    if (grow.keys_added) grow.keys_added(grow.ctx, w->knew.as<int64_t>(), U, nk + U, st);
    s.n_keys = nk + U;
    s.keys = nb.keys;
    s.krec = nb.krec;
    s.khash = nb.khash;
    s.khash_mask = nb.hcap - 1;
    s.kent = nb.kent;
    d.krec = nb.krec;
    d.kent = nb.kent;
    out->n_new_keys = U;
    out->new_keys = w->knew.as<int64_t>();
    out->key_pos = kpos;
    return AD_OK;
}

// Merge the sorted unique new ids (nflag/npos over the sorted order vs) into the dictionary: new
// arrays (spare buffers), then every stored rank remapped in place.
static int merge_dictionary(CfkUpdWork* w, DevSnapshot& s, CfkDevState& d, const DictSample& ds, const CfkGrow& grow,
                            const uint32_t* vs, uint64_t m, uint64_t cap, uint64_t U, hipStream_t st, CfkUpdOut* out,
                            std::string* err)
{
    const uint64_t n0 = s.n_dict, ne = s.n_ent, nk = s.n_keys;
    UALLOC(w->mh, 8 * U, false);
    UALLOC(w->ml, 8 * U, false);
    UALLOC(w->mn, 4 * U, false);
    UALLOC(w->mraw, 8 * U, false);
    UALLOC(w->mpos, 8 * U, false);
    uint64_t* mpos = w->mpos.as<uint64_t>();
    k_ins_append<<<blocks(m), 256, 0, st>>>(vs, m, w->nw.as<uint64_t>(), cap, w->nflag.as<uint32_t>(), w->npos.as<uint64_t>(), 0,
                                            w->mh.as<uint64_t>(), w->ml.as<uint64_t>(), w->mn.as<int32_t>(), w->mraw.as<uint64_t>());
    k_merge_pos<<<blocks(U), 256, 0, st>>>(s, ds, U, w->mh.as<uint64_t>(), w->ml.as<uint64_t>(), w->mn.as<int32_t>(), mpos);
    DictArrays nd{};
    if (int rc = grow.dict_spare(grow.ctx, n0 + U, &nd.hi, &nd.lo, &nd.node, &nd.raw)) { *err = "dictionary merge"; return rc; }
    if (n0) k_merge_old<<<blocks(n0), 256, 0, st>>>(s, d.dict_lsb_raw, mpos, U, nd);
    k_merge_new<<<blocks(U), 256, 0, st>>>(U, w->mh.as<uint64_t>(), w->ml.as<uint64_t>(), w->mn.as<int32_t>(),
                                           w->mraw.as<uint64_t>(), mpos, nd);
    if (ne) k_remap_entries<<<blocks(ne), 256, 0, st>>>(ne, d.ent, d.xrank, mpos, U);
    if (nk) k_remap_krec<<<blocks(nk), 256, 0, st>>>(nk, d.krec, mpos, U);
    if (grow.n_rtxw) k_remap_txw<<<blocks(grow.n_rtxw), 256, 0, st>>>(grow.n_rtxw, grow.r_txw, mpos, U);
    if (grow.n_cell_ent) k_remap_cells<<<blocks(grow.n_cell_ent), 256, 0, st>>>(grow.n_cell_ent, grow.cell_ent, mpos, U);
    if (grow.n_rb) k_remap_txw<<<blocks(grow.n_rb), 256, 0, st>>>(grow.n_rb, grow.rb_wm, mpos, U);
    if (grow.n_mids) k_remap_txw<<<blocks(grow.n_mids), 256, 0, st>>>(grow.n_mids, grow.m_ids, mpos, U);
    UCHK(hipGetLastError());
    if (int rc = grow.dict_swap(grow.ctx, &nd.hi, &nd.lo, &nd.node, &nd.raw)) { *err = "dictionary merge"; return rc; }
    uint64_t lh = 0, ll = 0;
    int32_t ln = 0;
    UCHK(d2h(&lh, nd.hi + n0 + U - 1, 8, st));
    UCHK(d2h(&ll, nd.lo + n0 + U - 1, 8, st));
    UCHK(d2h(&ln, nd.node + n0 + U - 1, 4, st));
    UCHK(hipStreamSynchronize(st));
    s.dict_hi = nd.hi;
    s.dict_lo = nd.lo;
    s.dict_node = nd.node;
    s.n_dict = n0 + U;
    s.dict_last_hi = lh;
    s.dict_last_lo = ll;
    s.dict_last_node = ln;
    d.dict_lsb_raw = nd.raw;
    out->n_new_ids = U;
    out->merged = true;
    out->merge_pos = mpos;
    return AD_OK;
}

// Add the batch's ids the dictionary does not hold (sorted, unique): appended when all are newer
// than its newest id, merged otherwise.
static int grow_dictionary(CfkUpdWork* w, DevSnapshot& s, CfkDevState& d, const DictSample& ds, const CfkUpdIn& u,
                           const CfkGrow& grow, hipStream_t st, CfkUpdOut* out, std::string* err, uint64_t ndep = 0)
{
    const uint64_t n = u.n, cap = 2 * n + ndep;
    UpdCtl* ctl = w->ctl.as<UpdCtl>();
    UALLOC(w->nw, 8 * 4 * cap, false);
    UALLOC(w->rk, 8 * n, false);
    k_ins_collect<<<blocks(n), 256, 0, st>>>(s, ds, u, w->nw.as<uint64_t>(), cap, w->rk.as<uint32_t>(), ctl);
    if (ndep) k_dep_collect<<<blocks(ndep), 256, 0, st>>>(s, ds, u, ndep, w->nw.as<uint64_t>(), cap, ctl);
    UCHK(hipGetLastError());
    UCHK(d2h(w->h_ctl, ctl, sizeof(UpdCtl), st));
    UCHK(hipStreamSynchronize(st));
    const uint64_t m = w->h_ctl->n_new;
    if (m == 0) return AD_OK;
    const uint64_t* nw = w->nw.as<uint64_t>();
    UALLOC(w->nk_a, 8 * m, false);
    UALLOC(w->nk_b, 8 * m, false);
    UALLOC(w->nv_a, 4 * m, false);
    UALLOC(w->nv_b, 4 * m, false);
    const uint64_t hist_n = radix_hist_entries(m);
    UALLOC(w->hist, 4 * hist_n, false);
    UALLOC(w->hoff, 8 * (hist_n + 1), false);
    UALLOC(w->bsum, 8 * ((std::max(hist_n, m) + 1023) / 1024 + 8), false);
    UALLOC(w->nflag, 4 * m, false);
    UALLOC(w->npos, 8 * (m + 1), false);
    // LSD over the three words of the normalised id: node, lo, hi (Timestamp.compareTo order)
    k_iota<<<blocks(m), 256, 0, st>>>(w->nv_a.as<uint32_t>(), m);
    UCHK(hipMemcpyAsync(w->nk_a.p, nw, 8 * m, hipMemcpyDeviceToDevice, st));
    uint64_t* ks = w->nk_a.as<uint64_t>();
    uint32_t* vs = w->nv_a.as<uint32_t>();
    for (int word = 0; word < 3; ++word)
    {
        if (word > 0)
        {
            uint64_t* dst = ks == w->nk_a.as<uint64_t>() ? w->nk_b.as<uint64_t>() : w->nk_a.as<uint64_t>();
            k_gather64<<<blocks(m), 256, 0, st>>>(nw + word * cap, vs, m, dst);
            ks = dst;
        }
        uint64_t* kt = ks == w->nk_a.as<uint64_t>() ? w->nk_b.as<uint64_t>() : w->nk_a.as<uint64_t>();
        uint32_t* vt = vs == w->nv_a.as<uint32_t>() ? w->nv_b.as<uint32_t>() : w->nv_a.as<uint32_t>();
        const uint32_t mask = digits_that_vary(w->h_ctl->diff[word]);
        if (!mask) continue;                      // constant word: the order stands
        UCHK(radix_sort_pairs(ks, vs, kt, vt, m, mask, w->hist.as<uint32_t>(), w->hoff.as<uint64_t>(),
                              w->bsum.as<uint64_t>(), st, &ks, &vs));
    }
    k_ins_unique<<<blocks(m), 256, 0, st>>>(vs, m, nw, cap, w->nflag.as<uint32_t>(), ctl);
    UCHK(run_scan_arrays(w->nflag.as<uint32_t>(), w->npos.as<uint64_t>(), m, 1, w->bsum.as<uint64_t>(), st));
    k_drv_totals<<<1, 64, 0, st>>>(w->npos.as<uint64_t>(), m, 1, ctl->tot2);
    UCHK(d2h(w->h_ctl, ctl, sizeof(UpdCtl), st));
    UCHK(hipStreamSynchronize(st));
    if (w->h_ctl->err) return AD_OK;          // reported by the caller
    const uint64_t U = w->h_ctl->tot2[0], n0 = s.n_dict;
    if (n0 + U > MAX_DICT) { *err = "id dictionary exceeds 2^28 entries"; return AD_E_CAPACITY; }
    if (w->h_ctl->older) return merge_dictionary(w, s, d, ds, grow, vs, m, cap, U, st, out, err);
    uint64_t *dh, *dl, *draw;
    int32_t* dn;
    if (int rc = grow.dict(grow.ctx, n0, n0 + U, &dh, &dl, &dn, &draw)) { *err = "dictionary growth"; return rc; }
    k_ins_append<<<blocks(m), 256, 0, st>>>(vs, m, nw, cap, w->nflag.as<uint32_t>(), w->npos.as<uint64_t>(), n0, dh, dl, dn,
                                            draw);
    UCHK(hipGetLastError());
    uint64_t lh = 0, ll = 0;
    int32_t ln = 0;
    UCHK(d2h(&lh, dh + n0 + U - 1, 8, st));
    UCHK(d2h(&ll, dl + n0 + U - 1, 8, st));
    UCHK(d2h(&ln, dn + n0 + U - 1, 4, st));
    UCHK(hipStreamSynchronize(st));
    s.dict_hi = dh;
    s.dict_lo = dl;
    s.dict_node = dn;
    s.n_dict = n0 + U;
    s.dict_last_hi = lh;
    s.dict_last_lo = ll;
    s.dict_last_node = ln;
    d.dict_lsb_raw = draw;
    out->n_new_ids = U;
    return AD_OK;
}

// Insert one entry per (key, txnId) group of the insertion updates at its byId position; the
// per-entry arrays move to the spare buffers (the current ones stay intact for a rollback).
struct InsUndo {
    bool krec_saved = false;    // krec was saved to krec_bk and then changed
    bool swapped = false;       // the per-entry arrays were swapped to the spare buffers
};

static int insert_entries(CfkUpdWork* w, DevSnapshot& s, CfkDevState& d, const CfkUpdIn& u, const CfkGrow& grow,
                          hipStream_t st, uint64_t q, uint64_t* G_out, InsUndo* undo, std::string* err, bool fold,
                          uint8_t* uapp)
{
    const uint64_t ne = s.n_ent, nk = s.n_keys;
    UpdCtl* ctl = w->ctl.as<UpdCtl>();
    UALLOC(w->ck, 8 * q, false);
    UALLOC(w->cv, 4 * q, false);
    UALLOC(w->ck2, 8 * q, false);
    UALLOC(w->cv2, 4 * q, false);
    const uint64_t hist_n = radix_hist_entries(q);
    UALLOC(w->hist, 4 * hist_n, false);
    UALLOC(w->hoff, 8 * (hist_n + 1), false);
    UALLOC(w->bsum, 8 * ((std::max(hist_n, q) + 1023) / 1024 + 8), false);
    UALLOC(w->gflag, 4 * q, false);
    UALLOC(w->gs, 8 * (q + 1), false);
    // ck / cv hold the insertion updates in batch order (k_compact)
    uint64_t* ks = w->ck.as<uint64_t>();
    uint32_t* vs = w->cv.as<uint32_t>();
    if (q > 1)
    {
        // stable: equal (key, txnId) groups keep batch order
        UCHK(radix_sort_pairs(ks, vs, w->ck2.as<uint64_t>(), w->cv2.as<uint32_t>(), q, key_rank_mask(s.n_dict, nk),
                              w->hist.as<uint32_t>(), w->hoff.as<uint64_t>(), w->bsum.as<uint64_t>(), st, &ks, &vs));
    }
    k_ins_gflags<<<blocks(q), 256, 0, st>>>(ks, q, w->gflag.as<uint32_t>());
    UCHK(run_scan_arrays(w->gflag.as<uint32_t>(), w->gs.as<uint64_t>(), q, 1, w->bsum.as<uint64_t>(), st));
    k_drv_totals<<<1, 64, 0, st>>>(w->gs.as<uint64_t>(), q, 1, ctl->tot2 + 1);
    UCHK(d2h(w->h_ctl, ctl, sizeof(UpdCtl), st));
    UCHK(hipStreamSynchronize(st));
    const uint64_t G = w->h_ctl->tot2[1];
    if (ne + G >= (1ull << 32)) { *err = "more than 2^32 CommandsForKey entries"; return AD_E_CAPACITY; }
    UALLOC(w->gword, 8 * G, false);
    UALLOC(w->gkey, 4 * G, false);
    UALLOC(w->grank, 4 * G, false);
    UALLOC(w->ib, 4 * (nk + 1), false);
    UALLOC(w->krec_bk, sizeof(KeyRec) * std::max<uint64_t>(nk, 1), false);
    UCHK(hipMemsetAsync(w->gword.p, 0, 8 * G, st));
    if (fold)
        k_ins_fold<<<blocks(q), 256, 0, st>>>(ks, vs, q, w->gflag.as<uint32_t>(), w->gs.as<uint64_t>(), u,
                                              w->gword.as<unsigned long long>(), w->gkey.as<uint32_t>(), w->grank.as<uint32_t>(), ctl,
                                              uapp);
    else
        k_ins_claim<<<blocks(q), 256, 0, st>>>(ks, vs, q, w->gflag.as<uint32_t>(), w->gs.as<uint64_t>(), u.status,
                                               w->gword.as<unsigned long long>(), w->gkey.as<uint32_t>(), w->grank.as<uint32_t>());
    k_ins_before<<<blocks(nk + 1), 256, 0, st>>>(nk, w->gkey.as<uint32_t>(), G, w->ib.as<uint32_t>());
    UCHK(hipGetLastError());
    UALLOC(w->chg[w->chg_cur ^ 1], ne + G, false);
    UALLOC(w->mv, 4 * std::max<uint64_t>(ne, 1), false);
    EntArrays a{d.ent, d.status, d.xrank, d.ekey, d.ballot, w->chg[w->chg_cur].as<uint8_t>(), d.mref}, b{};
    b.chg = w->chg[w->chg_cur ^ 1].as<uint8_t>();
    if (int rc = grow.entries(grow.ctx, ne + G, &b.ent, &b.status, &b.xrank, &b.ekey, &b.bal, &b.mref)) { *err = "entry growth"; return rc; }
    const uint64_t padded = std::max<uint64_t>(64, (ne + G + 63) / 64 * 64);
    if (padded > ne + G) UCHK(hipMemsetAsync(b.ent + ne + G, 0, sizeof(uint2) * (padded - ne - G), st));
    if (ne) k_ins_move_old<<<blocks(ne), 256, 0, st>>>(ne, a, w->ib.as<uint32_t>(), w->grank.as<uint32_t>(), b, w->mv.as<uint32_t>());
    k_ins_place<<<blocks(G), 256, 0, st>>>(G, w->gkey.as<uint32_t>(), w->grank.as<uint32_t>(), w->gword.as<unsigned long long>(),
                                           d.krec, a.ent, u, w->xr.as<uint32_t>(), b);
    if (nk)
    {
        UCHK(hipMemcpyAsync(w->krec_bk.p, d.krec, sizeof(KeyRec) * nk, hipMemcpyDeviceToDevice, st));
        undo->krec_saved = true;
        k_ins_krec<<<blocks(nk), 256, 0, st>>>(nk, w->ib.as<uint32_t>(), w->grank.as<uint32_t>(), d.krec);
    }
    UCHK(hipGetLastError());
    const int src = grow.swap(grow.ctx, ne + G, &d.ent, &d.status, &d.xrank, &d.ekey, &d.ballot, &d.mref);
    undo->swapped = true;         // the buffers are exchanged even when sizing the trees then failed
    w->chg_cur ^= 1;              // the changed flags moved with the entries
    w->moved = true;
    if (src) { *err = "entry swap"; return src; }
    s.ent = d.ent;
    s.n_ent = ne + G;
    *G_out = G;
    return AD_OK;
}

static int miss_after_batch(CfkUpdWork* w, DevSnapshot& s, CfkDevState& d, const CfkUpdIn& u, uint64_t ndep,
                            CfkDerivedBufs* bufs, int (*need)(void*, uint64_t, uint64_t, uint64_t, CfkDerivedBufs*),
                            void* need_ctx, const CfkGrow& grow, hipStream_t st, CfkUpdOut* out, std::string* err,
                            CfkMiss* miss);

int run_cfk_update(CfkUpdWork* w, DevSnapshot& s, CfkDevState& d, const CfkUpdIn& u, CfkDerivedBufs* bufs,
                   int (*need)(void*, uint64_t, uint64_t, uint64_t, CfkDerivedBufs*), void* need_ctx, const CfkGrow& grow,
                   hipStream_t st, CfkUpdOut* out, std::string* err, CfkMiss* miss)
{
    const uint64_t n = u.n;
    *out = CfkUpdOut{};
    if (n == 0) return AD_OK;
    // missing() maintenance (with the deps of the batch): the updates fold in batch order, so each
    // update knows whether it applied and which one an entry's TxnInfo comes from
    const bool track = miss && miss->on && u.dep_off && d.mref;
    uint64_t ndep = 0;
    if (track)
    {
        dev_quiesce();
        if (d2h(&ndep, u.dep_off + n, 8, dev_scope_stream()) != hipSuccess) { *err = "dep_off"; return AD_E_DEVICE; }
        UALLOC(w->uapp, n, false);
        UCHK(hipMemsetAsync(w->uapp.p, 0, n, st));
    }
    if (n >= 0x7FFFFFFFull) { *err = "more than 2^31-2 updates in one batch"; return AD_E_INVAL; }
    if (!w->h_ctl && hipHostMalloc((void**)&w->h_ctl, sizeof(UpdCtl)) != hipSuccess) { *err = "pinned ctl"; return AD_E_NOMEM; }
    for (auto& e : w->ev)
        if (!e) UCHK(timing_event(&e));
    auto describe = [&](uint32_t code, uint32_t idx) -> int {
        char b[256];
        const char* what = "";
        int rc = AD_E_INVAL;
        switch (code)
        {
            case UE_KEY: what = "key missing from the key arrays after its creation (internal)"; rc = AD_E_STATE; break;
            case UE_STATUS: what = "status is not an InternalStatus ordinal"; break;
            case UE_ABSENT: what = "txnId missing from the id dictionary after its merge (internal)"; rc = AD_E_STATE; break;
            case UE_NEW_EXEC: what = "executeAt missing from the id dictionary after its merge (internal)"; rc = AD_E_STATE; break;
            case UE_FLAGS: what = "ids equal under Timestamp.equals differ in flag bits"; rc = AD_E_INCONSISTENT_ID; break;
            case UE_DOMAIN: what = "live range-domain TxnId in a CommandsForKey"; break;
            case UE_DUP_EXEC: what = "two committed entries of one key share an executeAt (CommandsForKey.java:1439)"; rc = AD_E_DUP_EXEC; break;
        }
        snprintf(b, sizeof(b), "cfk update %u: %s", idx, what);
        *err = b;
        return rc;
    };
    UALLOC(w->ctl, sizeof(UpdCtl), false);
    UALLOC(w->loc, 4 * n, false);
    UALLOC(w->xr, 4 * n, false);
    UALLOC(w->bk, 8 * n, false);
    UALLOC(w->ins_k, 8 * n, false);
    UALLOC(w->ins_v, 4 * n, false);
    UALLOC(w->word, 8 * std::max<uint64_t>(s.n_ent, 1), true);   // zero between batches (winners clear theirs)
    UpdCtl* ctl = w->ctl.as<UpdCtl>();
    UCHK(hipMemsetAsync(ctl, 0, sizeof(UpdCtl), st));
    UCHK(hipEventRecord(w->ev[0], st));
    // per-entry changed flags of this batch (incremental committed order) and no insertion map yet
    UALLOC(w->chg[w->chg_cur], std::max<uint64_t>(s.n_ent, 1), false);
    if (s.n_ent) UCHK(hipMemsetAsync(w->chg[w->chg_cur].p, 0, s.n_ent, st));
    w->moved = false;

    // ---- 0. ids the dictionary does not hold join it. Ids newer than all of it are appended (no
    // rank changes): a batch that then fails drops them again (the arrays keep the bytes; nothing
    // refers to them). Older ones are merged with a rank remap of every stored rank: the merge
    // stands when the batch then fails (it changes no content), and the derived arrays are rebuilt.
    const uint64_t nd0 = s.n_dict, lh0 = s.dict_last_hi, ll0 = s.dict_last_lo;
    const int32_t ln0 = s.dict_last_node;
    auto drop_new_ids = [&](int code) -> int {
        if (out->merged) return code;
        s.n_dict = nd0;
        s.dict_last_hi = lh0;
        s.dict_last_lo = ll0;
        s.dict_last_node = ln0;
        out->n_new_ids = 0;
        return code;
    };
    UALLOC(w->sm_hi, 8 * std::max<uint64_t>((s.n_dict + n + n + SAMP - 1) / SAMP, 1), false);
    UALLOC(w->sm_lo, 8 * std::max<uint64_t>((s.n_dict + n + n + SAMP - 1) / SAMP, 1), false);
    UALLOC(w->sm_node, 4 * std::max<uint64_t>((s.n_dict + n + n + SAMP - 1) / SAMP, 1), false);
    auto sample = [&]() -> DictSample {
        const uint64_t n_samp = (s.n_dict + SAMP - 1) / SAMP;
        if (n_samp)
            k_dict_sample<<<blocks(n_samp), 256, 0, st>>>(s, w->sm_hi.as<uint64_t>(), w->sm_lo.as<uint64_t>(),
                                                          w->sm_node.as<int32_t>(), n_samp);
        return DictSample{w->sm_hi.as<uint64_t>(), w->sm_lo.as<uint64_t>(), w->sm_node.as<int32_t>(), n_samp};
    };
    // a failure after a merge or new keys: the entries are as they were, under the new ranks /
    // key indices; derive again
    auto rederive = [&](int code) -> int {
        if (!out->merged && !out->n_new_keys) return code;
        std::string e2;
        if (hipMemsetAsync(ctl, 0, sizeof(UpdCtl), st) != hipSuccess) { *err += "; re-derivation failed"; return AD_E_DEVICE; }
        if (int rc2 = cfk_derive(w, s, d, bufs, need, need_ctx, st, &e2)) { *err += "; re-derivation: " + e2; return rc2; }
        if (hipStreamSynchronize(st) != hipSuccess) { *err += "; re-derivation failed"; return AD_E_DEVICE; }
        out->rederived = true;
        return code;
    };
    if (int rc = add_keys(w, s, d, u, grow, st, out, err)) return rc == AD_E_CAPACITY ? rc : rederive(rc);
    host_trace("upd: add_keys");
    if (out->n_new_keys) UCHK(hipMemsetAsync(ctl, 0, sizeof(UpdCtl), st));
    {
        const DictSample ds0 = sample();
        if (int rc = grow_dictionary(w, s, d, ds0, u, grow, st, out, err, ndep))
            return rc == AD_E_CAPACITY ? drop_new_ids(rc) : rederive(rc);
    }
    if (w->h_ctl->err) return rederive(drop_new_ids(describe(w->h_ctl->err, w->h_ctl->err_idx)));

    // ---- 1. locate and validate; nothing changes unless the whole batch is valid
    const DictSample dsm = sample();
    const bool bm = u.bal_msb != nullptr;
    const bool fold = bm || track;
    const int nf = fold ? 2 : 1;
    if (track) UALLOC(w->trk, 4ull * 3 * n, false);
    UALLOC(w->uflag, 4ull * 2 * n, false);
    UALLOC(w->upos, 8ull * 2 * (n + 1), false);
    UALLOC(w->bsum, 8ull * 2 * ((n + 1023) / 1024 + 8), false);
    k_upd_locate<<<blocks(n), 256, 0, st>>>(s, dsm, d, u, w->loc.as<uint32_t>(), w->xr.as<uint32_t>(),
                                            w->word.as<unsigned long long>(), w->ins_k.as<uint64_t>(),
                                            w->uflag.as<uint32_t>(), w->rk.as<uint32_t>(), out->merge_pos,
                                            out->merged ? out->n_new_ids : 0, ctl, fold ? 1 : 0,
                                            track ? w->trk.as<uint32_t>() : nullptr);
    UCHK(hipGetLastError());
    UCHK(run_scan_arrays(w->uflag.as<uint32_t>(), w->upos.as<uint64_t>(), n, nf, w->bsum.as<uint64_t>(), st));
    k_drv_totals<<<1, 64, 0, st>>>(w->upos.as<uint64_t>(), n, nf, ctl->tot3);
    UCHK(d2h(w->h_ctl, ctl, sizeof(UpdCtl), st));
    UCHK(hipStreamSynchronize(st));
    if (w->h_ctl->err)
    {
        k_upd_release<<<blocks(n), 256, 0, st>>>(n, w->loc.as<uint32_t>(), w->word.as<unsigned long long>());
        UCHK(hipStreamSynchronize(st));
        return rederive(drop_new_ids(describe(w->h_ctl->err, w->h_ctl->err_idx)));
    }
    const uint64_t q = w->h_ctl->tot3[0], mp = fold ? w->h_ctl->tot3[1] : 0, ne0 = s.n_ent;
    // the batch's first ballots: the store's entries all hold Ballot.ZERO until now
    if (bm && !d.ballot && ne0)
        if (int rc = grow.ballot_init(grow.ctx, ne0, &d.ballot)) { *err = "ballot array"; return rederive(drop_new_ids(rc)); }
    const uint64_t cq = std::max<uint64_t>(std::max(q, mp), 1);
    UALLOC(w->ck, 8 * cq, false);
    UALLOC(w->cv, 4 * cq, false);
    UALLOC(w->ck2, 8 * cq, false);
    UALLOC(w->cv2, 4 * cq, false);
    UALLOC(w->bkb, sizeof(Bal) * n, false);
    UCHK(hipMemsetAsync(w->bk.p, 0xFF, 8 * n, st));          // bk[i].x = none: nothing to roll back
    if (fold)
    {
        if (mp)
        {
            // the present entries' updates, sorted by entry (stable: batch order within), folded
            uint64_t* ks = w->ck.as<uint64_t>();
            uint32_t* vs = w->cv.as<uint32_t>();
            k_compact<<<blocks(n), 256, 0, st>>>(n, w->uflag.as<uint32_t>() + n, w->upos.as<uint64_t>() + (n + 1), nullptr,
                                                 w->loc.as<uint32_t>(), ks, vs);
            if (mp > 1)
            {
                const uint64_t hist_n = radix_hist_entries(mp);
                UALLOC(w->hist, 4 * hist_n, false);
                UALLOC(w->hoff, 8 * (hist_n + 1), false);
                UALLOC(w->bsum, 8 * ((std::max(hist_n, mp) + 1023) / 1024 + 8), false);
                uint32_t mask = 0;
                for (uint32_t b = 0; b < bytes_of(ne0 ? ne0 - 1 : 0) && b < 4; ++b) mask |= 1u << b;
                if (mask)
                    UCHK(radix_sort_pairs(ks, vs, w->ck2.as<uint64_t>(), w->cv2.as<uint32_t>(), mp, mask, w->hist.as<uint32_t>(),
                                          w->hoff.as<uint64_t>(), w->bsum.as<uint64_t>(), st, &ks, &vs));
            }
            k_fold_present<<<blocks(mp), 256, 0, st>>>(mp, ks, vs, u, w->xr.as<uint32_t>(), d, w->bk.as<uint2>(),
                                                       w->bkb.as<Bal>(), w->chg[w->chg_cur].as<uint8_t>(), ctl,
                                                       track ? w->uapp.as<uint8_t>() : nullptr);
        }
    }
    else
        k_upd_apply<<<blocks(n), 256, 0, st>>>(n, w->loc.as<uint32_t>(), w->xr.as<uint32_t>(), w->word.as<unsigned long long>(),
                                               d, w->bk.as<uint2>(), w->bkb.as<Bal>(), w->chg[w->chg_cur].as<uint8_t>(), ctl);
    UCHK(hipGetLastError());
    if (q)   // the insertion updates in batch order, for insert_entries
        k_compact<<<blocks(n), 256, 0, st>>>(n, w->uflag.as<uint32_t>(), w->upos.as<uint64_t>(), w->ins_k.as<uint64_t>(),
                                             nullptr, w->ck.as<uint64_t>(), w->cv.as<uint32_t>());
    // From here on the per-entry state has changed: every failure undoes the batch (status and
    // executeAt restored, insertions swapped back, krec restored) and derives the previous state
    // again, so that nothing changes unless the whole batch is applied.
    InsUndo undo;
    auto rollback = [&](int code) -> int {
        std::string e2;
        if (undo.swapped)
        {
            if (grow.swap(grow.ctx, ne0, &d.ent, &d.status, &d.xrank, &d.ekey, &d.ballot, &d.mref)) { *err += "; rollback failed"; return AD_E_DEVICE; }
            s.ent = d.ent;
            s.n_ent = ne0;
        }
        if (undo.krec_saved && s.n_keys)
            if (hipMemcpyAsync(d.krec, w->krec_bk.p, sizeof(KeyRec) * s.n_keys, hipMemcpyDeviceToDevice, st) != hipSuccess)
            { *err += "; rollback failed"; return AD_E_DEVICE; }
        k_upd_rollback<<<blocks(n), 256, 0, st>>>(n, w->loc.as<uint32_t>(), w->bk.as<uint2>(), w->bkb.as<Bal>(), d);
        if (hipGetLastError() != hipSuccess || hipMemsetAsync(ctl, 0, sizeof(UpdCtl), st) != hipSuccess)
        { *err += "; rollback failed"; return AD_E_DEVICE; }
        if (int rc2 = cfk_derive(w, s, d, bufs, need, need_ctx, st, &e2)) { *err += "; rollback: " + e2; return rc2; }
        if (hipStreamSynchronize(st) != hipSuccess) { *err += "; rollback failed"; return AD_E_DEVICE; }
        out->n_applied = out->n_inserted = 0;
        out->rolled_back = true;
        return drop_new_ids(code);
    };
    uint64_t G = 0;
    if (q)
        if (int rc = insert_entries(w, s, d, u, grow, st, q, &G, &undo, err, fold, track ? w->uapp.as<uint8_t>() : nullptr))
            return rollback(rc);
    UCHK(hipEventRecord(w->ev[1], st));

    // ---- 2. re-derive the snapshot arrays from the per-entry state (committed order incrementally)
    if (int rc = cfk_derive(w, s, d, bufs, need, need_ctx, st, err, true)) return rollback(rc);
    UCHK(hipEventRecord(w->ev[2], st));
    UCHK(d2h(w->h_ctl, ctl, sizeof(UpdCtl), st));
    UCHK(hipStreamSynchronize(st));
    host_trace("upd: derive sync");
    float a = 0, b = 0;
    (void)hipEventElapsedTime(&a, w->ev[0], w->ev[1]);
    (void)hipEventElapsedTime(&b, w->ev[1], w->ev[2]);
    out->ms_locate = a;
    out->ms_derive = b;
    out->ms_total = a + b;
    out->n_applied = w->h_ctl->applied + G;
    out->n_inserted = G;
    // a duplicate committed executeAt: undo the batch and derive the previous state again
    if (w->h_ctl->err) return rollback(describe(w->h_ctl->err, w->h_ctl->err_idx));
    out->batch_stood = true;
    if (track) return miss_after_batch(w, s, d, u, ndep, bufs, need, need_ctx, grow, st, out, err, miss);
    return AD_OK;
}

// After a batch with deps (missing() maintenance on): the additions as a second batch of
// TRANSITIVELY_KNOWN insertions (their ids already joined the dictionary with the batch), then every
// entry's missing() rebuilt (k_miss_build). The explicit batch stands when this part fails.
static int miss_after_batch(CfkUpdWork* w, DevSnapshot& s, CfkDevState& d, const CfkUpdIn& u, uint64_t ndep,
                            CfkDerivedBufs* bufs, int (*need)(void*, uint64_t, uint64_t, uint64_t, CfkDerivedBufs*),
                            void* need_ctx, const CfkGrow& grow, hipStream_t st, CfkUpdOut* out, std::string* err,
                            CfkMiss* miss)
{
    const uint64_t n = u.n;
    UpdCtl* ctl = w->ctl.as<UpdCtl>();
    const uint8_t* uapp = w->uapp.as<uint8_t>();
    auto dsample = [&]() -> DictSample {
        const uint64_t n_samp = (s.n_dict + SAMP - 1) / SAMP;
        UALLOC_V(w->sm_hi, 8 * std::max<uint64_t>(n_samp, 1));
        UALLOC_V(w->sm_lo, 8 * std::max<uint64_t>(n_samp, 1));
        UALLOC_V(w->sm_node, 4 * std::max<uint64_t>(n_samp, 1));
        if (n_samp)
            k_dict_sample<<<blocks(n_samp), 256, 0, st>>>(s, w->sm_hi.as<uint64_t>(), w->sm_lo.as<uint64_t>(),
                                                          w->sm_node.as<int32_t>(), n_samp);
        return DictSample{w->sm_hi.as<uint64_t>(), w->sm_lo.as<uint64_t>(), w->sm_node.as<int32_t>(), n_samp};
    };
    // ---- additions (computeInfoAndAdditions :210-263, insertOrUpdateWithAdditions)
    UALLOC(w->drank, 4 * std::max<uint64_t>(ndep, 1), false);
    UALLOC(w->acnt, 4 * n, false);
    UALLOC(w->aoff, 8 * (n + 1), false);
    UALLOC(w->bsum, 8 * ((n + 1023) / 1024 + 8), false);
    {
        const DictSample ds = dsample();
        if (ndep) k_dep_rank<<<blocks(ndep), 256, 0, st>>>(s, ds, u, ndep, w->drank.as<uint32_t>());
    }
    // byId's last txnId per update as the sequential Java sees it (k_past_*)
    UALLOC(w->pk, 8 * n, false);
    UALLOC(w->pv, 4 * n, false);
    UALLOC(w->pk2, 8 * n, false);
    UALLOC(w->pv2, 4 * n, false);
    UALLOC(w->pvv, 4 * n, false);
    UALLOC(w->pw, 8 * n, false);
    UALLOC(w->pe, 8 * n, false);
    UALLOC(w->pbm, 8 * ((n + 1023) / 1024 + 1), false);
    UALLOC(w->plast, 4 * n, false);
    UALLOC(w->ppos, 4 * n, false);
    {
        const uint32_t* trk = w->trk.as<uint32_t>();
        k_past_keys<<<blocks(n), 256, 0, st>>>(u, uapp, trk, w->drank.as<uint32_t>(), w->pk.as<uint64_t>(), w->pv.as<uint32_t>(),
                                               w->pvv.as<uint32_t>());
        uint64_t* ks = w->pk.as<uint64_t>();
        uint32_t* vs = w->pv.as<uint32_t>();
        uint32_t mask = 0;
        for (uint32_t b = 0; b < bytes_of(n - 1) && b < 4; ++b) mask |= 1u << b;
        for (uint32_t b = 0; b < bytes_of(s.n_keys ? s.n_keys - 1 : 0) && b < 4; ++b) mask |= 1u << (4 + b);
        if (n > 1 && mask)
        {
            const uint64_t hist_n = radix_hist_entries(n);
            UALLOC(w->hist, 4 * hist_n, false);
            UALLOC(w->hoff, 8 * (hist_n + 1), false);
            UALLOC(w->bsum, 8 * ((std::max(hist_n, n) + 1023) / 1024 + 8), false);
            UCHK(radix_sort_pairs(ks, vs, w->pk2.as<uint64_t>(), w->pv2.as<uint32_t>(), n, mask, w->hist.as<uint32_t>(),
                                  w->hoff.as<uint64_t>(), w->bsum.as<uint64_t>(), st, &ks, &vs));
        }
        const uint64_t nb = (n + 1023) / 1024;
        k_past_words<<<blocks(n), 256, 0, st>>>(n, ks, vs, w->pvv.as<uint32_t>(), w->pw.as<uint64_t>());
        k_maxscan_blocks<<<(unsigned)nb, 256, 0, st>>>(w->pw.as<uint64_t>(), n, w->pbm.as<uint64_t>());
        k_maxscan_top<<<1, 256, 0, st>>>(w->pbm.as<uint64_t>(), nb);
        k_maxscan_apply<<<(unsigned)nb, 256, 0, st>>>(w->pw.as<uint64_t>(), n, w->pbm.as<uint64_t>(), w->pe.as<uint64_t>());
        k_past_last<<<blocks(n), 256, 0, st>>>(n, ks, vs, w->pe.as<uint64_t>(), trk, w->plast.as<uint32_t>(),
                                               w->ppos.as<uint32_t>());
        k_dep_check<<<blocks(n), 256, 0, st>>>(s, u, uapp, w->drank.as<uint32_t>(), w->plast.as<uint32_t>(), ks, vs,
                                               w->ppos.as<uint32_t>(), ctl);
        UCHK(hipGetLastError());
        UALLOC(w->bsum, 8 * ((n + 1023) / 1024 + 8), false);
    }
    UALLOC(w->lcnt, 4 * n, false);
    UALLOC(w->loff, 8 * (n + 1), false);
    AddOut ao{};
    ao.cnt = w->acnt.as<uint32_t>();
    ao.pcnt = w->lcnt.as<uint32_t>();
    k_add_deps<0><<<blocks(n), 256, 0, st>>>(s, u, uapp, w->drank.as<uint32_t>(), w->plast.as<uint32_t>(), ao);
    UCHK(run_scan_arrays(w->acnt.as<uint32_t>(), w->aoff.as<uint64_t>(), n, 1, w->bsum.as<uint64_t>(), st));
    UCHK(run_scan_arrays(w->lcnt.as<uint32_t>(), w->loff.as<uint64_t>(), n, 1, w->bsum.as<uint64_t>(), st));
    uint64_t na = 0, nl = 0;
    UCHK(d2h(&na, w->aoff.as<uint64_t>() + n, 8, st));
    UCHK(d2h(&nl, w->loff.as<uint64_t>() + n, 8, st));
    UCHK(d2h(w->h_ctl, ctl, sizeof(UpdCtl), st));
    UCHK(hipStreamSynchronize(st));
    if (w->h_ctl->err == UE_UNWITNESSED)
    {
        // the explicit batch stands (the Java would have applied the updates before the throwing one);
        // no additions, missing() lists marked for a reload
        char b[200];
        snprintf(b, sizeof(b), "cfk update %u: a dep its kind does not witness, absent from byId, is not an "
                               "ExclusiveSyncPoint (Updating.java:239-249)", w->h_ctl->err_idx);
        *err = b;
        out->failed_update = w->h_ctl->err_idx;
        UCHK(hipMemsetAsync(ctl, 0, sizeof(UpdCtl), st));
        return AD_E_INVAL;
    }
    if (na || nl)
    {
        UALLOC(w->a_k, 8 * std::max<uint64_t>(na, 1), false);
        UALLOC(w->a_tm, 8 * std::max<uint64_t>(na, 1), false);
        UALLOC(w->a_tl, 8 * std::max<uint64_t>(na, 1), false);
        UALLOC(w->a_tn, 4 * std::max<uint64_t>(na, 1), false);
        UALLOC(w->l_k, 8 * std::max<uint64_t>(nl, 1), false);
        UALLOC(w->l_tm, 8 * std::max<uint64_t>(nl, 1), false);
        UALLOC(w->l_tl, 8 * std::max<uint64_t>(nl, 1), false);
        UALLOC(w->l_tn, 4 * std::max<uint64_t>(nl, 1), false);
        UALLOC(w->l_i, 8 * std::max<uint64_t>(nl, 1), false);
        AddOut wo{nullptr, w->aoff.as<uint64_t>(), w->a_k.as<int64_t>(), w->a_tm.as<uint64_t>(), w->a_tl.as<uint64_t>(),
                  w->a_tn.as<int32_t>(), nullptr, w->loff.as<uint64_t>(), w->l_k.as<int64_t>(), w->l_tm.as<uint64_t>(),
                  w->l_tl.as<uint64_t>(), w->l_tn.as<int32_t>(), w->l_i.as<uint64_t>()};
        k_add_deps<1><<<blocks(n), 256, 0, st>>>(s, u, uapp, w->drank.as<uint32_t>(), w->plast.as<uint32_t>(), wo);
        UCHK(hipGetLastError());
    }
    out->n_load_pruned = nl;
    out->lp_keys = w->l_k.as<int64_t>();
    out->lp_msb = w->l_tm.as<uint64_t>();
    out->lp_lsb = w->l_tl.as<uint64_t>();
    out->lp_node = w->l_tn.as<int32_t>();
    out->lp_update = w->l_i.as<uint64_t>();
    if (na)
    {
        UALLOC(w->a_st, na, false);
        UCHK(hipMemsetAsync(w->a_st.p, AD_ST_TRANSITIVELY_KNOWN, na, st));
        UCHK(hipGetLastError());
        CfkUpdIn ua{na, w->a_k.as<int64_t>(), w->a_tm.as<uint64_t>(), w->a_tl.as<uint64_t>(), w->a_tn.as<int32_t>(),
                    w->a_tm.as<uint64_t>(), w->a_tl.as<uint64_t>(), w->a_tn.as<int32_t>(), w->a_st.as<uint8_t>(),
                    nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
        CfkUpdOut o2;
        if (int rc = run_cfk_update(w, s, d, ua, bufs, need, need_ctx, grow, st, &o2, err, nullptr))
        {
            *err = "deps-derived additions: " + *err;
            return rc;
        }
        if (o2.merged || o2.n_new_ids || o2.n_new_keys)
        {
            *err = "deps-derived additions grew the dictionary (internal: merged " + std::to_string((int)o2.merged) + ", new ids " +
                   std::to_string(o2.n_new_ids) + ", new keys " + std::to_string(o2.n_new_keys) + ")";
            return AD_E_STATE;
        }
        out->n_additions = o2.n_inserted;
        out->n_applied += o2.n_inserted;
        out->n_inserted += o2.n_inserted;
        out->ms_derive += o2.ms_total;
        out->ms_total += o2.ms_total;
    }
    // ---- every entry's missing() (k_miss_build)
    const uint64_t ne = s.n_ent;
    if (!ne) return AD_OK;
    UALLOC(w->dsrc, 4 * ne, false);
    UALLOC(w->mflag, 4 * 2 * ne, false);
    UALLOC(w->mpp, 8 * 2 * (ne + 1), false);
    UALLOC(w->mpend, 4 * 2 * ne, false);
    UALLOC(w->mcnt, 4 * ne, false);
    UALLOC(w->moff, 8 * (ne + 1), false);
    UALLOC(w->bsum, 8 * 2 * ((ne + 1023) / 1024 + 8), false);
    UCHK(hipMemsetAsync(w->dsrc.p, 0xFF, 4 * ne, st));
    {
        const DictSample ds = dsample();
        k_miss_src<<<blocks(n), 256, 0, st>>>(s, ds, u, uapp, w->dsrc.as<uint32_t>());
    }
    k_miss_flags<<<blocks(ne), 256, 0, st>>>(ne, d, w->mflag.as<uint32_t>());
    UCHK(run_scan_arrays(w->mflag.as<uint32_t>(), w->mpp.as<uint64_t>(), ne, 2, w->bsum.as<uint64_t>(), st));
    k_miss_scatter<<<blocks(ne), 256, 0, st>>>(ne, w->mflag.as<uint32_t>(), w->mpp.as<uint64_t>(), w->mpend.as<uint32_t>());
    k_miss_build<0><<<blocks(ne), 256, 0, st>>>(s, d, u, w->dsrc.as<uint32_t>(), w->drank.as<uint32_t>(), w->mpp.as<uint64_t>(),
                                                w->mpend.as<uint32_t>(), miss->off, miss->ids, w->mcnt.as<uint32_t>(), nullptr,
                                                nullptr);
    UCHK(run_scan_arrays(w->mcnt.as<uint32_t>(), w->moff.as<uint64_t>(), ne, 1, w->bsum.as<uint64_t>(), st));
    uint64_t nm = 0;
    UCHK(d2h(&nm, w->moff.as<uint64_t>() + ne, 8, st));
    UCHK(hipStreamSynchronize(st));
    uint64_t* noff = nullptr;
    uint32_t* nids = nullptr;
    if (int rc = miss->spare(miss->ctx, ne, nm, &noff, &nids)) { *err = "missing() lists"; return rc; }
    UCHK(hipMemcpyAsync(noff, w->moff.p, 8 * (ne + 1), hipMemcpyDeviceToDevice, st));
    k_miss_build<1><<<blocks(ne), 256, 0, st>>>(s, d, u, w->dsrc.as<uint32_t>(), w->drank.as<uint32_t>(), w->mpp.as<uint64_t>(),
                                                w->mpend.as<uint32_t>(), miss->off, miss->ids, nullptr, noff, nids);
    k_mref_identity<<<blocks(ne), 256, 0, st>>>(ne, d.mref);
    UCHK(hipGetLastError());
    UCHK(hipStreamSynchronize(st));
    if (int rc = miss->swap(miss->ctx, &miss->off, &miss->ids)) { *err = "missing() lists"; return rc; }
    miss->n_lists = ne;
    (void)ctl;
    return AD_OK;
}


// =============================================================================================
// Pruning.maybePrune (Pruning.java:164-199) and pruneBefore (:205-331) for a list of keys, on the
// device state. The store's TxnInfo.missing() lists are NO_TXNIDS in this model (the caller checks
// none are loaded), so pruneBefore removes, below the new prunedBefore's byId position, every
// INVALID_OR_TRUNCATED entry and every APPLIED entry executing before it; nothing else moves.
// =============================================================================================
namespace {

// Timestamp.hlc() of dictionary rank r (Timestamp.java:129-131: highHlc(msb) | lowHlc(lsb); the
// normalised lo holds lowHlc << 4)
__device__ __forceinline__ int64_t rank_hlc(const DevSnapshot& s, uint32_t r)
{
    const uint64_t i = (r - 1) >> 1;
    return (int64_t)(((s.dict_hi[i] & 0x7FFFull) << 48) | (s.dict_lo[i] >> 4));
}

__global__ void k_prune_cflag(uint64_t ne, const uint8_t* status, uint32_t* f)
{
    const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= ne) return;
    f[e] = (status[e] >= AD_ST_COMMITTED && status[e] <= AD_ST_APPLIED) ? 1u : 0u;
}

// thread per listed key: the new prunedBefore (maybePrune :166-189) -> p_pos[k] = its byId position
// (0: no prune), p_xr / p_tr = its executeAt / txnId ranks. cm: the committed entries sorted by
// (key, executeAt) (committedByExecuteAt of every key, :651-672); cpos: committed entries before e.
__global__ void k_prune_key(uint64_t nl, const uint32_t* klist, DevSnapshot s, CfkDevState d, const uint32_t* cm,
                            const uint64_t* cpos, int32_t prune_interval, int64_t min_hlc_delta, uint32_t* p_pos,
                            uint32_t* p_xr, uint32_t* p_tr)
{
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nl) return;
    const uint32_t k = klist ? klist[t] : (uint32_t)t;
    const KeyRec kr = d.krec[k];
    if (kr.maw < 0) return;                                   // no APPLIED Write: maxAppliedWrite = -1
    const uint64_t c_lo = cpos[kr.seg_lo], c_hi = cpos[kr.seg_hi];
    // maxAppliedWriteByExecuteAt as an index into the key's committedByExecuteAt
    const uint32_t mx = s.w[kr.maw].x;
    uint64_t lo = c_lo, hi = c_hi;
    while (lo < hi)
    {
        const uint64_t mid = (lo + hi) >> 1;
        if (d.xrank[cm[mid]] < mx) lo = mid + 1;
        else hi = mid;
    }
    const int64_t maw = (int64_t)(lo - c_lo);
    if (maw < (int64_t)prune_interval) return;
    const int64_t max_prune_hlc = rank_hlc(s, mx) - min_hlc_delta;
    int64_t i = maw;
    uint32_t e = 0;
    while (--i >= 0)
    {
        e = cm[c_lo + (uint64_t)i];
        const uint32_t kind = d.ent[e].y >> RANK_BITS;
        if (kind == AD_KIND_WRITE && rank_hlc(s, d.xrank[e]) <= max_prune_hlc && d.status[e] == AD_ST_APPLIED) break;
    }
    if (i < 0) return;
    const uint32_t tr = d.ent[e].y & RANK_MASK;
    if (kr.pruned && tr <= kr.pruned) return;                 // newPrunedBefore <= prunedBefore (:184)
    const uint32_t pos = e - kr.seg_lo;                       // insertPos: it is in byId
    if (pos == 0) return;
    p_pos[k] = pos;
    p_xr[k] = d.xrank[e];
    p_tr[k] = tr;
}

// thread per entry: removed by pruneBefore (:222-254). With missing() lists on the device (d.mref)
// the APPLIED entries are k_prune_subset's to decide; INVALID ones always go.
__global__ void k_prune_mark(uint64_t ne, CfkDevState d, const uint32_t* p_pos, const uint32_t* p_xr, uint32_t* rm)
{
    const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= ne) return;
    const uint32_t k = d.ekey[e];
    const uint32_t pos = p_pos[k];
    bool r = false;
    if (pos && e - d.krec[k].seg_lo < pos)
    {
        const uint32_t st = d.status[e];
        r = st == AD_ST_INVALID_OR_TRUNCATED_OR_UNMANAGED_COMMITTED || (!d.mref && st == AD_ST_APPLIED && d.xrank[e] < p_xr[k]);
    }
    rm[e] = r ? 1u : 0u;
}

// thread per pruned key, with missing() lists (:222-251): walking byId below the new prunedBefore,
// an APPLIED entry executing before it goes when its missing() is empty or inside the merged set --
// the new prunedBefore's list united with the lists of the APPLIED entries kept before it that
// execute at their txnId (the set is not built: the kept entries' indices go to `sc`, each id is
// searched in their lists).
__device__ inline bool list_has(const uint64_t* off, const uint32_t* ids, uint32_t L, uint32_t r)
{
    if (L == MREF_NONE || L == MREF_BORN) return false;
    uint64_t lo = off[L], hi = off[L + 1];
    while (lo < hi)
    {
        const uint64_t m = (lo + hi) >> 1;
        if (ids[m] < r) lo = m + 1;
        else hi = m;
    }
    return lo < off[L + 1] && ids[lo] == r;
}

__global__ void k_prune_subset(uint64_t nl, const uint32_t* klist, CfkDevState d, const uint32_t* p_pos, const uint32_t* p_xr,
                               const uint64_t* moff, const uint32_t* mids, uint32_t* sc, uint32_t* rm)
{
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nl) return;
    const uint32_t k = klist ? klist[t] : (uint32_t)t;
    const uint32_t pos = p_pos[k];
    if (!pos) return;
    const uint32_t lo = d.krec[k].seg_lo, npb = lo + pos, x_npb = p_xr[k];
    const uint32_t L0 = d.mref[npb];
    uint32_t nret = 0;
    for (uint32_t e = lo; e < npb; ++e)
    {
        if (d.status[e] != AD_ST_APPLIED || d.xrank[e] >= x_npb) continue;
        const uint32_t L = d.mref[e];
        bool subset = true;
        if (L != MREF_NONE && L != MREF_BORN)
            for (uint64_t j = moff[L]; j < moff[L + 1] && subset; ++j)
            {
                const uint32_t r = mids[j];
                bool in = list_has(moff, mids, L0, r);
                for (uint32_t q = 0; q < nret && !in; ++q) in = list_has(moff, mids, d.mref[sc[lo + q]], r);
                subset = in;
            }
        if (subset)
        {
            rm[e] = 1u;
            continue;
        }
        if (d.xrank[e] == (d.ent[e].y & RANK_MASK)) sc[lo + nret++] = e;
    }
}

// thread per key: segments after the removals; prunedBefore where entries went (:255-257: a key
// without removals keeps its CommandsForKey, prunedBefore included)
__global__ void k_prune_keys(uint64_t nk, KeyRec* krec, const uint64_t* rpos, const uint32_t* p_pos, const uint32_t* p_tr,
                             unsigned long long* n_keys_pruned)
{
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nk) return;
    KeyRec kr = krec[k];
    const uint64_t r_lo = rpos[kr.seg_lo], r_hi = rpos[kr.seg_hi];
    if (p_pos[k] && r_hi > r_lo)
    {
        kr.pruned = p_tr[k];
        atomicAdd(n_keys_pruned, 1ull);
    }
    kr.seg_lo -= (uint32_t)r_lo;
    kr.seg_hi -= (uint32_t)r_hi;
    krec[k] = kr;
}

__global__ __launch_bounds__(256) void k_prune_move(uint64_t ne, EntArrays a, const uint32_t* rm, const uint64_t* rpos,
                                                    EntArrays b)
{
    const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= ne || rm[e]) return;
    const uint64_t j = e - rpos[e];
    b.ent[j] = a.ent[e];
    b.status[j] = a.status[e];
    b.xrank[j] = a.xrank[e];
    b.ekey[j] = a.ekey[e];
    if (a.bal) b.bal[j] = a.bal[e];
    if (a.mref) b.mref[j] = a.mref[e];
}

}  // namespace

// A freshly ingested snapshot (ingest.hip): every derived array from the per-entry state, the
// committed order sorted in full.
int run_cfk_derive_full(CfkUpdWork* w, DevSnapshot& s, CfkDevState& d, CfkDerivedBufs* bufs,
                        int (*need)(void* ctx, uint64_t cand, uint64_t cwr, uint64_t w, CfkDerivedBufs* bufs), void* need_ctx,
                        hipStream_t st, uint64_t* bad_entry, std::string* err)
{
    if (!w->h_ctl && hipHostMalloc((void**)&w->h_ctl, sizeof(UpdCtl)) != hipSuccess) { *err = "pinned ctl"; return AD_E_NOMEM; }
    UALLOC(w->ctl, sizeof(UpdCtl), false);
    UCHK(hipMemsetAsync(w->ctl.p, 0, sizeof(UpdCtl), st));
    w->cm_valid = false;
    w->moved = false;
    if (int rc = cfk_derive(w, s, d, bufs, need, need_ctx, st, err)) return rc;
    UCHK(d2h(w->h_ctl, w->ctl.p, sizeof(UpdCtl), st));
    UCHK(hipStreamSynchronize(st));
    if (w->h_ctl->err)
    {
        *bad_entry = w->h_ctl->err_idx;
        *err = "two committed entries of one key share an executeAt (CommandsForKey.java:1439)";
        return AD_E_DUP_EXEC;
    }
    return AD_OK;
}

int run_cfk_prune(CfkUpdWork* w, DevSnapshot& s, CfkDevState& d, const uint32_t* klist, uint64_t nl, int32_t prune_interval,
                  int64_t min_hlc_delta, CfkDerivedBufs* bufs,
                  int (*need)(void* ctx, uint64_t cand, uint64_t cwr, uint64_t w, CfkDerivedBufs* bufs), void* need_ctx,
                  const CfkGrow& grow, hipStream_t st, CfkPruneOut* out, std::string* err, CfkMiss* miss)
{
    *out = CfkPruneOut{};
    const uint64_t ne = s.n_ent, nk = s.n_keys;
    if (!nk || !ne || !nl) return AD_OK;
    if (!w->h_ctl && hipHostMalloc((void**)&w->h_ctl, sizeof(UpdCtl)) != hipSuccess) { *err = "pinned ctl"; return AD_E_NOMEM; }
    for (auto& e : w->ev)
        if (!e) UCHK(timing_event(&e));
    UALLOC(w->ctl, sizeof(UpdCtl), false);
    UpdCtl* ctl = w->ctl.as<UpdCtl>();
    UCHK(hipMemsetAsync(ctl, 0, sizeof(UpdCtl), st));
    UCHK(hipEventRecord(w->ev[0], st));
    // the committed order of the current entries (a derivation keeps it; after the ingest, derive once)
    if (!w->cm_valid)
    {
        UALLOC(w->chg[w->chg_cur], ne, false);
        w->moved = false;
        if (int rc = cfk_derive(w, s, d, bufs, need, need_ctx, st, err)) return rc;
        UCHK(hipMemsetAsync(ctl, 0, sizeof(UpdCtl), st));
    }
    UALLOC(w->flags, 4 * ne, false);
    UALLOC(w->fs, 8 * (ne + 1), false);
    UALLOC(w->bsum, 8 * ((ne + 1023) / 1024 + 8), false);
    UALLOC(w->maw, 4 * nk, false);          // p_pos
    UALLOC(w->wtail, 4 * nk, false);        // p_xr
    UALLOC(w->gkey, 4 * nk, false);         // p_tr
    UALLOC(w->uflag, 4 * ne, false);        // rm
    UALLOC(w->upos, 8 * (ne + 1), false);   // rpos
    uint32_t* p_pos = w->maw.as<uint32_t>();
    uint32_t* p_xr = w->wtail.as<uint32_t>();
    uint32_t* p_tr = w->gkey.as<uint32_t>();
    k_prune_cflag<<<blocks(ne), 256, 0, st>>>(ne, d.status, w->flags.as<uint32_t>());
    UCHK(run_scan_arrays(w->flags.as<uint32_t>(), w->fs.as<uint64_t>(), ne, 1, w->bsum.as<uint64_t>(), st));
    UCHK(hipMemsetAsync(p_pos, 0, 4 * nk, st));
    k_prune_key<<<blocks(nl), 256, 0, st>>>(nl, klist, s, d, w->cm.as<uint32_t>(), w->fs.as<uint64_t>(), prune_interval,
                                            min_hlc_delta, p_pos, p_xr, p_tr);
    k_prune_mark<<<blocks(ne), 256, 0, st>>>(ne, d, p_pos, p_xr, w->uflag.as<uint32_t>());
    const bool lists = d.mref && miss && miss->on;
    if (lists)
    {
        UALLOC(w->dsrc, 4 * ne, false);       // the subset walk's kept entries (per key, in its segment)
        k_prune_subset<<<blocks(nl), 256, 0, st>>>(nl, klist, d, p_pos, p_xr, miss->off, miss->ids, w->dsrc.as<uint32_t>(),
                                                   w->uflag.as<uint32_t>());
    }
    UCHK(hipGetLastError());
    UCHK(run_scan_arrays(w->uflag.as<uint32_t>(), w->upos.as<uint64_t>(), ne, 1, w->bsum.as<uint64_t>(), st));
    k_drv_totals<<<1, 64, 0, st>>>(w->upos.as<uint64_t>(), ne, 1, ctl->tot2);
    UCHK(d2h(w->h_ctl, ctl, sizeof(UpdCtl), st));
    UCHK(hipStreamSynchronize(st));
    const uint64_t R = w->h_ctl->tot2[0];
    if (R == 0)
    {
        UCHK(hipEventRecord(w->ev[1], st));
        UCHK(hipEventSynchronize(w->ev[1]));
        float a = 0;
        (void)hipEventElapsedTime(&a, w->ev[0], w->ev[1]);
        out->ms_total = a;
        return AD_OK;
    }
    // compaction into the spare per-entry arrays, segments and prunedBefore, then a full derivation
    unsigned long long* nkp = reinterpret_cast<unsigned long long*>(&ctl->tot2[1]);
    UCHK(hipMemsetAsync(nkp, 0, 8, st));
    EntArrays a{d.ent, d.status, d.xrank, d.ekey, d.ballot, nullptr, d.mref}, b{};
    if (int rc = grow.entries(grow.ctx, ne - R, &b.ent, &b.status, &b.xrank, &b.ekey, &b.bal, &b.mref)) { *err = "entry arrays"; return rc; }
    const uint64_t padded = std::max<uint64_t>(64, (ne - R + 63) / 64 * 64);
    if (padded > ne - R) UCHK(hipMemsetAsync(b.ent + (ne - R), 0, sizeof(uint2) * (padded - (ne - R)), st));
    k_prune_move<<<blocks(ne), 256, 0, st>>>(ne, a, w->uflag.as<uint32_t>(), w->upos.as<uint64_t>(), b);
    k_prune_keys<<<blocks(nk), 256, 0, st>>>(nk, d.krec, w->upos.as<uint64_t>(), p_pos, p_tr, nkp);
    UCHK(hipGetLastError());
    if (int rc = grow.swap(grow.ctx, ne - R, &d.ent, &d.status, &d.xrank, &d.ekey, &d.ballot, &d.mref)) { *err = "entry swap"; return rc; }
    s.ent = d.ent;
    s.n_ent = ne - R;
    w->cm_valid = false;          // entry indices changed: the next derivation sorts afresh
    w->moved = false;
    UALLOC(w->chg[w->chg_cur], std::max<uint64_t>(ne - R, 1), false);
    UCHK(d2h(w->h_ctl, ctl, sizeof(UpdCtl), st));
    UCHK(hipStreamSynchronize(st));
    out->n_keys_pruned = w->h_ctl->tot2[1];
    out->n_removed = R;
    UCHK(hipMemsetAsync(ctl, 0, sizeof(UpdCtl), st));
    if (int rc = cfk_derive(w, s, d, bufs, need, need_ctx, st, err)) return rc;
    if (lists)
    {
        // the kept entries' lists, compacted again (each entry its own list, pruned ones dropped)
        const uint64_t n2 = s.n_ent;
        UALLOC(w->dsrc, 4 * n2, false);
        UALLOC(w->mflag, 4 * 2 * n2, false);
        UALLOC(w->mpp, 8 * 2 * (n2 + 1), false);
        UALLOC(w->mpend, 4 * 2 * n2, false);
        UALLOC(w->mcnt, 4 * n2, false);
        UALLOC(w->moff, 8 * (n2 + 1), false);
        UALLOC(w->bsum, 8 * 2 * ((n2 + 1023) / 1024 + 8), false);
        UCHK(hipMemsetAsync(w->dsrc.p, 0xFF, 4 * n2, st));
        k_miss_flags<<<blocks(n2), 256, 0, st>>>(n2, d, w->mflag.as<uint32_t>());
        UCHK(run_scan_arrays(w->mflag.as<uint32_t>(), w->mpp.as<uint64_t>(), n2, 2, w->bsum.as<uint64_t>(), st));
        k_miss_scatter<<<blocks(n2), 256, 0, st>>>(n2, w->mflag.as<uint32_t>(), w->mpp.as<uint64_t>(), w->mpend.as<uint32_t>());
        const CfkUpdIn none{};
        k_miss_build<0><<<blocks(n2), 256, 0, st>>>(s, d, none, w->dsrc.as<uint32_t>(), nullptr, w->mpp.as<uint64_t>(),
                                                    w->mpend.as<uint32_t>(), miss->off, miss->ids, w->mcnt.as<uint32_t>(),
                                                    nullptr, nullptr);
        UCHK(run_scan_arrays(w->mcnt.as<uint32_t>(), w->moff.as<uint64_t>(), n2, 1, w->bsum.as<uint64_t>(), st));
        uint64_t nm = 0;
        UCHK(d2h(&nm, w->moff.as<uint64_t>() + n2, 8, st));
        UCHK(hipStreamSynchronize(st));
        uint64_t* noff = nullptr;
        uint32_t* nids = nullptr;
        if (int rc = miss->spare(miss->ctx, n2, nm, &noff, &nids)) { *err = "missing() lists"; return rc; }
        UCHK(hipMemcpyAsync(noff, w->moff.p, 8 * (n2 + 1), hipMemcpyDeviceToDevice, st));
        k_miss_build<1><<<blocks(n2), 256, 0, st>>>(s, d, none, w->dsrc.as<uint32_t>(), nullptr, w->mpp.as<uint64_t>(),
                                                    w->mpend.as<uint32_t>(), miss->off, miss->ids, nullptr, noff, nids);
        k_mref_identity<<<blocks(n2), 256, 0, st>>>(n2, d.mref);
        UCHK(hipGetLastError());
        UCHK(hipStreamSynchronize(st));
        if (int rc = miss->swap(miss->ctx, &miss->off, &miss->ids)) { *err = "missing() lists"; return rc; }
        miss->n_lists = n2;
    }
    UCHK(hipEventRecord(w->ev[1], st));
    UCHK(d2h(w->h_ctl, ctl, sizeof(UpdCtl), st));
    UCHK(hipStreamSynchronize(st));
    float a_ms = 0;
    (void)hipEventElapsedTime(&a_ms, w->ev[0], w->ev[1]);
    out->ms_total = a_ms;
    if (w->h_ctl->err) { *err = "derivation after pruning reported an inconsistency"; return AD_E_STATE; }
    return AD_OK;
}


// =============================================================================================
// RedundantBefore on the device: SafeCommandStore.maybeTruncate (SafeCommandStore.java:165-171) ->
// SafeCommandsForKey.updateRedundantBefore -> CommandsForKey.withRedundantBeforeAtLeast
// (CommandsForKey.java:1317-1341). For every key, the byId entries below its RedundantBefore entry's
// shardRedundantBefore leave and the missing() lists of the rest lose the ids below it
// (Utils.removeRedundantMissing, Utils.java:265-275) -- both only where something left
// (insertPos != 0); a prunedBefore at or below it becomes NO_INFO (the constructor, :646-648). The
// watermarks are the snapshot's rb_wm ranks (dictionary members; 0 = NONE).
// =============================================================================================
namespace {

// the RedundantBefore entry holding key x (RedundantBefore.get: a lookup over the disjoint ascending
// entries; epochs not read), or ~0
__device__ inline uint64_t rb_entry_holding(const DevSnapshot& s, int64_t x)
{
    const bool incl = s.start_inclusive != 0;
    uint64_t lo = 0, hi = s.n_rb;
    while (lo < hi)
    {
        const uint64_t m = (lo + hi) >> 1;
        if (incl ? s.rb_start[m] <= x : s.rb_start[m] < x) lo = m + 1;
        else hi = m;
    }
    if (!lo) return ~0ull;
    return range_contains(s.start_inclusive, s.rb_start[lo - 1], s.rb_end[lo - 1], x) ? lo - 1 : ~0ull;
}

// thread per key: t_pos[k] = insertPos(shardRedundantBefore) within byId (the entries that leave),
// t_wm[k] = its rank (0: NONE or no entry); a prunedBefore at or below it is cleared in place;
// *n_chg counts the keys that change
__global__ void k_trunc_key(uint64_t nk, DevSnapshot s, KeyRec* krec, uint32_t* t_pos, uint32_t* t_wm,
                            unsigned long long* n_chg)
{
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nk) return;
    uint32_t pos = 0, wm = 0;
    const uint64_t e = rb_entry_holding(s, s.keys[k]);
    if (e != ~0ull) wm = s.rb_wm[e];
    bool chg = false;
    if (wm)
    {
        const KeyRec kr = krec[k];
        uint32_t lo = kr.seg_lo, hi = kr.seg_hi;
        while (lo < hi)
        {
            const uint32_t m = (lo + hi) >> 1;
            if ((s.ent[m].y & RANK_MASK) < wm) lo = m + 1;
            else hi = m;
        }
        pos = lo - kr.seg_lo;
        chg = pos != 0;
        if (kr.pruned && wm >= kr.pruned)
        {
            krec[k].pruned = 0;
            chg = true;
        }
    }
    t_pos[k] = pos;
    t_wm[k] = wm;
    if (chg) atomicAdd(n_chg, 1ull);
}

// thread per entry: below its key's shardRedundantBefore (a prefix of the key's byId)
__global__ void k_trunc_mark(uint64_t ne, const uint32_t* ekey, const KeyRec* krec, const uint32_t* t_pos, uint32_t* rm)
{
    const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= ne) return;
    const uint32_t k = ekey[e];
    rm[e] = (e - krec[k].seg_lo < t_pos[k]) ? 1u : 0u;
}

// thread per key: segments after the removals (an emptied byId has no last txnId)
__global__ void k_trunc_keys(uint64_t nk, KeyRec* krec, const uint64_t* rpos)
{
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nk) return;
    KeyRec kr = krec[k];
    kr.seg_lo -= (uint32_t)rpos[kr.seg_lo];
    kr.seg_hi -= (uint32_t)rpos[kr.seg_hi];
    if (kr.seg_hi == kr.seg_lo) kr.last_txn = 0;
    krec[k] = kr;
}

// thread per kept entry (its list mref[j] of the old CSR): the ids at or above the key's
// shardRedundantBefore where entries left (removeRedundantMissing), all of them elsewhere. Pass 0
// counts, pass 1 writes.
template <int WRITE>
__global__ __launch_bounds__(256) void k_trunc_miss(uint64_t n, const uint32_t* mref, const uint32_t* ekey,
                                                    const uint32_t* t_pos, const uint32_t* t_wm, const uint64_t* ooff,
                                                    const uint32_t* oids, uint32_t* cnt, const uint64_t* noff, uint32_t* nids)
{
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const uint32_t L = mref[j];
    uint64_t c = 0, o = WRITE ? noff[j] : 0;
    if (L != MREF_NONE && L != MREF_BORN)
    {
        const uint32_t k = ekey[j];
        const uint32_t lb = t_pos[k] ? t_wm[k] : 0;
        for (uint64_t a = ooff[L]; a < ooff[L + 1]; ++a)
        {
            const uint32_t r = oids[a];
            if (r < lb) continue;
            if (WRITE) nids[o++] = r;
            ++c;
        }
    }
    if (!WRITE) cnt[j] = (uint32_t)c;
}

// thread per id: its dictionary rank (a member after run_cfk_dict_ensure); a miss flags ctl->err
__global__ void k_id_ranks(DevSnapshot s, DictSample ds, uint64_t n, const uint64_t* msb, const uint64_t* lsb,
                           const int32_t* node, const uint64_t* dict_lsb_raw, uint32_t* rank, UpdCtl* ctl)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t p;
    const uint32_t r = dict_member_rank(s, ds, norm_tid(msb[i], lsb[i], node[i]), &p);
    rank[i] = r;
    if (!r) upd_fail(ctl, UE_ABSENT, (uint32_t)i);
    else if (dict_lsb_raw[p] != lsb[i]) upd_fail(ctl, UE_FLAGS, (uint32_t)i);     // equal ids, other flag bits
}

}  // namespace

int run_cfk_truncate(CfkUpdWork* w, DevSnapshot& s, CfkDevState& d, CfkDerivedBufs* bufs,
                     int (*need)(void* ctx, uint64_t cand, uint64_t cwr, uint64_t w, CfkDerivedBufs* bufs), void* need_ctx,
                     const CfkGrow& grow, hipStream_t st, CfkTruncOut* out, std::string* err, CfkMiss* miss,
                     uint32_t* h_pos)
{
    *out = CfkTruncOut{};
    const uint64_t ne = s.n_ent, nk = s.n_keys;
    if (!nk || !s.n_rb) return AD_OK;
    if (!w->h_ctl && hipHostMalloc((void**)&w->h_ctl, sizeof(UpdCtl)) != hipSuccess) { *err = "pinned ctl"; return AD_E_NOMEM; }
    for (auto& e : w->ev)
        if (!e) UCHK(timing_event(&e));
    UALLOC(w->ctl, sizeof(UpdCtl), false);
    UpdCtl* ctl = w->ctl.as<UpdCtl>();
    UCHK(hipMemsetAsync(ctl, 0, sizeof(UpdCtl), st));
    UCHK(hipEventRecord(w->ev[0], st));
    UALLOC(w->tpos, 4 * nk, false);
    UALLOC(w->twm, 4 * nk, false);
    uint32_t* t_pos = w->tpos.as<uint32_t>();
    uint32_t* t_wm = w->twm.as<uint32_t>();
    unsigned long long* n_chg = reinterpret_cast<unsigned long long*>(&ctl->tot2[1]);
    k_trunc_key<<<blocks(nk), 256, 0, st>>>(nk, s, d.krec, t_pos, t_wm, n_chg);
    if (ne)
    {
        UALLOC(w->uflag, 4 * ne, false);        // rm
        UALLOC(w->upos, 8 * (ne + 1), false);   // rpos
        UALLOC(w->bsum, 8 * ((ne + 1023) / 1024 + 8), false);
        k_trunc_mark<<<blocks(ne), 256, 0, st>>>(ne, d.ekey, d.krec, t_pos, w->uflag.as<uint32_t>());
        UCHK(run_scan_arrays(w->uflag.as<uint32_t>(), w->upos.as<uint64_t>(), ne, 1, w->bsum.as<uint64_t>(), st));
        k_drv_totals<<<1, 64, 0, st>>>(w->upos.as<uint64_t>(), ne, 1, ctl->tot2);
    }
    UCHK(hipGetLastError());
    UCHK(d2h(w->h_ctl, ctl, sizeof(UpdCtl), st));
    UCHK(hipStreamSynchronize(st));
    const uint64_t R = ne ? w->h_ctl->tot2[0] : 0, changed = w->h_ctl->tot2[1];
    auto finish = [&]() -> int {
        UCHK(hipEventRecord(w->ev[1], st));
        UCHK(hipEventSynchronize(w->ev[1]));
        float a = 0;
        (void)hipEventElapsedTime(&a, w->ev[0], w->ev[1]);
        out->ms_total = a;
        return AD_OK;
    };
    if (!changed) return finish();
    if (h_pos) UCHK(d2h(h_pos, t_pos, 4 * nk, st));      // the host's lists follow (the caller trims them)
    if (R)
    {
        // compaction into the spare per-entry arrays and the segments, as pruning does
        EntArrays a{d.ent, d.status, d.xrank, d.ekey, d.ballot, nullptr, d.mref}, b{};
        if (int rc = grow.entries(grow.ctx, ne - R, &b.ent, &b.status, &b.xrank, &b.ekey, &b.bal, &b.mref)) { *err = "entry arrays"; return rc; }
        const uint64_t padded = std::max<uint64_t>(64, (ne - R + 63) / 64 * 64);
        if (padded > ne - R) UCHK(hipMemsetAsync(b.ent + (ne - R), 0, sizeof(uint2) * (padded - (ne - R)), st));
        k_prune_move<<<blocks(ne), 256, 0, st>>>(ne, a, w->uflag.as<uint32_t>(), w->upos.as<uint64_t>(), b);
        k_trunc_keys<<<blocks(nk), 256, 0, st>>>(nk, d.krec, w->upos.as<uint64_t>());
        UCHK(hipGetLastError());
        if (int rc = grow.swap(grow.ctx, ne - R, &d.ent, &d.status, &d.xrank, &d.ekey, &d.ballot, &d.mref)) { *err = "entry swap"; return rc; }
        s.ent = d.ent;
        s.n_ent = ne - R;
        UALLOC(w->chg[w->chg_cur], std::max<uint64_t>(ne - R, 1), false);
    }
    if (!R)
    {
        // only prunedBefore moved (krec, in place): nothing derived reads it
        out->n_keys = changed;
        return finish();
    }
    w->cm_valid = false;          // entry indices changed: the next derivation sorts afresh
    w->moved = false;
    UCHK(hipMemsetAsync(ctl, 0, sizeof(UpdCtl), st));
    if (int rc = cfk_derive(w, s, d, bufs, need, need_ctx, st, err)) return rc;
    if (d.mref && miss && miss->on)
    {
        // the kept entries' lists, trimmed and compacted (each entry its own list again)
        const uint64_t n2 = s.n_ent;
        UALLOC(w->mcnt, 4 * std::max<uint64_t>(n2, 1), false);
        UALLOC(w->moff, 8 * (n2 + 1), false);
        UALLOC(w->bsum, 8 * ((n2 + 1023) / 1024 + 8), false);
        if (n2)
            k_trunc_miss<0><<<blocks(n2), 256, 0, st>>>(n2, d.mref, d.ekey, t_pos, t_wm, miss->off, miss->ids,
                                                        w->mcnt.as<uint32_t>(), nullptr, nullptr);
        UCHK(run_scan_arrays(w->mcnt.as<uint32_t>(), w->moff.as<uint64_t>(), n2, 1, w->bsum.as<uint64_t>(), st));
        uint64_t nm = 0;
        UCHK(d2h(&nm, w->moff.as<uint64_t>() + n2, 8, st));
        UCHK(hipStreamSynchronize(st));
        uint64_t* noff = nullptr;
        uint32_t* nids = nullptr;
        if (int rc = miss->spare(miss->ctx, n2, nm, &noff, &nids)) { *err = "missing() lists"; return rc; }
        UCHK(hipMemcpyAsync(noff, w->moff.p, 8 * (n2 + 1), hipMemcpyDeviceToDevice, st));
        if (n2)
        {
            k_trunc_miss<1><<<blocks(n2), 256, 0, st>>>(n2, d.mref, d.ekey, t_pos, t_wm, miss->off, miss->ids, nullptr, noff,
                                                        nids);
            k_mref_identity<<<blocks(n2), 256, 0, st>>>(n2, d.mref);
        }
        UCHK(hipGetLastError());
        UCHK(hipStreamSynchronize(st));
        if (int rc = miss->swap(miss->ctx, &miss->off, &miss->ids)) { *err = "missing() lists"; return rc; }
        miss->n_lists = n2;
    }
    UCHK(d2h(w->h_ctl, ctl, sizeof(UpdCtl), st));
    UCHK(hipStreamSynchronize(st));
    if (w->h_ctl->err) { *err = "derivation after truncation reported an inconsistency"; return AD_E_STATE; }
    out->n_removed = R;
    out->n_keys = changed;
    return finish();
}

int run_cfk_dict_ensure(CfkUpdWork* w, DevSnapshot& s, CfkDevState& d, const uint64_t* msb, const uint64_t* lsb,
                        const int32_t* node, uint64_t n, const CfkGrow& grow, CfkDerivedBufs* bufs,
                        int (*need)(void* ctx, uint64_t cand, uint64_t cwr, uint64_t w, CfkDerivedBufs* bufs), void* need_ctx,
                        hipStream_t st, CfkUpdOut* out, uint32_t* ranks, std::string* err)
{
    *out = CfkUpdOut{};
    if (!n) return AD_OK;
    if (!w->h_ctl && hipHostMalloc((void**)&w->h_ctl, sizeof(UpdCtl)) != hipSuccess) { *err = "pinned ctl"; return AD_E_NOMEM; }
    UALLOC(w->ctl, sizeof(UpdCtl), false);
    UpdCtl* ctl = w->ctl.as<UpdCtl>();
    UCHK(hipMemsetAsync(ctl, 0, sizeof(UpdCtl), st));
    UALLOC(w->ids_st, n, false);
    UCHK(hipMemsetAsync(w->ids_st.p, 0, n, st));       // TRANSITIVELY_KNOWN: the txnId side only
    CfkUpdIn u{};
    u.n = n;
    u.txn_msb = u.exec_msb = msb;
    u.txn_lsb = u.exec_lsb = lsb;
    u.txn_node = u.exec_node = node;
    u.status = w->ids_st.as<uint8_t>();
    const uint64_t ns = std::max<uint64_t>((s.n_dict + n + SAMP - 1) / SAMP, 1);
    UALLOC(w->sm_hi, 8 * ns, false);
    UALLOC(w->sm_lo, 8 * ns, false);
    UALLOC(w->sm_node, 4 * ns, false);
    auto sample = [&]() -> DictSample {
        const uint64_t n_samp = (s.n_dict + SAMP - 1) / SAMP;
        if (n_samp)
            k_dict_sample<<<blocks(n_samp), 256, 0, st>>>(s, w->sm_hi.as<uint64_t>(), w->sm_lo.as<uint64_t>(),
                                                          w->sm_node.as<int32_t>(), n_samp);
        return DictSample{w->sm_hi.as<uint64_t>(), w->sm_lo.as<uint64_t>(), w->sm_node.as<int32_t>(), n_samp};
    };
    const DictSample ds0 = sample();
    if (int rc = grow_dictionary(w, s, d, ds0, u, grow, st, out, err)) return rc;
    if (w->h_ctl->err)
    {
        *err = "ids equal under Timestamp.equals differ in flag bits";
        return AD_E_INCONSISTENT_ID;
    }
    if (out->merged)
    {
        // a merge remapped the per-entry ranks in place: the derived arrays (cand / cwr / w / KeyEntry / trees) hold
        // the old ones -- derive them again (the committed order's entry indices stand, its ranks do not: sort afresh)
        w->cm_valid = false;
        w->moved = false;
        UALLOC(w->chg[w->chg_cur], std::max<uint64_t>(s.n_ent, 1), false);
        UCHK(hipMemsetAsync(ctl, 0, sizeof(UpdCtl), st));
        if (int rc = cfk_derive(w, s, d, bufs, need, need_ctx, st, err)) return rc;
        out->rederived = true;
    }
    const DictSample ds1 = sample();
    UCHK(hipMemsetAsync(ctl, 0, sizeof(UpdCtl), st));
    k_id_ranks<<<blocks(n), 256, 0, st>>>(s, ds1, n, msb, lsb, node, d.dict_lsb_raw, ranks, ctl);
    UCHK(hipGetLastError());
    UCHK(d2h(w->h_ctl, ctl, sizeof(UpdCtl), st));
    UCHK(hipStreamSynchronize(st));
    if (w->h_ctl->err == UE_FLAGS)
    {
        *err = "ids equal under Timestamp.equals differ in flag bits";
        return AD_E_INCONSISTENT_ID;
    }
    if (w->h_ctl->err) { *err = "id missing from the dictionary after its growth (internal)"; return AD_E_STATE; }
    return AD_OK;
}

}  // namespace adx
