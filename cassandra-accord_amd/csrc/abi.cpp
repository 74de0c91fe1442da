// abi.cpp — C ABI of libaccord_deps.so: store context, snapshot ingest (id dictionary, ranks,
// per-key index arrays, range-entry table) and the batch pipeline driving kernels.hip.
//
// Ingest restates the derived state of CommandsForKey's constructor (CommandsForKey.java:642-681:
// committedByExecuteAt, maxAppliedWriteByExecuteAt, prunedBefore) and of
// InMemoryCommandStore.rangeCommands (:740-763) once per snapshot; the batch pipeline then
// answers calculatePartialDeps for every request of a batch on the GPU.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <sys/mman.h>
#include <numeric>
#include <string>
#include <thread>
#include <vector>

#include "../../include/accord_deps.h"
#include "common.hpp"
#include "exchange.hpp"
#include "kernels.hpp"
#include "levels.hpp"
#include "cfk_update.hpp"
#include "ingest.hpp"
#include "check.hpp"
#include "devmem.hpp"

using namespace adx;

namespace {

// ---------------------------------------------------------------------------------------
// helpers
// ---------------------------------------------------------------------------------------
struct Tid {
    uint64_t msb, lsb;
    int32_t node;
};

static inline NormTid norm(const Tid& t) { return norm_tid(t.msb, t.lsb, t.node); }

static unsigned n_threads()
{
    unsigned n = std::thread::hardware_concurrency();
    if (const char* e = getenv("OMP_NUM_THREADS")) n = std::max(1, atoi(e));
    return std::max(1u, std::min(n, 16u));
}

template <class T, class Cmp>
static void parallel_sort(std::vector<T>& v, Cmp cmp)
{
    const size_t n = v.size();
    unsigned T_ = n_threads();
    if (n < (1u << 16) || T_ == 1)
    {
        std::sort(v.begin(), v.end(), cmp);
        return;
    }
    std::vector<size_t> cut(T_ + 1);
    for (unsigned i = 0; i <= T_; ++i) cut[i] = n * i / T_;
    {
        std::vector<std::thread> th;
        for (unsigned i = 0; i < T_; ++i)
            th.emplace_back([&, i] { std::sort(v.begin() + cut[i], v.begin() + cut[i + 1], cmp); });
        for (auto& t : th) t.join();
    }
    std::vector<T> tmp(n);
    std::vector<size_t> bounds = cut;
    bool in_v = true;
    while (bounds.size() > 2)
    {
        std::vector<size_t> nb;
        std::vector<std::thread> th;
        std::vector<T>& src = in_v ? v : tmp;
        std::vector<T>& dst = in_v ? tmp : v;
        for (size_t i = 0; i + 1 < bounds.size(); i += 2)
        {
            if (i + 2 < bounds.size())
            {
                size_t a = bounds[i], m = bounds[i + 1], e = bounds[i + 2];
                th.emplace_back([&, a, m, e] {
                    std::merge(src.begin() + a, src.begin() + m, src.begin() + m, src.begin() + e, dst.begin() + a, cmp);
                });
                nb.push_back(a);
            }
            else
            {
                size_t a = bounds[i], e = bounds[i + 1];
                th.emplace_back([&, a, e] { std::copy(src.begin() + a, src.begin() + e, dst.begin() + a); });
                nb.push_back(a);
            }
        }
        nb.push_back(n);
        for (auto& t : th) t.join();
        bounds.swap(nb);
        in_v = !in_v;
    }
    if (!in_v) v.swap(tmp);
}

// f(a, b) over host_threads() ranges of [0, n), on the persistent worker pool (devmem.hpp)
template <class F>
static void parallel_for(size_t n, F f, size_t grain = 1 << 14)
{
    const unsigned T_ = std::min(n_threads(), host_threads());
    if (n < grain * 2 || T_ == 1)
    {
        f(0, n);
        return;
    }
    host_parallel(T_, [&](size_t i) { f(n * i / T_, n * (i + 1) / T_); });
}

static double now_ms()
{
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // namespace

// ---------------------------------------------------------------------------------------
// the store context
// ---------------------------------------------------------------------------------------
struct ad_ctx {
    ad_config cfg{};
    std::vector<int64_t> slice_s, slice_e;
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;

    // host copies of the loaded inputs (needed to rebuild after SEQUENTIAL insertions)
    struct {
        std::vector<int64_t> keys;
        std::vector<uint64_t> seg;
        std::vector<Tid> txn, exec;
        std::vector<uint8_t> status;
        std::vector<int64_t> pruned;           // per key; -1 none
        std::vector<uint64_t> miss_off;        // TxnInfo.missing() per entry (ad_cfk_missing_load); empty = none
        std::vector<Tid> miss;
        std::vector<Tid> ballot;               // TxnInfo.ballot() per entry; empty = all Ballot.ZERO
        bool miss_stale = false;               // SEQUENTIAL insertions moved the entries after the load
        bool loaded = false;
    } cfk;
    struct {
        std::vector<Tid> txn;
        std::vector<uint8_t> erased, historical;
        std::vector<uint64_t> off;
        std::vector<int64_t> start, end;
        // recovery facts (ad_range_cmds_recovery_load)
        bool rec = false;
        std::vector<uint8_t> rec_status, rec_has_deps;
        std::vector<Tid> rec_exec, rec_deps;
        std::vector<uint64_t> rec_dep_off;
    } cmds;
    // per range entry of the snapshot (device order): live-command flag, and the command of each rank
    std::vector<uint32_t> h_rtxw;
    std::vector<uint8_t> h_rlive;
    std::vector<uint32_t> h_cmd_rank;
    struct {
        std::vector<int64_t> start, end, e0, e1;
        std::vector<Tid> wm;
    } rb;
    bool dirty = true;
    double ms_ingest = 0;

    // built snapshot
    std::vector<uint64_t> dict_msb, dict_lsb;
    std::vector<int32_t> dict_node;
    std::vector<int64_t> rt_start, rt_end;     // range table (distinct ranges, by Range.compare)
    DevSnapshot ds{};
    DevBuf d_dict_hi, d_dict_lo, d_dict_node, d_keys, d_krec, d_khash, d_kent, d_cand, d_cwr, d_ent, d_w;
    DevBuf d_lvl[NCLASS][MAX_LEVELS];
    DevBuf d_rstart, d_rend, d_rtxw, d_rrid, d_cell_E, d_cell_off, d_cell_ent;
    uint64_t n_cell_ent = 0;                   // entries of d_cell_ent
    DevBuf d_rlvl[NCLASS][MAX_LEVELS];
    DevBuf d_rb_s, d_rb_e, d_rb_e0, d_rb_e1, d_rb_wm, d_rb_rid, d_slices_s, d_slices_e;
    DevBuf d_dict_lsb_raw, d_rt_start, d_rt_end;   // raw ids and range table (multi-GPU export)
    DevBuf d_ds_hi, d_ds_lo, d_ds_node;            // every DICT_SAMP-th dictionary id (rank searches)
    DevBuf d_kline, d_kslot, d_kcell, d_kl_disp;   // KeyLine table; per key its line and stabbing cell; displacements
    uint64_t kline_slots = 0;
    // host state of the KeyLine perfect hash (incremental placement of new keys)
    std::vector<uint32_t> kl_disp_h;
    std::vector<uint8_t> kl_used;
    std::vector<std::vector<int64_t>> kl_members;   // per bucket (built on first use from kl_keys_all)
    std::vector<int64_t> kl_keys_all;
    uint64_t kl_nb_h = 0;
    DevBuf d_keys2, d_krec2, d_kcell2, d_khash2, d_kent2;   // spare key-indexed arrays (new keys)

    // batch buffers
    DevBuf q_tm, q_tl, q_tn, q_em, q_el, q_en, q_me, q_ko, q_k;
    DevBuf q_ro, q_rs, q_re;                   // Range-domain requests: staged ranges
    DevBuf lg_stage, lg_rec, lg_keys, lg_dummy;   // lean gather + build: staged emissions, build records, keys
    bool upd_applied = false;                  // ad_cfk_update_status: the last update batch stands
    int64_t upd_failed = -1;                   //   and the update its failure names
    DevBuf rq_cnt, rq_off, rq_err, rq_bsum, rq_keys, rq_hi, rq_kind, rq_list;   // their expansion into probes
    struct SplitBufs {       // per-request / per-probe arrays of the split kernels
        DevBuf t_S, t_self, t_kinds, t_epoch, p_txn, p_rec, p_off, p_c0, p_c1, p_roff, p_rcnt, p_rb, sz, t_reg;
    } split, sub;
    DevBuf s_tm, s_tl, s_tn, s_em, s_el, s_en, s_me, s_ko, s_k, s_cnt, s_khi, s_kind;   // deferred sub-batch inputs
    DevBuf p_slot;                             // lean passes: per probe its KeyLine (k_lean_slots)
    DevBuf arena, rarena;
    DevBuf sz, off, bsum, t_reg, reg, scratch, ctl, deferred, deferred1, deferred2, q_rec, big;
    DevBuf o_keys[3], o_txns[3], o_k2t[3];
    uint64_t o_cap[9] = {};                    // capacities of the packed outputs (elements)
    DevBuf d_prune_keys;                       // ad_cfk_prune: key indices of the list
    DevBuf chk;                                // ad_check_*: {violations, first failing item}
    DevBuf lb_agg, lb_inc;                     // tile sums and their prefixes (run_pack_lb)
    uint64_t key_cap = 0, rng_cap = 0, scr_cap = 0, reg_cap = 0;
    hipEvent_t ev[8] = {};
    hipEvent_t ev_slot = nullptr;      // fused path: after k_prepare
    hipEvent_t ev_lean = nullptr;      // fused path: after k_resolve_lean (both passes)
    hipEvent_t ev_lean1 = nullptr;     // fused path: after lean pass 1
    // lean pass 1's width for the next batch (lean_wide1): wide while the batches carry enough requests of
    // 33..64 raw emissions; lean_other = the share of requests the wide pass 1 still deferred
    bool lean_wide = true, lean_ran_wide = false;
    double lean_other = 0.0;
    hipEvent_t ev_sp0 = nullptr, ev_sp1 = nullptr;   // split path on the fused kernels' deferrals
    hipEvent_t ev_done = nullptr;      // end of a batch's work (default flags: the host reads what it copied)
    BatchCtl* h_ctl = nullptr;         // pinned mirror of the batch control block
    uint64_t* h_small = nullptr;       // pinned words the batch prologue reads back (key / range totals)
    // small uploads inside a call's stream of work (the export's owner bounds, the merge's source starts):
    // one pinned slot per use, each reused after the event of its previous copy (up_small)
    uint64_t* h_up[2] = {};
    hipEvent_t ev_up[2] = {};
    bool up_busy[2] = {};
    uint64_t* h_rb = nullptr;          // pinned words for small read-backs that end in one stream sync (rb_slot)
    // ad_deps_batch_into: a second result bank (offsets + packed arrays) so that one slice of a batch is
    // copied out while the next resolves, the copy-out stream and its events
    DevBuf off_b, o_keys_b[3], o_txns_b[3], o_k2t_b[3];
    hipStream_t cstream = nullptr;
    hipEvent_t ev_ready = nullptr, ev_copied[2] = {};
    // its key-only SNAPSHOT path: two pinned host staging buffers (slice j + 1 is packed into one while
    // slice j's H2D from the other has completed) and the device region one slice's inputs land in
    void* in_pin[2] = {nullptr, nullptr};
    size_t in_pin_cap[2] = {0, 0};
    DevBuf in_dev[2];
    hipStream_t hstream = nullptr;     // its host-to-device copies (beside the resolve and the copy-out)
    hipEvent_t ev_h2d[2] = {};
    // the wire form of keyDeps (key indices u8, k2t u16): device index buffer, flag, pinned landing
    // buffers per result bank
    DevBuf w_idx, w_flag;
    void* w_pin[2][2] = {{nullptr, nullptr}, {nullptr, nullptr}};
    size_t w_pin_cap[2][2] = {{0, 0}, {0, 0}};
    // multi-GPU export / merge buffers
    DevBuf x_sz, x_off, x_bsum, x_df, x_cnt;
    // regions of the last device batch (ad_parts_export of an AD_PARTS_ONLY result)
    const uint8_t* last_reg = nullptr;
    const uint64_t* last_t_reg = nullptr;
    uint64_t last_n = 0;
    bool last_parts_only = false;
    DevBuf m_pinfo, m_heavy;
    DevBuf m_src, m_psz, m_poff, m_slot, m_dup, m_gsz, m_goff, m_bsum, m_err, m_bases;
    DevBuf m_ko, m_to, m_oo, m_keys, m_ids, m_k2t, m_u, m_ppre;
    DevBuf m_kdp, m_kuk, m_khead, m_pdp, m_ppos;   // ad_parts_union scratch
    // maxConflicts / rejectBefore of the PreAccept timestamp proposal (ad_preaccept_maps_load)
    struct RangeMapBufs {
        DevBuf starts, msb, lsb, node, present;
        uint64_t n = 0;
        uint32_t inclusive_ends = 0;
        bool has_present = false;
    } pa_mc, pa_rb;
    uint64_t pa_gen = 0, snap_gen = 0;         // map loads / snapshot builds
    uint64_t pa_iv_gen[2] = {~0ull, ~0ull};    // (pa_gen, snap_gen) the per-key values were built for
    DevBuf pa_key_val;
    // recovery scans (ad_recovery_batch*): entry ranks kept from the last snapshot build, device view
    std::vector<uint32_t> h_txn_rank, h_exec_rank, h_pruned;
    uint64_t rv_gen = ~0ull;                   // snap_gen the device view was built for
    uint64_t rank_gen = 0, rv_rng_gen = ~0ull; // rank-space changes (builds, dictionary merges); the view's range part
    DevBuf rv_cnt, rv_eoff, rv_bsum, rv_err, rv_pk, rv_pv, rv_pk2, rv_pv2, rv_hist, rv_hoff;   // device-built view scratch
    bool rv_dev_miss = false;                  // the view's missing() ids are the device lists (d_mids)
    DevBuf rv_ent, rv_seg, rv_pruned, rv_miss, rv_tree, rv_inv_off, rv_inv;
    DevBuf rv_rcmd, rv_rflags, rv_rex_hi, rv_rex_lo, rv_rex_node, rv_rdep_off, rv_rdep_hi, rv_rdep_lo, rv_rdep_node;
    bool rv_ranges = false;
    int rv_levels = 0;
    std::vector<uint64_t> rv_lvl_at;
    uint64_t rv_per_set = 0;
    // global dictionary of the multi-store exchange (ad_set_global_dict)
    // node-wide dictionary installed with ad_set_global_dict (host copy): the snapshot's dictionary
    std::vector<uint64_t> gd_msb, gd_lsb;
    std::vector<int32_t> gd_node;
    bool gd_set = false, gd_strict = false;
    uint64_t n_global = 0;
    bool global_ok = false;
    // node exchange (ad_exchange / ad_exchange_local): library-owned part buffers, RCCL communicator
    DevBuf xs_hdr, xs_keys, xs_ids, xs_k2t;    // this store's exported parts (grouped by owner)
    DevBuf xr_hdr, xr_keys, xr_ids, xr_k2t;    // parts received for the requests this store owns
    DevBuf xc_dev;                             // exchange table of the RCCL all-gather (+ own row, status words)
    uint64_t* h_xtab = nullptr;                // pinned host copy of the exchange table
    size_t h_xtab_words = 0;
    uint64_t xr_total[4] = {};
    ncclComm_t comm = nullptr;
    int comm_rank = 0, comm_world = 1;
    hipEvent_t x_ev[3] = {};                   // ad_exchange: step start, parts emitted, move done
    // execution levels (K5)
    LevelsWork* lv = nullptr;
    DevBuf g_em, g_el, g_en, g_kind, g_ko, g_k, g_do, g_d, g_out;
    // device-resident CommandsForKey maintenance (ad_cfk_update*): per-entry status, executeAt
    // rank and key index; host copies (cfk.status / cfk.exec / h_exec_rank) are refreshed from
    // them on demand (host_stale)
    DevBuf d_status, d_xrank, d_ekey;
    DevBuf d_ent2, d_status2, d_xrank2, d_ekey2;    // spare per-entry arrays (insertions)
    DevBuf d_dict_hi2, d_dict_lo2, d_dict_node2, d_dict_raw2;   // spare dictionary arrays (merges)
    bool host_moved = false;                         // entries were inserted on the device
    DevBuf u_k, u_tm, u_tl, u_tn, u_em, u_el, u_en, u_st, u_bm, u_bl, u_bn;
    DevBuf d_ballot, d_ballot2;                      // TxnInfo.ballot() per entry (Bal), when the store has any
    // TxnInfo.missing() on the device (CfkMiss): per entry its list (mref), the lists as rank CSR
    DevBuf d_mref, d_mref2, d_moff, d_moff2, d_mids, d_mids2;
    bool dmiss_on = false;                           // the device maintains them (ad_cfk_update with deps)
    uint64_t dmiss_lists = 0, dmiss_ids = 0;
    DevBuf u_do, u_dm, u_dl, u_dn;                   // staged deps of a host update batch
    CfkUpdWork* cu = nullptr;
    bool host_stale = false;
    // device ingest (ingest.hip): ad_cfk_load puts the snapshot's columns in HBM (raw_dev) and the
    // build derives everything there; the host's byId ids and dictionary copy follow on demand
    DevBuf d_in_seg, d_in_pruned, d_in_tm, d_in_tl, d_in_tn, d_in_em, d_in_el, d_in_en, d_in_xm, d_in_xl, d_in_xn, d_ing_rank;
    bool raw_dev = false;                            // d_in_* hold the loaded snapshot (no device update since)
    uint64_t raw_ne = 0;
    bool host_dict_stale = false;                    // dict_msb/lsb/node not yet read back from the device
    bool host_ingested = false;                      // host copies pending from a device ingest (entries did not move)
    IngestWork* ing = nullptr;
    std::vector<uint64_t> x_msb, x_lsb;        // ad_cfk_entries views
    std::vector<int32_t> x_node;
    std::vector<uint64_t> y_msb, y_lsb;        // ad_cfk_byid views
    std::vector<int32_t> y_node;
    std::vector<int64_t> y_pruned;
    std::vector<uint64_t> z_off;
    // LoadPruned requests of the last update batch (ad_cfk_load_pruned)
    std::vector<uint64_t> lp_upd, lp_msb, lp_lsb;
    std::vector<int64_t> lp_keys;
    std::vector<int32_t> lp_node;

    int fail(int code, const char* fmt, ...)
    {
        char buf[512];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof(buf), fmt, ap);
        va_end(ap);
        err = buf;
        return code;
    }
};

// A synchronous copy ordered after the work queued on the call's streams: the ctx streams are
// non-blocking, so a plain null-stream hipMemcpy would not wait for their kernels (nor they for it).
// Host memory goes through h2d / d2h (devmem.hpp: never a pageable HIP copy).
static hipError_t copy_sync(void* dst, const void* src, size_t bytes, hipMemcpyKind kind)
{
    dev_quiesce();
    const hipStream_t st = dev_scope_stream();
    const hipError_t e = kind == hipMemcpyHostToDevice   ? h2d(dst, src, bytes, st)
                         : kind == hipMemcpyDeviceToHost ? d2h(dst, src, bytes, st)
                                                         : hipMemcpyAsync(dst, src, bytes, kind, st);
    if (e != hipSuccess) return e;
    return st ? hipStreamSynchronize(st) : hipDeviceSynchronize();
}

#define HIPCHK(ctx, expr)                                                                         \
    do {                                                                                          \
        hipError_t _e = (expr);                                                                   \
        if (_e != hipSuccess) return (ctx)->fail(AD_E_DEVICE, "%s: %s", #expr, hipGetErrorString(_e)); \
    } while (0)

extern "C" {
// the device ingest reuses the update path's derived-array allocation (defined with the f1 entry points)
static int cfk_need_bufs(void* vc, uint64_t n_cand, uint64_t n_cwr, uint64_t n_w, CfkDerivedBufs* b);
}

namespace {

// ---------------------------------------------------------------------------------------
// ingest
// ---------------------------------------------------------------------------------------
struct DictRec {
    uint64_t hi, lo;
    int32_t node;
    uint32_t pad;
    uint64_t src;
};
static inline bool rec_less(const DictRec& a, const DictRec& b)
{
    if (a.hi != b.hi) return a.hi < b.hi;
    if (a.lo != b.lo) return a.lo < b.lo;
    return a.node < b.node;
}
static inline bool rec_eq(const DictRec& a, const DictRec& b) { return a.hi == b.hi && a.lo == b.lo && a.node == b.node; }

static bool tid_gt_none(const Tid& t)
{
    // compareTo(Timestamp.NONE) > 0, NONE = (0, 0, 0)
    const NormTid z = {0, 0, 0};
    return norm_cmp(norm(t), z) > 0;
}

template <class T>
static int upload(ad_ctx* c, DevBuf& b, const std::vector<T>& v)
{
    if (!b.ensure(sizeof(T) * std::max<size_t>(v.size(), 1))) return c->fail(AD_E_NOMEM, "hipMalloc %zu", sizeof(T) * v.size());
    if (!v.empty()) HIPCHK(c, h2d(b.p, v.data(), sizeof(T) * v.size(), c->stream));
    return 0;
}

static int sync_host(ad_ctx* c);

// uninstall the node-wide dictionary (a new snapshot, or ids it does not hold)
static void drop_global_dict(ad_ctx* c)
{
    c->gd_set = false;
    c->global_ok = false;
    std::vector<uint64_t>().swap(c->gd_msb);
    std::vector<uint64_t>().swap(c->gd_lsb);
    std::vector<int32_t>().swap(c->gd_node);
}

// The KeyLine perfect hash (hash and displace): every bucket gets the first displacement that puts
// all its keys on free lines, biggest buckets first; the table grows by half when a bucket does not
// fit. Keeps the host state (displacements, used lines, bucket members) for incremental placement.
static int kl_place_all(ad_ctx* c, const std::vector<int64_t>& keys, uint64_t nb, bool sparse)
{
    const uint64_t nk = keys.size();
    // a snapshot's table is 80 % full (the lean kernels' lines stay dense); once keys arrive through
    // updates it is rebuilt half full, where a bucket of ~4 keys is placed again in ~16 displacement
    // tries (kl_add_keys)
    uint64_t m = std::max<uint64_t>(1, sparse ? 2 * nk : nk + nk / 4);
    // the keys' second hashes grouped by bucket (counting sort), buckets by size, largest first
    // (stable: equal sizes in bucket order)
    std::vector<uint32_t> kb(nk), boff(nb + 1, 0);
    parallel_for(nk, [&](size_t a, size_t e) {
        for (size_t i = a; i < e; ++i) kb[i] = (uint32_t)kl_bucket(key_hash(keys[i]), nb);
    });
    for (uint64_t i = 0; i < nk; ++i) ++boff[kb[i] + 1];
    uint32_t max_sz = 0;
    for (uint64_t x = 0; x < nb; ++x) max_sz = std::max(max_sz, boff[x + 1]);
    for (uint64_t x = 0; x < nb; ++x) boff[x + 1] += boff[x];
    std::vector<uint64_t> hs(nk);
    {
        std::vector<uint32_t> cur(boff.begin(), boff.end() - 1);
        for (uint64_t i = 0; i < nk; ++i) hs[cur[kb[i]]++] = key_hash2(keys[i]);
    }
    std::vector<uint32_t> border;
    border.reserve(nb);
    {
        std::vector<uint32_t> by(max_sz + 2, 0);
        for (uint64_t x = 0; x < nb; ++x) ++by[max_sz - (boff[x + 1] - boff[x]) + 1];
        for (uint32_t z = 0; z <= max_sz; ++z) by[z + 1] += by[z];
        border.resize(nb);
        for (uint64_t x = 0; x < nb; ++x) border[by[max_sz - (boff[x + 1] - boff[x])]++] = (uint32_t)x;
    }
    std::vector<uint32_t> disp(nb, 0);
    std::vector<uint64_t> pos;
    for (int attempt = 0;; ++attempt)
    {
        std::vector<uint8_t> used(m, 0);
        bool ok = true;
        for (uint32_t bk : border)
        {
            const uint32_t lo = boff[bk], hi = boff[bk + 1];
            if (lo == hi) continue;
            uint32_t d = 0;
            for (;; ++d)
            {
                if (d == (1u << 22)) { ok = false; break; }
                pos.clear();
                bool fit = true;
                for (uint32_t i = lo; i < hi && fit; ++i)
                {
                    const uint64_t p = kl_index(hs[i], d, m);
                    if (used[p] || std::find(pos.begin(), pos.end(), p) != pos.end()) fit = false;
                    pos.push_back(p);
                }
                if (fit) break;
            }
            if (!ok) break;
            disp[bk] = d;
            for (uint64_t p : pos) used[p] = 1;
        }
        if (ok)
        {
            c->kl_used.swap(used);
            break;
        }
        if (attempt == 4) return AD_E_DEVICE;           // the caller reports it (this may run on a helper thread)
        m += m / 2;              // more room, try again
    }
    c->kline_slots = m;
    c->kl_nb_h = nb;
    c->kl_disp_h.swap(disp);
    // members per bucket, for new keys later (kl_add_keys): built on first use
    c->kl_members.clear();
    c->kl_keys_all = keys;
    return 0;
}

// the per-bucket members of the placed keys (kl_add_keys), from the keys the table was placed for
static void kl_members_ensure(ad_ctx* c)
{
    if (!c->kl_members.empty() || c->kl_keys_all.empty()) return;
    c->kl_members.assign(c->kl_nb_h, {});
    for (int64_t key : c->kl_keys_all) c->kl_members[kl_bucket(key_hash(key), c->kl_nb_h)].push_back(key);
    std::vector<int64_t>().swap(c->kl_keys_all);
}

// New keys into the perfect hash: a bucket keeps its displacement when its new keys land on free
// lines, else it is placed again (its old lines freed first); a bucket that does not fit, or a table
// above 70 % load, rebuilds the whole hash. Returns whether the table was rebuilt (size may change).
static int kl_add_keys(ad_ctx* c, const std::vector<int64_t>& nkeys, uint64_t nk_total, bool* need_rebuild)
{
    *need_rebuild = false;
    const uint64_t nb = c->kl_nb_h, m = c->kline_slots;
    if (nb == 0 || 10 * nk_total > 7 * m)
    {
        *need_rebuild = true;
        return 0;
    }
    kl_members_ensure(c);
    std::vector<std::pair<uint32_t, int64_t>> adds;
    adds.reserve(nkeys.size());
    for (int64_t key : nkeys) adds.push_back({(uint32_t)kl_bucket(key_hash(key), nb), key});
    std::sort(adds.begin(), adds.end());
    std::vector<uint64_t> pos;
    for (size_t i = 0; i < adds.size();)
    {
        const uint32_t b = adds[i].first;
        size_t j = i;
        while (j < adds.size() && adds[j].first == b) ++j;
        auto& mb = c->kl_members[b];
        const uint32_t d0 = c->kl_disp_h[b];
        // 1. the new keys on free lines under the bucket's displacement
        pos.clear();
        bool fit = true;
        for (size_t x = i; x < j && fit; ++x)
        {
            const uint64_t p = kl_index(key_hash2(adds[x].second), d0, m);
            if (c->kl_used[p] || std::find(pos.begin(), pos.end(), p) != pos.end()) fit = false;
            pos.push_back(p);
        }
        if (!fit)
        {
            // 2. place the bucket again
            for (int64_t key : mb) c->kl_used[kl_index(key_hash2(key), d0, m)] = 0;
            std::vector<int64_t> allb(mb);
            for (size_t x = i; x < j; ++x) allb.push_back(adds[x].second);
            uint32_t d = 0;
            for (;; ++d)
            {
                if (d == (1u << 20))
                {
                    *need_rebuild = true;
                    return 0;
                }
                pos.clear();
                fit = true;
                for (size_t x = 0; x < allb.size() && fit; ++x)
                {
                    const uint64_t p = kl_index(key_hash2(allb[x]), d, m);
                    if (c->kl_used[p] || std::find(pos.begin(), pos.end(), p) != pos.end()) fit = false;
                    pos.push_back(p);
                }
                if (fit) break;
            }
            c->kl_disp_h[b] = d;
        }
        for (uint64_t p : pos) c->kl_used[p] = 1;
        for (size_t x = i; x < j; ++x) mb.push_back(adds[x].second);
        i = j;
    }
    return 0;
}

// Range commands and RedundantBefore of a snapshot build (both routes): (range, command) entries
// sorted by (start, end, txnId), the range table, the stabbing index, uploads. cmd_rank / wm_rank:
// the dictionary ranks of the commands' txnIds and the watermarks (0: none).
struct RangePart {
    std::vector<int64_t> cell_E;
    bool cell_ok = false;
    uint64_t n_rent = 0;
};
static int build_ranges(ad_ctx* c, const std::vector<uint32_t>& cmd_rank, const std::vector<uint32_t>& wm_rank, RangePart* out)
{
    const uint64_t ncmd = c->cmds.txn.size(), nrb = c->rb.wm.size();
    struct REnt { int64_t s, e; uint32_t txw; uint32_t rid; uint8_t live; };
    std::vector<int64_t>& cell_E = out->cell_E;
    bool& cell_ok = out->cell_ok;
    std::vector<REnt> rent;
    for (uint64_t i = 0; i < ncmd; ++i)
    {
        const bool hist = !c->cmds.historical.empty() && c->cmds.historical[i];
        if (!hist && !c->cmds.erased.empty() && c->cmds.erased[i]) continue;   // saveStatus >= Erased, :897 (historical: no status)
        const uint32_t kind = (uint32_t)((c->cmds.txn[i].lsb >> 1) & 7);
        if ((c->cmds.txn[i].lsb & 1) == 0) return c->fail(AD_E_INVAL, "range command %llu has a key-domain TxnId", (unsigned long long)i);
        const bool live = !hist && (c->cmds.erased.empty() || !c->cmds.erased[i]);     // rangeCommands, not erased
        for (uint64_t r = c->cmds.off[i]; r < c->cmds.off[i + 1]; ++r)
            rent.push_back({c->cmds.start[r], c->cmds.end[r], cmd_rank[i] | (kind << RANK_BITS), 0, (uint8_t)live});
    }
    for (uint64_t i = 0; i < nrb; ++i)
        if (i > 0 && c->rb.start[i] <= c->rb.start[i - 1]) return c->fail(AD_E_INVAL, "redundantBefore entries not ascending");
    {
        std::vector<std::pair<int64_t, int64_t>> rt;
        rt.reserve(rent.size() + nrb);
        for (auto& r : rent) rt.push_back({r.s, r.e});
        for (uint64_t i = 0; i < nrb; ++i) rt.push_back({c->rb.start[i], c->rb.end[i]});
        std::sort(rt.begin(), rt.end());
        rt.erase(std::unique(rt.begin(), rt.end()), rt.end());
        c->rt_start.resize(rt.size());
        c->rt_end.resize(rt.size());
        for (size_t i = 0; i < rt.size(); ++i) { c->rt_start[i] = rt[i].first; c->rt_end[i] = rt[i].second; }
        auto rid_of = [&](int64_t s, int64_t e) -> uint32_t {
            return (uint32_t)(std::lower_bound(rt.begin(), rt.end(), std::make_pair(s, e)) - rt.begin());
        };
        for (auto& r : rent) r.rid = rid_of(r.s, r.e);
        std::sort(rent.begin(), rent.end(), [](const REnt& a, const REnt& b) {
            if (a.rid != b.rid) return a.rid < b.rid;
            return (a.txw & RANK_MASK) < (b.txw & RANK_MASK);
        });
        {
            // one entry per (range, txnId); live if a live command contributed it
            size_t o = 0;
            for (size_t i = 0; i < rent.size(); ++i)
            {
                if (o > 0 && rent[o - 1].rid == rent[i].rid && (rent[o - 1].txw & RANK_MASK) == (rent[i].txw & RANK_MASK))
                    rent[o - 1].live |= rent[i].live;
                else
                    rent[o++] = rent[i];
            }
            rent.resize(o);
        }
        std::vector<uint32_t> rb_rid(nrb);
        for (uint64_t i = 0; i < nrb; ++i) rb_rid[i] = rid_of(c->rb.start[i], c->rb.end[i]);
        // padded to whole 64-entry frames: the fused kernel reads frames with vector loads
        const size_t rpad = (rent.size() + 63) / 64 * 64;
        std::vector<int64_t> rs(rpad, INT64_MAX), re(rpad, INT64_MIN);
        std::vector<uint32_t> rtxw(rpad, 0), rrid(rpad, 0);
        for (size_t i = 0; i < rent.size(); ++i) { rs[i] = rent[i].s; re[i] = rent[i].e; rtxw[i] = rent[i].txw; rrid[i] = rent[i].rid; }
        c->h_rtxw.assign(rtxw.begin(), rtxw.begin() + rent.size());
        c->h_rlive.resize(rent.size());
        for (size_t i = 0; i < rent.size(); ++i) c->h_rlive[i] = rent[i].live;
        for (uint64_t i = 0; i < nrb; ++i)
            if (wm_rank[i] && (c->rb.wm[i].lsb & 1) == 0) return c->fail(AD_E_INVAL, "redundantBefore watermark must be range-domain");
        int rc;
        if ((rc = upload(c, c->d_rstart, rs)) || (rc = upload(c, c->d_rend, re)) || (rc = upload(c, c->d_rtxw, rtxw)) ||
            (rc = upload(c, c->d_rrid, rrid)) || (rc = upload(c, c->d_rb_s, c->rb.start)) || (rc = upload(c, c->d_rb_e, c->rb.end)) ||
            (rc = upload(c, c->d_rb_e0, c->rb.e0)) || (rc = upload(c, c->d_rb_e1, c->rb.e1)) || (rc = upload(c, c->d_rb_wm, wm_rank)) ||
            (rc = upload(c, c->d_rb_rid, rb_rid)))
            return rc;

        // Stabbing index of the range entries (the role of SearchableRangeList /
        // CheckpointIntervalArray, CheckpointIntervalArray.java:101-249): the distinct endpoints cut
        // the key line into cells; cell(x) = #endpoints < x (EndInclusive) or <= x (StartInclusive),
        // and every entry covers a contiguous run of cells [cell(start) + 1, cell(end)], with
        // `cell` the endpoint's index. Each cell lists the (range id, txw) of the entries covering
        // it, in entry order = (Range.compare, TxnId) order. Skipped when the total coverage is
        // too large (deeply nested ranges): the max-end tree then serves every probe.
        cell_E.clear();
        cell_ok = false;
        if (!rent.empty())
        {
            for (auto& r : rent) { cell_E.push_back(r.s); cell_E.push_back(r.e); }
            std::sort(cell_E.begin(), cell_E.end());
            cell_E.erase(std::unique(cell_E.begin(), cell_E.end()), cell_E.end());
            const size_t m = cell_E.size();
            auto idx = [&](int64_t v) { return (size_t)(std::lower_bound(cell_E.begin(), cell_E.end(), v) - cell_E.begin()); };
            std::vector<uint64_t> cnt(m + 2, 0);
            uint64_t total = 0;
            std::vector<std::pair<uint32_t, uint32_t>> span(rent.size());
            for (size_t i = 0; i < rent.size(); ++i)
            {
                const uint32_t a = (uint32_t)idx(rent[i].s) + 1, b = (uint32_t)idx(rent[i].e);
                span[i] = {a, b};
                if (b >= a) { cnt[a] += 1; cnt[b + 1] -= 1; total += b - a + 1; }
            }
            uint64_t budget = std::max<uint64_t>(64ull << 20, 32 * (uint64_t)rent.size());
            if (const char* e = getenv("AD_CELL_BUDGET")) budget = strtoull(e, nullptr, 10);   // tests: force the tree
            if (total <= budget && total < (1ull << 32))
            {
                std::vector<uint32_t> off(m + 2, 0);
                uint64_t run = 0, acc = 0;
                for (size_t cl = 0; cl <= m; ++cl)
                {
                    run += cnt[cl];
                    off[cl] = (uint32_t)acc;
                    acc += run;
                }
                off[m + 1] = (uint32_t)acc;
                std::vector<uint64_t> ents(std::max<uint64_t>(acc, 1));
                std::vector<uint32_t> cur(off.begin(), off.end());
                for (size_t i = 0; i < rent.size(); ++i)
                    for (uint32_t cl = span[i].first; cl <= span[i].second && span[i].second >= span[i].first; ++cl)
                        ents[cur[cl]++] = ((uint64_t)rent[i].rid << 32) | rent[i].txw;
                if ((rc = upload(c, c->d_cell_E, cell_E)) || (rc = upload(c, c->d_cell_off, off)) ||
                    (rc = upload(c, c->d_cell_ent, ents)))
                    return rc;
                cell_ok = true;
                c->n_cell_ent = acc;
            }
        }
    }

    out->n_rent = rent.size();
    return 0;
}

// The DevSnapshot views over the ctx's device buffers of a built snapshot (both build routes)
static int set_views(ad_ctx* c, uint64_t n_dict, uint64_t n_samp, const NormTid& last, uint64_t nk, uint64_t ne, uint64_t hcap,
                     const RangePart& rp, uint64_t nrb)
{
    DevSnapshot& s = c->ds;
    s = DevSnapshot{};
    s.dict_hi = c->d_dict_hi.as<uint64_t>();
    s.dict_lo = c->d_dict_lo.as<uint64_t>();
    s.dict_node = c->d_dict_node.as<int32_t>();
    s.n_dict = n_dict;
    s.ds_hi = c->d_ds_hi.as<uint64_t>();
    s.ds_lo = c->d_ds_lo.as<uint64_t>();
    s.ds_node = c->d_ds_node.as<int32_t>();
    s.n_samp = n_samp;
    s.n_samp2 = n_samp ? dict_samples2(n_dict) : 0;    // both build routes fill the second level
    if (n_dict)
    {
        s.dict_last_hi = last.hi;
        s.dict_last_lo = last.lo;
        s.dict_last_node = last.node;
    }
    s.n_keys = nk;
    s.keys = c->d_keys.as<int64_t>();
    s.krec = c->d_krec.as<KeyRec>();
    s.khash = c->d_khash.as<KeySlot>();
    s.kent = c->d_kent.as<KeyEntry>();
    s.cand = c->d_cand.as<uint32_t>();
    s.cwr = c->d_cwr.as<uint32_t>();
    s.khash_mask = hcap - 1;
    s.n_ent = ne;
    s.ent = c->d_ent.as<uint2>();
    s.w = c->d_w.as<uint2>();
    s.lvl_n[0] = ne;
    int L = 1;
    while (s.lvl_n[L - 1] > 64 && L < MAX_LEVELS)
    {
        s.lvl_n[L] = (s.lvl_n[L - 1] + 63) / 64;
        ++L;
    }
    s.n_levels = L;
    for (int l = 1; l < L; ++l)
        for (int cl = 0; cl < NCLASS; ++cl)
        {
            if (!c->d_lvl[cl][l].ensure(sizeof(uint32_t) * ((s.lvl_n[l] + 63) / 64 * 64))) return c->fail(AD_E_NOMEM, "tree level");
            s.lvl[cl][l] = c->d_lvl[cl][l].as<uint32_t>();
        }
    const bool cell_ok = rp.cell_ok;
    s.n_rent = rp.n_rent;
    s.n_cell_E = cell_ok ? rp.cell_E.size() : 0;
    s.cell_E = cell_ok ? c->d_cell_E.as<int64_t>() : nullptr;
    s.cell_off = cell_ok ? c->d_cell_off.as<uint32_t>() : nullptr;
    s.cell_ent = cell_ok ? c->d_cell_ent.as<uint64_t>() : nullptr;
    if (!cell_ok) c->n_cell_ent = 0;
    s.r_start = c->d_rstart.as<int64_t>();
    s.r_end = c->d_rend.as<int64_t>();
    s.r_txw = c->d_rtxw.as<uint32_t>();
    s.r_rid = c->d_rrid.as<uint32_t>();
    s.rlvl_n[0] = s.n_rent;
    L = 1;
    while (s.rlvl_n[L - 1] > 64 && L < MAX_LEVELS)
    {
        s.rlvl_n[L] = (s.rlvl_n[L - 1] + 63) / 64;
        ++L;
    }
    s.n_rlevels = L;
    for (int l = 1; l < L; ++l)
        for (int cl = 0; cl < NCLASS; ++cl)
        {
            if (!c->d_rlvl[cl][l].ensure(sizeof(int64_t) * ((s.rlvl_n[l] + 63) / 64 * 64))) return c->fail(AD_E_NOMEM, "range tree level");
            s.rlvl[cl][l] = c->d_rlvl[cl][l].as<int64_t>();
        }
    s.n_rb = nrb;
    s.rb_start = c->d_rb_s.as<int64_t>();
    s.rb_end = c->d_rb_e.as<int64_t>();
    s.rb_e0 = c->d_rb_e0.as<int64_t>();
    s.rb_e1 = c->d_rb_e1.as<int64_t>();
    s.rb_wm = c->d_rb_wm.as<uint32_t>();
    s.rb_rid = c->d_rb_rid.as<uint32_t>();
    s.n_slices = c->slice_s.size();
    s.slice_start = c->d_slices_s.as<int64_t>();
    s.slice_end = c->d_slices_e.as<int64_t>();
    s.start_inclusive = c->cfg.range_start_inclusive;
    s.elide = c->cfg.elide;
    s.rng32 = getenv("AD_RNG64") == nullptr && c->rt_start.size() < (1ull << 26) && 2 * n_dict + 2 < (1ull << 26);
    return 0;
}

// ---- the snapshot built on the device (ingest.hip + the update path's derivation) ----------------
static int host_inputs(ad_ctx* c);
static int build_snapshot_device(ad_ctx* c)
{
    const double t0 = now_ms();
    const bool trace = getenv("AD_INGEST_TRACE") != nullptr;
    double tp = t0;
    auto phase = [&](const char* what) {
        if (!trace) return;
        const double t = now_ms();
        fprintf(stderr, "ingest(device) %-28s %8.1f ms\n", what, t - tp);
        tp = t;
    };
    auto& K = c->cfk;
    const uint64_t nk = K.keys.size(), ne = c->raw_ne, ncmd = c->cmds.txn.size(), nrb = c->rb.wm.size();
    hipStream_t st = c->stream;
    c->dmiss_on = false;
    // extra dictionary ids: range command txnIds, then the watermarks above NONE
    std::vector<uint64_t> xm, xl, wm_at;
    std::vector<int32_t> xn;
    for (uint64_t i = 0; i < ncmd; ++i) { xm.push_back(c->cmds.txn[i].msb); xl.push_back(c->cmds.txn[i].lsb); xn.push_back(c->cmds.txn[i].node); }
    for (uint64_t i = 0; i < nrb; ++i)
        if (tid_gt_none(c->rb.wm[i]))
        {
            xm.push_back(c->rb.wm[i].msb);
            xl.push_back(c->rb.wm[i].lsb);
            xn.push_back(c->rb.wm[i].node);
            wm_at.push_back(i);
        }
    const uint64_t nx = xm.size();
    int rc;
    if ((rc = upload(c, c->d_in_xm, xm)) || (rc = upload(c, c->d_in_xl, xl)) || (rc = upload(c, c->d_in_xn, xn))) return rc;
    IngestIn in{nk, ne, nx, c->d_keys.as<int64_t>(), c->d_in_seg.as<uint64_t>(),
                K.pruned.empty() ? nullptr : c->d_in_pruned.as<int64_t>(),
                c->d_in_tm.as<uint64_t>(), c->d_in_tl.as<uint64_t>(), c->d_in_tn.as<int32_t>(),
                c->d_in_em.as<uint64_t>(), c->d_in_el.as<uint64_t>(), c->d_in_en.as<int32_t>(), c->d_status.as<uint8_t>(),
                c->d_in_xm.as<uint64_t>(), c->d_in_xl.as<uint64_t>(), c->d_in_xn.as<int32_t>()};
    const uint64_t nrec = std::max<uint64_t>(ingest_records(in), 1);
    const uint64_t padded = std::max<uint64_t>(64, (ne + 63) / 64 * 64);     // whole 64-entry frames (tau 0)
    if (!c->d_dict_hi.ensure(8 * nrec) || !c->d_dict_lo.ensure(8 * nrec) || !c->d_dict_node.ensure(4 * nrec) ||
        !c->d_dict_lsb_raw.ensure(8 * nrec) || !c->d_ing_rank.ensure(4 * nrec) || !c->d_ent.ensure(8 * padded) ||
        !c->d_xrank.ensure(4 * std::max<uint64_t>(ne, 1)) || !c->d_ekey.ensure(4 * std::max<uint64_t>(ne, 1)) ||
        !c->d_krec.ensure(sizeof(KeyRec) * std::max<uint64_t>(nk, 1)) || !c->d_kent.ensure(sizeof(KeyEntry) * std::max<uint64_t>(nk, 1)))
        return c->fail(AD_E_NOMEM, "snapshot buffers");
    HIPCHK(c, hipMemsetAsync(c->d_ent.as<uint2>() + ne, 0, 8 * (padded - ne), st));
    IngestOut o{c->d_dict_hi.as<uint64_t>(), c->d_dict_lo.as<uint64_t>(), c->d_dict_node.as<int32_t>(),
                c->d_dict_lsb_raw.as<uint64_t>(), c->d_ing_rank.as<uint32_t>(), c->d_ent.as<uint2>(),
                c->d_xrank.as<uint32_t>(), c->d_ekey.as<uint32_t>(), c->d_krec.as<KeyRec>(), 0};
    if (!c->ing) c->ing = ingest_work_create();
    uint64_t n_dict = 0, bad = 0;
    std::string e;
    // the KeyLine perfect hash is placed on a host thread (keys only) while the device builds the
    // dictionary and the entries
    // The thread reads only the loaded keys (const) and writes only the ctx's KeyLine host state
    // (kl_used, kline_slots, kl_nb_h, kl_disp_h, kl_members, kl_keys_all), which nothing else touches
    // before the join below; it makes no HIP call and reports failure through kl_rc (not c->err).
    const uint64_t kl_nb = std::max<uint64_t>(1, nk / 4);
    int kl_rc = 0;
    std::thread kl_thread([&]() { kl_rc = kl_place_all(c, K.keys, kl_nb, false); });
    struct Joiner {
        std::thread& t;
        ~Joiner() { if (t.joinable()) t.join(); }
    } kl_join{kl_thread};
    phase("columns");
    if ((rc = ingest_dictionary(c->ing, in, o, st, &n_dict, &bad, &e)))
        return c->fail(rc, "%s", e.c_str());
    if (n_dict > MAX_DICT) return c->fail(AD_E_CAPACITY, "more than %llu distinct ids", (unsigned long long)MAX_DICT);
    phase("dictionary");
    if ((rc = ingest_entries(c->ing, in, o, st, &bad, &e)))
    {
        const long long key = bad < nk ? (long long)K.keys[bad] : -1;
        if (rc == AD_E_STATE) return c->fail(AD_E_INVAL, "prunedBefore of key %lld is not in byId", key);
        if (rc == AD_E_ORDER) return c->fail(rc, "CommandsForKey of key %lld violates byId strict order (CommandsForKey.java:1438)", key);
        return c->fail(rc, "CommandsForKey of key %lld violates status range / key-domain ids / keys ascending", key);
    }
    phase("entries");
    // the extras' ranks (range commands, watermarks) for the host's range part
    std::vector<uint32_t> xr(nx), cmd_rank(ncmd), wm_rank(nrb, 0);
    if (nx) HIPCHK(c, copy_sync(xr.data(), c->d_ing_rank.as<uint32_t>() + ne + o.n_diff, 4 * nx, hipMemcpyDeviceToHost));
    for (uint64_t i = 0; i < ncmd; ++i) cmd_rank[i] = xr[i];
    for (uint64_t j = 0; j < wm_at.size(); ++j) wm_rank[wm_at[j]] = xr[ncmd + j];
    c->h_cmd_rank = cmd_rank;
    RangePart rp;
    if ((rc = build_ranges(c, cmd_rank, wm_rank, &rp))) return rc;
    phase("range commands");
    // keys: the KeyLine perfect hash placed on the host (keys only), then on the device every key's
    // line (k_key_slots), stabbing cell and slot of the open-addressing key hash
    uint64_t hcap = 16;
    while (hcap < 2 * nk) hcap <<= 1;
    kl_thread.join();
    if (kl_rc) return c->fail(kl_rc, "key perfect hash did not converge");
    phase("key line perfect hash (wait)");
    if ((rc = upload(c, c->d_kl_disp, c->kl_disp_h)) || (rc = upload(c, c->d_slices_s, c->slice_s)) ||
        (rc = upload(c, c->d_slices_e, c->slice_e)) || (rc = upload(c, c->d_rt_start, c->rt_start)) ||
        (rc = upload(c, c->d_rt_end, c->rt_end)))
        return rc;
    if (!c->d_khash.ensure(sizeof(KeySlot) * hcap) || !c->d_kslot.ensure(4 * std::max<uint64_t>(nk, 1)) ||
        !c->d_kcell.ensure(4 * std::max<uint64_t>(nk, 1)))
        return c->fail(AD_E_NOMEM, "key tables");
    HIPCHK(c, run_key_slots(c->d_keys.as<int64_t>(), nk, c->d_kl_disp.as<uint32_t>(), kl_nb, c->kline_slots,
                            c->d_kslot.as<uint32_t>(), st));
    HIPCHK(c, ingest_keys(c->d_keys.as<int64_t>(), nk, rp.cell_ok ? c->d_cell_E.as<int64_t>() : nullptr,
                          rp.cell_ok ? rp.cell_E.size() : 0, c->cfg.range_start_inclusive, c->d_kcell.as<uint32_t>(),
                          c->d_khash.as<KeySlot>(), hcap, st));
    if (!K.ballot.empty())
    {
        std::vector<Bal> bl(ne);
        for (uint64_t i = 0; i < ne; ++i) bl[i] = Bal{K.ballot[i].msb, K.ballot[i].lsb, K.ballot[i].node, 0};
        if ((rc = upload(c, c->d_ballot, bl))) return rc;
    }
    else
        c->d_ballot.release();
    phase("keys");
    // views, the sampled dictionary, the derivation (cand / cwr / w, KeyEntry, trees)
    const uint64_t n_samp = dict_samples(n_dict), n_sent = std::max<uint64_t>(dict_sample_entries(n_dict), 1);
    if (!c->d_ds_hi.ensure(8 * n_sent) || !c->d_ds_lo.ensure(8 * n_sent) || !c->d_ds_node.ensure(4 * n_sent))
        return c->fail(AD_E_NOMEM, "dictionary sample");
    NormTid last{0, 0, 0};
    if (n_dict)
    {
        HIPCHK(c, copy_sync(&last.hi, c->d_dict_hi.as<uint64_t>() + n_dict - 1, 8, hipMemcpyDeviceToHost));
        HIPCHK(c, copy_sync(&last.lo, c->d_dict_lo.as<uint64_t>() + n_dict - 1, 8, hipMemcpyDeviceToHost));
        HIPCHK(c, copy_sync(&last.node, c->d_dict_node.as<int32_t>() + n_dict - 1, 4, hipMemcpyDeviceToHost));
    }
    if ((rc = set_views(c, n_dict, n_samp, last, nk, ne, hcap, rp, nrb))) return rc;
    if (n_samp) HIPCHK(c, run_dict_sample(c->ds, c->d_ds_hi.as<uint64_t>(), c->d_ds_lo.as<uint64_t>(), c->d_ds_node.as<int32_t>(), st));
    if (!c->cu) c->cu = cfk_upd_work_create();
    CfkDevState d{c->d_status.as<uint8_t>(), c->d_xrank.as<uint32_t>(), c->d_ekey.as<uint32_t>(),
                  c->d_dict_lsb_raw.as<uint64_t>(), c->d_ballot.p ? c->d_ballot.as<Bal>() : nullptr, nullptr,
                  c->d_ent.as<uint2>(), c->d_krec.as<KeyRec>(), c->d_kent.as<KeyEntry>()};
    CfkDerivedBufs b{c->d_cand.as<uint32_t>(), c->d_cand.cap / 4, c->d_cwr.as<uint32_t>(), c->d_cwr.cap / 4,
                     c->d_w.as<uint2>(), c->d_w.cap / 8};
    uint64_t bad_e = 0;
    if ((rc = run_cfk_derive_full(c->cu, c->ds, d, &b, cfk_need_bufs, c, st, &bad_e, &e)))
    {
        if (rc == AD_E_DUP_EXEC)
        {
            uint32_t k = 0;
            if (bad_e < ne) (void)copy_sync(&k, c->d_ekey.as<uint32_t>() + bad_e, 4, hipMemcpyDeviceToHost);
            return c->fail(rc, "CommandsForKey of key %lld violates unique committed executeAt (CommandsForKey.java:1439)",
                           k < nk ? (long long)K.keys[k] : -1ll);
        }
        return c->fail(rc, "%s", e.c_str());
    }
    phase("derivation + trees");
    DevSnapshot& s = c->ds;
    HIPCHK(c, build_range_trees(s, st));
    if (!c->d_kline.ensure(kline_table_bytes(c->kline_slots))) return c->fail(AD_E_NOMEM, "key lines");
    s.kline = c->d_kline.as<KeyLine>();
    s.kl_lines = c->kline_slots;
    s.kquad = kline_quads(s.kline, c->kline_slots);
    s.kl_buckets = kl_nb;
    s.kl_disp = c->d_kl_disp.as<uint32_t>();
    HIPCHK(c, run_build_klines(s, c->d_kslot.as<uint32_t>(), c->d_kcell.as<uint32_t>(), c->d_kline.as<KeyLine>(),
                               c->kline_slots, st));
    HIPCHK(c, hipStreamSynchronize(st));
    phase("range trees + key lines");
    // the raw columns are consumed; the host's copies (byId ids, ranks, dictionary) follow on demand
    c->raw_dev = false;
    for (DevBuf* bb : {&c->d_in_tm, &c->d_in_tl, &c->d_in_tn, &c->d_in_em, &c->d_in_el, &c->d_in_en}) bb->release();
    c->dict_msb.clear();
    c->dict_lsb.clear();
    c->dict_node.clear();
    c->h_txn_rank.clear();
    c->h_exec_rank.clear();
    c->h_pruned.assign(nk, 0);
    K.txn.clear();
    K.exec.clear();
    c->host_dict_stale = true;
    c->host_stale = true;
    c->host_moved = true;
    c->host_ingested = true;
    c->dirty = false;
    ++c->snap_gen;
    ++c->rank_gen;
    // the update path's state between batches (incremental committed order, per-entry change flags)
    // starts afresh, as after a host build
    cfk_upd_work_invalidate(c->cu);
    c->global_ok = false;
    c->n_global = 0;
    c->ms_ingest = now_ms() - t0;
    return 0;
}

static int build_snapshot_host(ad_ctx* c);
static int build_snapshot(ad_ctx* c)
{
    // the device route takes a snapshot whose columns the load put in HBM, unless a node-wide
    // dictionary is installed (its ranks are the installed dictionary's: the host route)
    if (c->raw_dev && !c->gd_set) return build_snapshot_device(c);
    if (int rc = host_inputs(c)) return rc;
    c->raw_dev = false;
    return build_snapshot_host(c);
}

static int build_snapshot_host(ad_ctx* c)
{
    if (int rc0 = sync_host(c)) return rc0;
    c->dmiss_on = false;          // the host copy holds the missing() lists now; uploaded again on demand
    const double t0 = now_ms();
    const bool trace = getenv("AD_INGEST_TRACE") != nullptr;
    double tp = t0;
    auto phase = [&](const char* what) {
        if (!trace) return;
        const double t = now_ms();
        fprintf(stderr, "ingest %-28s %8.1f ms\n", what, t - tp);
        tp = t;
    };
    auto& K = c->cfk;
    const uint64_t nk = K.keys.size(), ne = K.status.size();
    const uint64_t ncmd = c->cmds.txn.size(), nrb = c->rb.wm.size();

    // ---- 1. id dictionary over every id the kernels compare
    std::vector<uint8_t> exec_differs(ne);
    std::vector<DictRec> recs;
    recs.reserve(ne * 2 + ncmd + nrb);
    for (uint64_t e = 0; e < ne; ++e)
    {
        const NormTid n = norm(K.txn[e]);
        recs.push_back({n.hi, n.lo, n.node, 0, e});
        const Tid& x = K.exec[e];
        exec_differs[e] = !(x.msb == K.txn[e].msb && x.lsb == K.txn[e].lsb && x.node == K.txn[e].node);
        if (exec_differs[e])
        {
            const NormTid m = norm(x);
            recs.push_back({m.hi, m.lo, m.node, 0, ne + e});
        }
    }
    for (uint64_t i = 0; i < ncmd; ++i)
    {
        const NormTid n = norm(c->cmds.txn[i]);
        recs.push_back({n.hi, n.lo, n.node, 0, 2 * ne + i});
    }
    for (uint64_t i = 0; i < nrb; ++i)
    {
        if (!tid_gt_none(c->rb.wm[i])) continue;
        const NormTid n = norm(c->rb.wm[i]);
        recs.push_back({n.hi, n.lo, n.node, 0, 2 * ne + ncmd + i});
    }
    phase("dictionary records");
    parallel_sort(recs, rec_less);
    phase("dictionary sort");
    auto src_tid = [&](uint64_t s) -> const Tid& {
        if (s < ne) return K.txn[s];
        if (s < 2 * ne) return K.exec[s - ne];
        if (s < 2 * ne + ncmd) return c->cmds.txn[s - 2 * ne];
        return c->rb.wm[s - 2 * ne - ncmd];
    };
    std::vector<uint32_t> txn_rank(ne), exec_rank(ne), cmd_rank(ncmd), wm_rank(nrb, 0);
    c->dict_msb.clear();
    c->dict_lsb.clear();
    c->dict_node.clear();
    std::vector<uint64_t> dhi, dlo;
    std::vector<int32_t> dnode;
    auto set_rank = [&](uint64_t s, uint32_t rank) {
        if (s < ne) txn_rank[s] = rank;
        else if (s < 2 * ne) exec_rank[s - ne] = rank;
        else if (s < 2 * ne + ncmd) cmd_rank[s - 2 * ne] = rank;
        else wm_rank[s - 2 * ne - ncmd] = rank;
    };
    bool use_global = c->gd_set;
    if (use_global)
    {
        // the installed node-wide dictionary (ad_set_global_dict) is this store's dictionary: every
        // rank is a global rank, so exported parts carry the kernels' own ids (no translation)
        const uint64_t ng = c->gd_msb.size();
        dhi.resize(ng);
        dlo.resize(ng);
        dnode.resize(ng);
        parallel_for(ng, [&](size_t a, size_t b) {
            for (size_t i = a; i < b; ++i)
            {
                const NormTid n = norm(Tid{c->gd_msb[i], c->gd_lsb[i], c->gd_node[i]});
                dhi[i] = n.hi;
                dlo[i] = n.lo;
                dnode[i] = n.node;
            }
        });
        uint64_t gi = 0;
        for (size_t i = 0; i < recs.size() && use_global; ++i)
        {
            const DictRec& r = recs[i];
            auto g_less = [&](uint64_t j) {
                if (dhi[j] != r.hi) return dhi[j] < r.hi;
                if (dlo[j] != r.lo) return dlo[j] < r.lo;
                return dnode[j] < r.node;
            };
            while (gi < ng && g_less(gi)) ++gi;
            if (gi == ng || dhi[gi] != r.hi || dlo[gi] != r.lo || dnode[gi] != r.node)
            {
                use_global = false;
                break;
            }
            const Tid& t = src_tid(r.src);
            if (t.lsb != c->gd_lsb[gi])
                return c->fail(AD_E_INCONSISTENT_ID, "ids equal under Timestamp.equals differ in flag bits (lsb %llx vs %llx)",
                               (unsigned long long)t.lsb, (unsigned long long)c->gd_lsb[gi]);
            set_rank(r.src, (uint32_t)(2 * gi + 1));
        }
        if (use_global)
        {
            if (ng > MAX_DICT) return c->fail(AD_E_CAPACITY, "more than %llu distinct ids", (unsigned long long)MAX_DICT);
            c->dict_msb = c->gd_msb;
            c->dict_lsb = c->gd_lsb;
            c->dict_node = c->gd_node;
        }
        else
        {
            if (c->gd_strict) return c->fail(AD_E_INVAL, "ad_set_global_dict: an id of this store's snapshot is missing");
            // the snapshot outgrew the installed dictionary: uninstalled, the store's own dictionary instead
            drop_global_dict(c);
            dhi.clear();
            dlo.clear();
            dnode.clear();
        }
    }
    for (size_t i = 0; i < recs.size() && !use_global; ++i)
    {
        const DictRec& r = recs[i];
        if (i == 0 || !rec_eq(recs[i - 1], r))
        {
            if (c->dict_msb.size() >= MAX_DICT) return c->fail(AD_E_CAPACITY, "more than %llu distinct ids", (unsigned long long)MAX_DICT);
            const Tid& t = src_tid(r.src);
            c->dict_msb.push_back(t.msb);
            c->dict_lsb.push_back(t.lsb);
            c->dict_node.push_back(t.node);
            dhi.push_back(r.hi);
            dlo.push_back(r.lo);
            dnode.push_back(r.node);
        }
        else
        {
            const Tid& t = src_tid(r.src);
            if (t.lsb != c->dict_lsb.back())
                return c->fail(AD_E_INCONSISTENT_ID, "ids equal under Timestamp.equals differ in flag bits (lsb %llx vs %llx)",
                               (unsigned long long)t.lsb, (unsigned long long)c->dict_lsb.back());
        }
        set_rank(r.src, (uint32_t)(2 * (c->dict_msb.size() - 1) + 1));
    }
    std::vector<DictRec>().swap(recs);
    for (uint64_t e = 0; e < ne; ++e)
        if (!exec_differs[e]) exec_rank[e] = txn_rank[e];
    c->h_cmd_rank = cmd_rank;
    phase("dictionary + ranks");

    // ---- 2. per key validation, tau/txw, committed Writes by executeAt
    std::vector<uint2> ent(ne);
    std::vector<uint32_t> seg32(nk + 1), woff(nk + 1), pruned(nk, 0);
    std::vector<int32_t> maw(nk, -1);
    for (uint64_t k = 0; k <= nk; ++k) seg32[k] = (uint32_t)K.seg[k];
    std::atomic<int> bad{0};
    std::atomic<uint64_t> bad_key{0};
    std::vector<uint32_t> wcount(nk, 0);
    parallel_for(nk, [&](size_t ka, size_t kb) {
        std::vector<uint32_t> ce;
        for (size_t k = ka; k < kb; ++k)
        {
            const uint64_t s0 = K.seg[k], s1 = K.seg[k + 1];
            ce.clear();
            uint32_t nw = 0;
            for (uint64_t e = s0; e < s1; ++e)
            {
                const uint8_t st = K.status[e];
                const uint32_t kind = (uint32_t)((K.txn[e].lsb >> 1) & 7);
                const uint32_t dom = (uint32_t)(K.txn[e].lsb & 1);
                if (st > 7) { bad = AD_E_INVAL; bad_key = k; continue; }
                if (e > s0 && txn_rank[e] <= txn_rank[e - 1]) { bad = AD_E_ORDER; bad_key = k; }
                uint32_t tau;
                if (st == AD_ST_TRANSITIVELY_KNOWN || st == AD_ST_INVALID_OR_TRUNCATED_OR_UNMANAGED_COMMITTED) tau = 0;
                else if (st >= AD_ST_COMMITTED && ((KINDS_RS_OR_WS >> kind) & 1)) tau = exec_rank[e];
                else tau = TAU_NEVER_ELIDED;
                if (tau != 0 && dom != 0) { bad = AD_E_INVAL; bad_key = k; }   // live range-domain id in a CFK
                ent[e] = make_uint2(tau, txn_rank[e] | (kind << RANK_BITS));
                if (st >= AD_ST_COMMITTED && st <= AD_ST_APPLIED)
                {
                    ce.push_back(exec_rank[e]);
                    if (kind == AD_KIND_WRITE) ++nw;
                }
            }
            std::sort(ce.begin(), ce.end());
            for (size_t i = 1; i < ce.size(); ++i)
                if (ce[i] == ce[i - 1]) { bad = AD_E_DUP_EXEC; bad_key = k; }
            wcount[k] = nw;
        }
    });
    if (bad.load())
    {
        const int code = bad.load();
        return c->fail(code, "CommandsForKey of key %lld violates %s", (long long)K.keys[bad_key.load()],
                       code == AD_E_ORDER ? "byId strict order (CommandsForKey.java:1438)"
                       : code == AD_E_DUP_EXEC ? "unique committed executeAt (CommandsForKey.java:1439)"
                                               : "status range / key-domain ids");
    }
    for (uint64_t k = 0; k + 1 <= nk; ++k)
        if (k > 0 && K.keys[k - 1] >= K.keys[k]) return c->fail(AD_E_INVAL, "keys not strictly ascending");
    woff[0] = 0;
    for (uint64_t k = 0; k < nk; ++k) woff[k + 1] = woff[k] + wcount[k];
    std::vector<uint2> w(woff[nk]);
    parallel_for(nk, [&](size_t ka, size_t kb) {
        std::vector<std::pair<uint32_t, std::pair<uint32_t, uint8_t>>> tmp;
        for (size_t k = ka; k < kb; ++k)
        {
            tmp.clear();
            for (uint64_t e = K.seg[k]; e < K.seg[k + 1]; ++e)
            {
                const uint8_t st = K.status[e];
                const uint32_t kind = (uint32_t)((K.txn[e].lsb >> 1) & 7);
                if (st >= AD_ST_COMMITTED && st <= AD_ST_APPLIED && kind == AD_KIND_WRITE)
                    tmp.push_back({exec_rank[e], {txn_rank[e], st}});
            }
            std::sort(tmp.begin(), tmp.end());
            int32_t m = -1;
            for (size_t i = 0; i < tmp.size(); ++i)
            {
                w[woff[k] + i] = make_uint2(tmp[i].first, tmp[i].second.first);
                if (tmp[i].second.second == AD_ST_APPLIED) m = (int32_t)(woff[k] + i);   // maxAppliedWriteByExecuteAt
            }
            maw[k] = m;
            if (!K.pruned.empty() && K.pruned[k] >= 0)
            {
                const uint64_t idx = K.seg[k] + (uint64_t)K.pruned[k];
                if (idx >= K.seg[k + 1]) { bad = AD_E_INVAL; bad_key = k; continue; }
                pruned[k] = txn_rank[idx];
            }
        }
    });
    if (bad.load()) return c->fail(AD_E_INVAL, "prunedBefore of key %lld is not in byId", (long long)K.keys[bad_key.load()]);
    phase("entries + committed Writes");

    // ---- 3. range commands: (range, command) entries sorted by (start, end, txnId); range table
    RangePart rp;
    if (int rc = build_ranges(c, cmd_rank, wm_rank, &rp)) return rc;
    const std::vector<int64_t>& cell_E = rp.cell_E;
    const bool cell_ok = rp.cell_ok;
    struct { uint64_t n; uint64_t size() const { return n; } } rent{rp.n_rent};
    phase("range commands");
    // ---- 4. upload CFK + dictionary, build the trees
    int rc;
    ent.resize(std::max<uint64_t>(64, (ne + 63) / 64 * 64), make_uint2(0u, 0u));   // whole 64-entry frames (tau 0: never emitted)
    std::vector<KeyRec> krec(nk);
    for (uint64_t k = 0; k < nk; ++k)
    {
        KeyRec& r = krec[k];
        r.seg_lo = seg32[k];
        r.seg_hi = seg32[k + 1];
        r.w_lo = woff[k];
        r.w_hi = woff[k + 1];
        r.last_txn = r.seg_hi > r.seg_lo ? (ent[r.seg_hi - 1].y & RANK_MASK) : 0u;
        r.last_wexec = r.w_hi > r.w_lo ? w[r.w_hi - 1].x : 0u;
        r.pruned = pruned[k];
        r.maw = maw[k];
    }
    uint64_t hcap = 16;
    while (hcap < 2 * nk) hcap <<= 1;
    std::vector<KeySlot> khash(hcap, KeySlot{0, KEY_EMPTY, 0});
    // emission lists of the fused kernel's newest-probe path (KeyEntry, common.hpp)
    std::vector<uint32_t> cand_off(NCLASS * nk + 1), cwr_off(nk + 1), cwr_tail(nk), last_w_txn(nk, 0);
    {
        std::vector<uint32_t> ccount(NCLASS * nk, 0), wcnt(nk, 0);
        parallel_for(nk, [&](size_t ka, size_t kb) {
            for (size_t k = ka; k < kb; ++k)
                for (uint64_t e = seg32[k]; e < seg32[k + 1]; ++e)
                {
                    const uint32_t tau = ent[e].x, kd = ent[e].y >> RANK_BITS;
                    if (tau == TAU_NEVER_ELIDED)
                        for (int cl = 0; cl < NCLASS; ++cl) ccount[cl * nk + k] += (CLASS_KINDS[cl] >> kd) & 1;
                    else if (tau != 0) ++wcnt[k];
                }
        });
        // class-major: all keys' class-0 lists, then class 1, then class 2
        cand_off[0] = 0;
        for (uint64_t i = 0; i < NCLASS * nk; ++i) cand_off[i + 1] = cand_off[i] + ccount[i];
        cwr_off[0] = 0;
        for (uint64_t k = 0; k < nk; ++k) cwr_off[k + 1] = cwr_off[k] + wcnt[k];
    }
    std::vector<uint32_t> cand(std::max<uint32_t>(cand_off[NCLASS * nk], 1)), cwr(std::max<uint32_t>(cwr_off[nk], 1));
    parallel_for(nk, [&](size_t ka, size_t kb) {
        std::vector<uint2> tmp;
        for (size_t k = ka; k < kb; ++k)
        {
            uint32_t cur[NCLASS];
            for (int cl = 0; cl < NCLASS; ++cl) cur[cl] = cand_off[cl * nk + k];
            tmp.clear();
            for (uint64_t e = seg32[k]; e < seg32[k + 1]; ++e)
            {
                const uint32_t tau = ent[e].x, kd = ent[e].y >> RANK_BITS;
                if (tau == TAU_NEVER_ELIDED)
                {
                    for (int cl = 0; cl < NCLASS; ++cl)
                        if ((CLASS_KINDS[cl] >> kd) & 1) cand[cur[cl]++] = ent[e].y;
                }
                else if (tau != 0)
                    tmp.push_back(make_uint2(tau, ent[e].y));
            }
            std::sort(tmp.begin(), tmp.end(), [](const uint2& a, const uint2& b) { return a.x < b.x; });
            uint32_t tail = 0;
            bool has_w = false;
            for (size_t i = 0; i < tmp.size(); ++i)
            {
                cwr[cwr_off[k] + i] = tmp[i].y;
                if ((tmp[i].y >> RANK_BITS) == AD_KIND_WRITE) { tail = (uint32_t)i; has_w = true; }
            }
            cwr_tail[k] = cwr_off[k] + (has_w ? tail : 0);      // no committed Write: M = NONE, all emitted
            last_w_txn[k] = has_w ? (tmp[tail].y & RANK_MASK) : 0u;
        }
    });
    phase("emission lists");
    std::vector<KeyEntry> kent(std::max<uint64_t>(nk, 1));
    std::vector<uint32_t> kslot(std::max<uint64_t>(nk, 1)), kcells(std::max<uint64_t>(nk, 1), NO_CELL);
    // perfect hash of the keys onto KeyLines (hash and displace, common.hpp): buckets of ~4 keys,
    // the biggest placed first, each with the first displacement that puts all its keys on free lines
    uint64_t kl_nb = std::max<uint64_t>(1, nk / 4);
    if (int rc = kl_place_all(c, K.keys, kl_nb, false)) return c->fail(rc, "key perfect hash did not converge");
    for (uint64_t k = 0; k < nk; ++k)
        kslot[k] = (uint32_t)kl_index(key_hash2(K.keys[k]), c->kl_disp_h[kl_bucket(key_hash(K.keys[k]), kl_nb)], c->kline_slots);
    const std::vector<uint32_t>& kl_disp = c->kl_disp_h;
    phase("key line perfect hash");
    for (uint64_t k = 0; k < nk; ++k)
    {
        uint64_t h = key_hash(K.keys[k]) & (hcap - 1);
        while (khash[h].idx != KEY_EMPTY) h = (h + 1) & (hcap - 1);
        uint32_t kcell = NO_CELL;
        if (cell_ok)
        {
            const int64_t x = K.keys[k];
            kcell = (uint32_t)(c->cfg.range_start_inclusive ? std::upper_bound(cell_E.begin(), cell_E.end(), x) - cell_E.begin()
                                                             : std::lower_bound(cell_E.begin(), cell_E.end(), x) - cell_E.begin());
        }
        khash[h] = KeySlot{K.keys[k], (uint32_t)k, kcell};
        kcells[k] = kcell;
        KeyEntry& ke = kent[k];
        ke.last_w_txn = last_w_txn[k];
        ke.last_txn = krec[k].last_txn;
        ke.last_wexec = krec[k].last_wexec;
        ke.pad = 0;
        for (int cl = 0; cl < NCLASS; ++cl)
        {
            ke.cl[cl].cand_lo = cand_off[cl * nk + k];
            ke.cl[cl].cand_hi = cand_off[cl * nk + k + 1];
            ke.cl[cl].cwr_tail = cwr_tail[k];
            ke.cl[cl].cwr_hi = cwr_off[k + 1];
        }
    }
    {
        std::vector<uint32_t> ekey(std::max<uint64_t>(ne, 1), 0);
        for (uint64_t k = 0; k < nk; ++k)
            for (uint64_t e = K.seg[k]; e < K.seg[k + 1]; ++e) ekey[e] = (uint32_t)k;
        if (!K.ballot.empty())
        {
            std::vector<Bal> bl(ne);
            for (uint64_t e = 0; e < ne; ++e) bl[e] = Bal{K.ballot[e].msb, K.ballot[e].lsb, K.ballot[e].node, 0};
            if ((rc = upload(c, c->d_ballot, bl))) return rc;
        }
        else
            c->d_ballot.release();
        if ((rc = upload(c, c->d_status, K.status)) || (rc = upload(c, c->d_xrank, exec_rank)) || (rc = upload(c, c->d_ekey, ekey)))
            return rc;
    }
    phase("key hash + KeyEntry + entry uploads");
    std::vector<uint64_t> shi, slo;
    std::vector<int32_t> snode;
    for (uint64_t i = 0; i < dhi.size(); i += DICT_SAMP)
    {
        shi.push_back(dhi[i]);
        slo.push_back(dlo[i]);
        snode.push_back(dnode[i]);
    }
    const uint64_t n_samp1 = shi.size();
    // the second level (common.hpp dict_rank_sampled) after the first, from a 16-entry boundary
    shi.resize(dict_samp2_base(n_samp1));
    slo.resize(shi.size());
    snode.resize(shi.size());
    for (uint64_t i = 0; n_samp1 && i < dhi.size(); i += DICT_SAMP2)
    {
        shi.push_back(dhi[i]);
        slo.push_back(dlo[i]);
        snode.push_back(dnode[i]);
    }
    if ((rc = upload(c, c->d_ds_hi, shi)) || (rc = upload(c, c->d_ds_lo, slo)) || (rc = upload(c, c->d_ds_node, snode)))
        return rc;
    if ((rc = upload(c, c->d_dict_hi, dhi)) || (rc = upload(c, c->d_dict_lo, dlo)) || (rc = upload(c, c->d_dict_node, dnode)) ||
        (rc = upload(c, c->d_keys, K.keys)) || (rc = upload(c, c->d_krec, krec)) || (rc = upload(c, c->d_khash, khash)) || (rc = upload(c, c->d_kent, kent)) || (rc = upload(c, c->d_cand, cand)) || (rc = upload(c, c->d_cwr, cwr)) ||
        (rc = upload(c, c->d_ent, ent)) || (rc = upload(c, c->d_kslot, kslot)) || (rc = upload(c, c->d_kcell, kcells)) ||
        (rc = upload(c, c->d_kl_disp, kl_disp)) ||
        (rc = upload(c, c->d_w, w)) || (rc = upload(c, c->d_slices_s, c->slice_s)) || (rc = upload(c, c->d_slices_e, c->slice_e)) ||
        (rc = upload(c, c->d_dict_lsb_raw, c->dict_lsb)) || (rc = upload(c, c->d_rt_start, c->rt_start)) ||
        (rc = upload(c, c->d_rt_end, c->rt_end)))
        return rc;

    phase("uploads");
    DevSnapshot& s = c->ds;
    {
        const NormTid last = dhi.empty() ? NormTid{0, 0, 0} : NormTid{dhi.back(), dlo.back(), dnode.back()};
        RangePart rpv;
        rpv.cell_ok = cell_ok;
        rpv.n_rent = rent.size();
        if (cell_ok) rpv.cell_E = cell_E;
        if (int rc2 = set_views(c, dhi.size(), n_samp1, last, nk, ne, hcap, rpv, nrb)) return rc2;
    }
    HIPCHK(c, build_cfk_trees(s, c->stream));
    HIPCHK(c, build_range_trees(s, c->stream));
    // the lean kernels' KeyLine table, indexed by the keys' perfect hash
    if (!c->d_kline.ensure(kline_table_bytes(c->kline_slots))) return c->fail(AD_E_NOMEM, "key lines");
    s.kline = c->d_kline.as<KeyLine>();
    s.kl_lines = c->kline_slots;
    s.kquad = kline_quads(s.kline, c->kline_slots);
    s.kl_buckets = kl_nb;
    s.kl_disp = c->d_kl_disp.as<uint32_t>();
    HIPCHK(c, run_build_klines(s, c->d_kslot.as<uint32_t>(), c->d_kcell.as<uint32_t>(), c->d_kline.as<KeyLine>(),
                               c->kline_slots, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    phase("device trees + key lines");
    c->h_txn_rank.swap(txn_rank);
    c->h_exec_rank.swap(exec_rank);
    c->h_pruned.swap(pruned);
    c->dirty = false;
    ++c->snap_gen;
    ++c->rank_gen;
    cfk_upd_work_invalidate(c->cu);      // state the update path keeps between batches
    c->global_ok = use_global;   // parts carry global ranks exactly when the dictionary is the installed one
    c->n_global = use_global ? c->dict_msb.size() : 0;
    c->ms_ingest = now_ms() - t0;
    return 0;
}

// Host copies of the per-entry state after ad_cfk_update* changed it on the device: status and
// executeAt (from its rank through the dictionary, raw bits of the dictionary member).
static int sync_host_entries(ad_ctx* c);

// TxnInfo.missing() lists maintained on the device -> the host copy (ids from their ranks)
static int pull_missing(ad_ctx* c)
{
    auto& K = c->cfk;
    const uint64_t ne = c->dmiss_lists, nm = c->dmiss_ids;
    K.miss_off.resize(ne + 1);
    std::vector<uint32_t> r(nm);
    HIPCHK(c, copy_sync(K.miss_off.data(), c->d_moff.p, 8 * (ne + 1), hipMemcpyDeviceToHost));
    if (nm) HIPCHK(c, copy_sync(r.data(), c->d_mids.p, 4 * nm, hipMemcpyDeviceToHost));
    K.miss.resize(nm);
    for (uint64_t j = 0; j < nm; ++j)
    {
        const uint64_t i = (r[j] - 1) / 2;
        K.miss[j] = Tid{c->dict_msb[i], c->dict_lsb[i], c->dict_node[i]};
    }
    K.miss_stale = false;
    return 0;
}

// The dictionary's host copy after a device ingest (read back on first use)
static int host_dict(ad_ctx* c)
{
    if (!c->host_dict_stale) return 0;
    const uint64_t nd = c->ds.n_dict;
    c->dict_msb.resize(nd);
    c->dict_lsb.resize(nd);
    c->dict_node.resize(nd);
    if (nd)
    {
        HIPCHK(c, d2h(c->dict_msb.data(), c->d_dict_hi.p, 8 * nd, c->stream));
        HIPCHK(c, d2h(c->dict_lsb.data(), c->d_dict_lsb_raw.p, 8 * nd, c->stream));
        HIPCHK(c, d2h(c->dict_node.data(), c->d_dict_node.p, 4 * nd, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    c->host_dict_stale = false;
    return 0;
}

// The loaded byId ids on the host (ad_cfk_load left them in HBM only): read back from the raw columns
static int host_inputs(ad_ctx* c)
{
    auto& K = c->cfk;
    if (!c->raw_dev || K.txn.size() == c->raw_ne) return 0;
    const uint64_t ne = c->raw_ne;
    std::vector<uint64_t> tm(ne), tl(ne), em(ne), el(ne);
    std::vector<int32_t> tn(ne), en(ne);
    if (ne)
    {
        HIPCHK(c, copy_sync(tm.data(), c->d_in_tm.p, 8 * ne, hipMemcpyDeviceToHost));
        HIPCHK(c, copy_sync(tl.data(), c->d_in_tl.p, 8 * ne, hipMemcpyDeviceToHost));
        HIPCHK(c, copy_sync(tn.data(), c->d_in_tn.p, 4 * ne, hipMemcpyDeviceToHost));
        HIPCHK(c, copy_sync(em.data(), c->d_in_em.p, 8 * ne, hipMemcpyDeviceToHost));
        HIPCHK(c, copy_sync(el.data(), c->d_in_el.p, 8 * ne, hipMemcpyDeviceToHost));
        HIPCHK(c, copy_sync(en.data(), c->d_in_en.p, 4 * ne, hipMemcpyDeviceToHost));
    }
    K.txn.resize(ne);
    K.exec.resize(ne);
    parallel_for(ne, [&](size_t a, size_t b) {
        for (size_t e = a; e < b; ++e)
        {
            K.txn[e] = {tm[e], tl[e], tn[e]};
            K.exec[e] = {em[e], el[e], en[e]};
        }
    });
    return 0;
}

static int sync_host(ad_ctx* c)
{
    if (int rc = host_dict(c)) return rc;
    if (int rc = host_inputs(c)) return rc;
    if (!c->host_stale) return 0;
    if (int rc = sync_host_entries(c)) return rc;
    return c->dmiss_on ? pull_missing(c) : 0;
}

static int sync_host_entries(ad_ctx* c)
{
    if (!c->host_stale) return 0;
    auto& K = c->cfk;
    if (c->d_ballot.p)
    {
        const uint64_t ne = c->ds.n_ent;
        std::vector<Bal> bl(ne);
        if (ne) HIPCHK(c, copy_sync(bl.data(), c->d_ballot.p, sizeof(Bal) * ne, hipMemcpyDeviceToHost));
        K.ballot.resize(ne);
        for (uint64_t e = 0; e < ne; ++e) K.ballot[e] = Tid{bl[e].msb, bl[e].lsb, bl[e].node};
    }
    if (c->host_moved)
    {
        // entries were inserted: rebuild the host copies (byId ids from their ranks) from the device
        const uint64_t ne = c->ds.n_ent, nk = c->ds.n_keys;
        std::vector<uint2> ent(ne);
        std::vector<KeyRec> kr(nk);
        K.status.resize(ne);
        std::vector<uint32_t> xr(ne);
        if (ne)
        {
            HIPCHK(c, d2h(ent.data(), c->d_ent.p, 8 * ne, c->stream));
            HIPCHK(c, d2h(K.status.data(), c->d_status.p, ne, c->stream));
            HIPCHK(c, d2h(xr.data(), c->d_xrank.p, 4 * ne, c->stream));
        }
        if (nk) HIPCHK(c, d2h(kr.data(), c->d_krec.p, sizeof(KeyRec) * nk, c->stream));
        if (K.keys.size() != nk)
        {
            // keys created on the device
            K.keys.resize(nk);
            if (nk) HIPCHK(c, d2h(K.keys.data(), c->d_keys.p, 8 * nk, c->stream));
            K.seg.assign(nk + 1, 0);
            if (!K.pruned.empty()) K.pruned.assign(nk, -1);
            c->h_pruned.assign(nk, 0);
        }
        HIPCHK(c, hipStreamSynchronize(c->stream));
        auto tid = [&](uint32_t rank) -> Tid {
            const uint64_t i = (rank - 1) / 2;
            return Tid{c->dict_msb[i], c->dict_lsb[i], c->dict_node[i]};
        };
        K.txn.resize(ne);
        K.exec.resize(ne);
        c->h_txn_rank.resize(ne);
        for (uint64_t e = 0; e < ne; ++e)
        {
            const uint32_t tr = ent[e].y & RANK_MASK;
            c->h_txn_rank[e] = tr;
            K.txn[e] = tid(tr);
            K.exec[e] = xr[e] == tr ? K.txn[e] : tid(xr[e]);
        }
        for (uint64_t k = 0; k < nk; ++k) K.seg[k + 1] = kr[k].seg_hi;
        // prunedBefore as an index into the key's byId (insertions may have moved it), and its rank
        if (!K.pruned.empty())
            for (uint64_t k = 0; k < nk; ++k)
            {
                K.pruned[k] = -1;
                if (!kr[k].pruned) continue;
                const auto b = c->h_txn_rank.begin();
                const auto it = std::lower_bound(b + kr[k].seg_lo, b + kr[k].seg_hi, kr[k].pruned);
                if (it != b + kr[k].seg_hi && *it == kr[k].pruned) K.pruned[k] = (int64_t)(it - (b + kr[k].seg_lo));
            }
        if (c->h_pruned.size() == nk)
            for (uint64_t k = 0; k < nk; ++k) c->h_pruned[k] = kr[k].pruned;
        c->h_exec_rank.swap(xr);
        if (!K.miss_off.empty() && !c->host_ingested) K.miss_stale = true;       // entries moved: load the lists again
        c->host_ingested = false;
        c->host_moved = false;
        c->host_stale = false;
        return 0;
    }
    const uint64_t ne = K.status.size();
    std::vector<uint32_t> xr(ne);
    if (ne)
    {
        HIPCHK(c, d2h(K.status.data(), c->d_status.p, ne, c->stream));
        HIPCHK(c, d2h(xr.data(), c->d_xrank.p, 4 * ne, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    for (uint64_t e = 0; e < ne; ++e)
        if (xr[e] != c->h_exec_rank[e])
        {
            const uint64_t i = (xr[e] - 1) / 2;
            K.exec[e] = {c->dict_msb[i], c->dict_lsb[i], c->dict_node[i]};
        }
    c->h_exec_rank.swap(xr);
    // TxnInfo.missing() exists only for ACCEPTED..APPLIED (CommandsForKey.java:278): an entry that
    // left that range through an update needs its lists loaded again
    if (!K.miss_off.empty())
        for (uint64_t e = 0; e < ne && !K.miss_stale; ++e)
            if (K.miss_off[e + 1] > K.miss_off[e] && !(K.status[e] >= AD_ST_ACCEPTED && K.status[e] <= AD_ST_APPLIED))
                K.miss_stale = true;
    c->host_stale = false;
    return 0;
}

// SEQUENTIAL PreAccepts of Range-domain txns (sync points, range reads / writes): Commands.preaccept
// stores the command and InMemorySafeStore.update registers it as a range command
// (InMemoryCommandStore.java:740-763): rangeCommands[txnId].update(ranges.slice(slice, Minimal)), slice =
// the store's ranges less the shard-redundant ones (RedundantBefore.removeShardRedundant,
// RedundantBefore.java:216-225,433-437: an entry in the epoch bounds of (txnId, executeAt = txnId)
// whose shardAppliedOrInvalidatedBefore is above txnId takes its range away). Appended to the store's
// range commands (live, not historical; recovery facts, when loaded, those of a PreAccepted command:
// neither proposed nor stable, no deps, executeAtOrTxnId = txnId); the snapshot is rebuilt before the
// batch resolves, so every request sees the ones below its txnId (STARTED_BEFORE) -- the sequential
// answer (PreAccept.java:116-132). A txnId already among the range commands is refused (AD_E_INVAL;
// RangeCommand.update's union with its earlier ranges is not modelled).
static int register_range_txns(ad_ctx* c, const ad_query_soa* q, const std::vector<uint64_t>& idx)
{
    auto& R = c->cmds;
    std::vector<NormTid> have;
    have.reserve(R.txn.size());
    for (const Tid& t : R.txn) have.push_back(norm(t));
    std::sort(have.begin(), have.end(), [](const NormTid& a, const NormTid& b) { return norm_cmp(a, b) < 0; });
    const bool incl_rb = !c->rb.wm.empty();
    const size_t n_sl = c->slice_s.empty() ? 1 : c->slice_s.size();
    for (uint64_t i : idx)
    {
        const Tid t{q->txn_msb[i], q->txn_lsb[i], q->txn_node[i]};
        const NormTid tn = norm(t);
        auto it = std::lower_bound(have.begin(), have.end(), tn, [](const NormTid& a, const NormTid& b) { return norm_cmp(a, b) < 0; });
        if (it != have.end() && norm_cmp(*it, tn) == 0)
            return c->fail(AD_E_INVAL, "SEQUENTIAL request %llu: its Range-domain txnId is already a range command of the store",
                           (unsigned long long)i);
        // ranges.slice(slice, Minimal): every non-empty intersection with a slice range, ascending
        std::vector<std::pair<int64_t, int64_t>> rs;
        for (uint64_t j = q->range_off[i]; j < q->range_off[i + 1]; ++j)
            for (size_t sl = 0; sl < n_sl; ++sl)
            {
                int64_t a = q->range_start[j], b = q->range_end[j];
                if (!c->slice_s.empty())
                {
                    a = std::max(a, c->slice_s[sl]);
                    b = std::min(b, c->slice_e[sl]);
                }
                if (a < b) rs.push_back({a, b});
            }
        // removeShardRedundant: Ranges.subtract of each redundant entry's range
        const int64_t ep = (int64_t)(t.msb >> 15);
        for (size_t e = 0; incl_rb && e < c->rb.wm.size(); ++e)
        {
            if (ep < c->rb.e0[e] || ep >= c->rb.e1[e]) continue;                        // outOfBounds(txnId, executeAt)
            if (!(norm_cmp(tn, norm(c->rb.wm[e])) < 0)) continue;                      // txnId < shardAppliedOrInvalidatedBefore
            const int64_t x0 = c->rb.start[e], x1 = c->rb.end[e];
            std::vector<std::pair<int64_t, int64_t>> out;
            for (auto& r : rs)
            {
                if (!(r.first < x1 && r.second > x0)) { out.push_back(r); continue; }
                if (r.first < x0) out.push_back({r.first, x0});
                if (x1 < r.second) out.push_back({x1, r.second});
            }
            rs.swap(out);
        }
        if (R.off.empty()) R.off.push_back(0);
        R.txn.push_back(t);
        for (auto& r : rs)
        {
            R.start.push_back(r.first);
            R.end.push_back(r.second);
        }
        R.off.push_back(R.start.size());
        if (!R.erased.empty()) R.erased.push_back(0);
        if (!R.historical.empty()) R.historical.push_back(0);
        if (R.rec)
        {
            R.rec_status.push_back(0);
            R.rec_has_deps.push_back(0);
            R.rec_exec.push_back(t);
            R.rec_dep_off.push_back(R.rec_dep_off.empty() ? 0 : R.rec_dep_off.back());
        }
        have.insert(std::lower_bound(have.begin(), have.end(), tn, [](const NormTid& a, const NormTid& b) { return norm_cmp(a, b) < 0; }), tn);
    }
    c->rv_gen = ~0ull;
    c->rv_rng_gen = ~0ull;
    drop_global_dict(c);            // new ids: a node-wide dictionary must be installed again
    c->dirty = true;
    return 0;
}

// SEQUENTIAL: insert every request's txnId as PREACCEPTED_OR_ACCEPTED_INVALIDATE into the
// CommandsForKey of each of its keys in the slice (CommandsForKey.update, :972-1042; a present
// entry below PREACCEPTED is raised, otherwise left alone); Range-domain requests register as range
// commands (register_range_txns).
static int apply_preaccepts(ad_ctx* c, const ad_query_soa* q)
{
    if (int rc0 = sync_host(c)) return rc0;
    auto& K = c->cfk;
    struct Ins { int64_t key; NormTid n; Tid t; };
    std::vector<Ins> ins;
    std::vector<uint64_t> rng;        // the batch's Range-domain requests
    for (uint64_t i = 0; i < q->n_txns; ++i)
    {
        const Tid t{q->txn_msb[i], q->txn_lsb[i], q->txn_node[i]};
        const Tid x{q->exec_msb[i], q->exec_lsb[i], q->exec_node[i]};
        if (!(t.msb == x.msb && ((t.lsb ^ x.lsb) & 0xFFFFFFFFFFFF001EULL) == 0 && t.node == x.node))
            return c->fail(AD_E_INVAL, "SEQUENTIAL (PreAccept) requests need executeAt == txnId");
        if (i > 0)
        {
            const Tid p{q->txn_msb[i - 1], q->txn_lsb[i - 1], q->txn_node[i - 1]};
            if (norm_cmp(norm(p), norm(t)) >= 0) return c->fail(AD_E_INVAL, "SEQUENTIAL requests must be in ascending TxnId order");
        }
        if (q->range_off && q->range_off[i + 1] > q->range_off[i])
        {
            rng.push_back(i);
            continue;
        }
        const uint32_t kind = (uint32_t)((t.lsb >> 1) & 7);
        const bool manages = (t.lsb & 1) == 0 && ((KINDS_ANY_GLOBALLY_VISIBLE >> kind) & 1);  // CommandsForKey.manages :185-188
        if (!manages) continue;
        for (uint64_t k = q->key_off[i]; k < q->key_off[i + 1]; ++k)
        {
            const int64_t key = q->keys[k];
            bool in = c->slice_s.empty();
            for (size_t s = 0; s < c->slice_s.size() && !in; ++s)
                in = range_contains(c->cfg.range_start_inclusive, c->slice_s[s], c->slice_e[s], key);
            if (in) ins.push_back({key, norm(t), t});
        }
    }
    if (!rng.empty())
        if (int rc = register_range_txns(c, q, rng)) return rc;
    if (ins.empty()) return 0;
    if (!K.miss_off.empty()) K.miss_stale = true;
    std::stable_sort(ins.begin(), ins.end(), [](const Ins& a, const Ins& b) {
        if (a.key != b.key) return a.key < b.key;
        return norm_cmp(a.n, b.n) < 0;
    });
    std::vector<int64_t> nkeys;
    std::vector<uint64_t> nseg{0};
    std::vector<Tid> ntx, nex;
    std::vector<uint8_t> nst;
    std::vector<int64_t> npr;
    std::vector<Tid> nbal;
    const bool bal = !K.ballot.empty();
    size_t ki = 0, ii = 0;
    const size_t nk = K.keys.size();
    while (ki < nk || ii < ins.size())
    {
        int64_t key;
        if (ii >= ins.size() || (ki < nk && K.keys[ki] <= ins[ii].key)) key = K.keys[ki];
        else key = ins[ii].key;
        const bool has_old = ki < nk && K.keys[ki] == key;
        uint64_t e = has_old ? K.seg[ki] : 0, e1 = has_old ? K.seg[ki + 1] : 0;
        const size_t base = ntx.size();
        int64_t pr = has_old && !K.pruned.empty() ? K.pruned[ki] : -1;
        int64_t pr_new = -1;
        while (e < e1 || (ii < ins.size() && ins[ii].key == key))
        {
            const bool take_old = e < e1 && (!(ii < ins.size() && ins[ii].key == key) || norm_cmp(norm(K.txn[e]), ins[ii].n) <= 0);
            if (take_old)
            {
                if ((int64_t)(e - K.seg[ki]) == pr) pr_new = (int64_t)(ntx.size() - base);
                const bool same = ii < ins.size() && ins[ii].key == key && norm_cmp(norm(K.txn[e]), ins[ii].n) == 0;
                ntx.push_back(K.txn[e]);
                if (bal) nbal.push_back(K.ballot[e]);
                if (same && K.status[e] < AD_ST_PREACCEPTED_OR_ACCEPTED_INVALIDATE)
                {
                    nex.push_back(K.txn[e]);
                    nst.push_back(AD_ST_PREACCEPTED_OR_ACCEPTED_INVALIDATE);
                }
                else
                {
                    nex.push_back(K.exec[e]);
                    nst.push_back(K.status[e]);
                }
                if (same) ++ii;
                ++e;
            }
            else
            {
                ntx.push_back(ins[ii].t);
                if (bal) nbal.push_back(Tid{0, 0, 0});          // a PreAccept: Ballot.ZERO
                nex.push_back(ins[ii].t);
                nst.push_back(AD_ST_PREACCEPTED_OR_ACCEPTED_INVALIDATE);
                ++ii;
            }
        }
        nkeys.push_back(key);
        nseg.push_back(ntx.size());
        npr.push_back(pr_new);
        if (has_old) ++ki;
    }
    K.keys.swap(nkeys);
    K.seg.swap(nseg);
    K.txn.swap(ntx);
    K.exec.swap(nex);
    K.status.swap(nst);
    K.pruned.swap(npr);
    K.ballot.swap(nbal);
    c->dirty = true;
    return 0;
}

// ---------------------------------------------------------------------------------------
// batch pipeline
// ---------------------------------------------------------------------------------------
template <class T>
static bool ens(DevBuf& b, uint64_t n) { return b.ensure(sizeof(T) * std::max<uint64_t>(n, 1)); }

// A small upload (at most UP_WORDS words) ordered on st without a host wait: copied into the context's
// pinned slot `k`, whose previous copy has completed first (its event; normally long done). A pageable
// h2d would return only after the copy -- after everything queued before it on st.
constexpr uint64_t UP_WORDS = 512;
static hipError_t up_small(ad_ctx* c, int k, void* dst, const void* src, size_t bytes, hipStream_t st)
{
    if (!bytes) return hipSuccess;
    if (bytes > sizeof(uint64_t) * UP_WORDS) return h2d(dst, src, bytes, st);
    if (!c->h_up[k])
        if (hipError_t e = hipHostMalloc((void**)&c->h_up[k], sizeof(uint64_t) * UP_WORDS, hipHostMallocDefault))
        {
            c->h_up[k] = nullptr;
            return e;
        }
    if (!c->ev_up[k])
        if (hipError_t e = hipEventCreateWithFlags(&c->ev_up[k], hipEventDisableTiming))
        {
            c->ev_up[k] = nullptr;
            return e;
        }
    if (c->up_busy[k])
    {
        if (hipError_t e = hipEventSynchronize(c->ev_up[k])) return e;
        c->up_busy[k] = false;
    }
    memcpy(c->h_up[k], src, bytes);
    if (hipError_t e = hipMemcpyAsync(dst, c->h_up[k], bytes, hipMemcpyHostToDevice, st)) return e;
    if (hipError_t e = hipEventRecord(c->ev_up[k], st))
    {
        // the copy may be queued with no event covering it: the slot is free only once the stream is done
        (void)hipStreamSynchronize(st);
        return e;
    }
    c->up_busy[k] = true;
    return hipSuccess;
}

// UP_WORDS pinned words for read-backs: several async copies into them, then one synchronisation (a
// pageable d2h waits for its own copy -- two of them cost two round trips). Only between a call's copies
// and its synchronisation.
static uint64_t* rb_slot(ad_ctx* c)
{
    if (!c->h_rb && hipHostMalloc((void**)&c->h_rb, sizeof(uint64_t) * UP_WORDS, hipHostMallocDefault) != hipSuccess)
        c->h_rb = nullptr;
    return c->h_rb;
}

// bind the split kernels' per-batch arrays for a batch of n requests / np probes
static bool bind_split(ad_ctx::SplitBufs& S, BatchBufs& b, uint64_t n, uint64_t np, bool own_sizes)
{
    if (!ens<uint32_t>(S.t_S, n) || !ens<uint32_t>(S.t_self, n) || !ens<uint32_t>(S.t_kinds, n) ||
        !ens<int64_t>(S.t_epoch, n) || !ens<uint32_t>(S.p_txn, np) || !ens<uint4>(S.p_rec, np) ||
        !ens<uint32_t>(S.p_off, np) || !ens<uint32_t>(S.p_c0, np) || !ens<uint32_t>(S.p_c1, np) ||
        !ens<uint32_t>(S.p_roff, np) || !ens<uint32_t>(S.p_rcnt, np) || !ens<uint64_t>(S.p_rb, np))
        return false;
    b.t_S = S.t_S.as<uint32_t>(); b.t_self = S.t_self.as<uint32_t>(); b.t_kinds = S.t_kinds.as<uint32_t>();
    b.t_epoch = S.t_epoch.as<int64_t>(); b.p_txn = S.p_txn.as<uint32_t>(); b.p_rec = S.p_rec.as<uint4>();
    b.p_off = S.p_off.as<uint32_t>(); b.p_c0 = S.p_c0.as<uint32_t>(); b.p_c1 = S.p_c1.as<uint32_t>();
    b.p_roff = S.p_roff.as<uint32_t>(); b.p_rcnt = S.p_rcnt.as<uint32_t>(); b.p_rb = S.p_rb.as<uint64_t>();
    if (own_sizes)
    {
        if (!ens<uint32_t>(S.sz, 9 * n) || !ens<uint64_t>(S.t_reg, 3 * n)) return false;
        b.sz = S.sz.as<uint32_t>();
        b.t_reg = S.t_reg.as<uint64_t>();
    }
    return true;
}

static int run_split(ad_ctx* c, const BatchBufs& b, hipStream_t st)
{
    HIPCHK(c, run_encode(c->ds, b, st));
    HIPCHK(c, run_scan(c->ds, b, st));
    HIPCHK(c, run_range(c->ds, b, st));
    HIPCHK(c, run_build(c->ds, b, st));
    return 0;
}

// requests per wave of lean pass 1 by the batch's keys per request (lean_rpw1): four up to 4.5 keys on
// average, else two; AD_LEAN_RPW overrides (8: opt-in, measured no faster on a store's share of
// requests spanning many stores).
// Lean pass 1 as gather + build (k_lean_gather, k_lean_build): opt-in, AD_LEAN_GB=1. Measured on config 2
// (DESIGN §4): gather 0.19-0.30 ms + build 0.36 + wide build 0.15 against 0.54 ms for the fused pass -- the
// build alone is issue-bound (its SIMDs ~98 % busy at ~390 VALU per two requests), so the split buys no
// latency hiding the fused pass lacks
static bool lean_gb_on()
{
    const char* e = getenv("AD_LEAN_GB");
    return e && atoi(e) != 0;
}

static uint32_t lean_rpw1(uint64_t n, uint64_t np)
{
    if (const char* e = getenv("AD_LEAN_RPW")) return atoi(e) == 8 ? 8u : (atoi(e) == 4 ? 4u : 2u);
    // With range commands up to 4 keys per request on average: four per wave (config 4: pass 1 0.90 ->
    // 0.58 ms, its deferrals -- above 16 raw emissions -- two per wave in pass 2); up to 4.5, so that a few
    // Range-domain requests (their expanded probes; the split kernels resolve them) do not tip a 4-key batch
    // over (config 4 with 1 % of them: pass 1 0.93 ms at two per wave). Without range commands also up to 4.5:
    // config 3's store (4 uniform keys per request) pass 1 0.725 -> 0.477 ms, pass 2 0.010 -> 0.099 ms for the
    // 4 % above 16 raw emissions (scripts/lean_lab.py --config 3)
    return 2 * np <= 9 * n ? 4u : 2u;
}

// Lean pass 1 wide or narrow (rpw 2, no range commands; results identical either way). The wide kernel
// resolves requests of 33..64 raw emissions in pass 1 but runs at 4 waves per SIMD instead of 5: worth it
// on config 2 (Zipf keys, ~8 % of requests above 32: 0.613 -> 0.560 ms for passes 1 + 2), not on config
// 3's store (uniform keys: 0.743 -> 0.841 ms). Chosen from the previous batch of the store: after a wide
// batch by its share of requests above 32 (BatchCtl.n_wide1); after a narrow one by its pass-2 share less
// what a wide pass 1 also deferred. AD_LEAN_WIDE1=0/1 forces it.
constexpr double LEAN_WIDE_SHARE = 0.06;
static bool lean_wide1(const ad_ctx* c)
{
    if (const char* e = getenv("AD_LEAN_WIDE1")) return atoi(e) != 0;
    return c->lean_wide;
}
static void lean_wide1_update(ad_ctx* c, uint64_t n, const BatchCtl& h)
{
    if (!n) return;
    if (c->lean_ran_wide)
    {
        c->lean_other = (double)h.n_real1 / (double)n;
        c->lean_wide = (double)h.n_wide1 / (double)n >= LEAN_WIDE_SHARE;
    }
    else
        c->lean_wide = (double)h.n_real1 / (double)n - c->lean_other >= LEAN_WIDE_SHARE;
}

// The wait at the end of a batch (its one host round trip): the calling thread polls an event recorded
// behind the control-block copy rather than sleeping in hipStreamSynchronize -- the host's wake-up
// latency is part of every step (config 2: 0.698 / 0.697 ms per step synchronized, 0.686 / 0.695
// polled). AD_SPIN_WAIT=0 restores the synchronize.
static hipError_t batch_wait(ad_ctx* c, hipStream_t st)
{
    static const bool spin = getenv("AD_SPIN_WAIT") == nullptr || atoi(getenv("AD_SPIN_WAIT")) != 0;
    if (!spin) return hipStreamSynchronize(st);
    if (!c->ev_done)
        if (hipError_t e = hipEventCreateWithFlags(&c->ev_done, hipEventDisableTiming)) return e;
    if (hipError_t e = hipEventRecord(c->ev_done, st)) return e;
    // bounded: busy polls for up to ~2 ms (a batch's usual span), then polls that yield the core (50 us
    // sleeps), and after AD_WAIT_TIMEOUT_MS (default 120 s) the batch is given up (hipErrorLaunchTimeOut ->
    // AD_E_DEVICE) instead of a store thread spinning on a completion that never comes
    static const double timeout_ms = getenv("AD_WAIT_TIMEOUT_MS") ? atof(getenv("AD_WAIT_TIMEOUT_MS")) : 120000.0;
    const double t0 = now_ms();
    hipError_t e;
    while ((e = hipEventQuery(c->ev_done)) == hipErrorNotReady)
    {
        const double dt = now_ms() - t0;
        if (dt < 2.0) continue;
        if (dt > timeout_ms) return hipErrorLaunchTimeOut;
        std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
    return e;
}

static int run_pipeline(ad_ctx* c, const ad_query_soa* q, hipStream_t st, ad_deps_result* out, bool parts_only = false,
                        bool n_keys_given = false, int recovery_scan = -1, const RecoveryView* rv = nullptr)
{
    const uint64_t n = q->n_txns;
    uint64_t np = 0;
    // Range-domain requests (ad_query_soa.range_off): expanded into probes on the device -- keys inside
    // the sliced ranges, the sliced ranges, the unsliced ranges (kernels.hip k_range_count /
    // k_range_fill). Recovery scans take no RedundantBefore (mapReduceFull, InMemoryCommandStore.java:874-882):
    // no unsliced-range probes. The totals the host needs come back through pinned words, one wait each.
    const bool ranges = n && q->range_off;
    if (ranges && (!q->range_start || !q->range_end)) return c->fail(AD_E_INVAL, "range_off without range_start / range_end");
    if ((n && !n_keys_given) || ranges)
        if (!c->h_small) HIPCHK(c, hipHostMalloc((void**)&c->h_small, 64, hipHostMallocDefault));
    uint64_t nr = 0;
    if (n && n_keys_given)
    {
        np = q->n_keys;
        if (ranges) nr = q->n_ranges;
    }
    else if (n)
    {
        uint64_t* hs = c->h_small;
        hs[0] = hs[1] = hs[2] = 0;
        HIPCHK(c, hipMemcpyAsync(&hs[0], q->key_off + n, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
        if (ranges)
        {
            HIPCHK(c, hipMemcpyAsync(&hs[1], q->range_off, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
            HIPCHK(c, hipMemcpyAsync(&hs[2], q->range_off + n, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
        }
        HIPCHK(c, hipStreamSynchronize(st));
        np = hs[0];
        nr = hs[2] - hs[1];
    }
    if (nr)
    {
        if (!ens<uint32_t>(c->rq_cnt, n) || !ens<uint64_t>(c->rq_off, n + 1) || !ens<uint32_t>(c->rq_err, 2) ||
            !ens<uint64_t>(c->rq_bsum, (n + 1023) / 1024 + 16) || !ens<uint32_t>(c->rq_list, n))
            return c->fail(AD_E_NOMEM, "range request expansion");
        HIPCHK(c, hipMemsetAsync(c->rq_err.p, 0, 8, st));
        // rq_err[0]: the rejection flag; rq_err[1]: the Range-domain requests, listed in rq_list
        HIPCHK(c, run_range_count(c->ds, n, q->key_off, q->range_off, q->range_start, q->range_end, c->rq_cnt.as<uint32_t>(),
                                  c->rq_err.as<uint32_t>(), c->rq_list.as<uint32_t>(), nr, recovery_scan < 0, st));
        HIPCHK(c, run_scan_arrays(c->rq_cnt.as<uint32_t>(), c->rq_off.as<uint64_t>(), n, 1, c->rq_bsum.as<uint64_t>(), st));
        uint64_t* hs = c->h_small;
        HIPCHK(c, hipMemcpyAsync(&hs[3], c->rq_off.as<uint64_t>() + n, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
        HIPCHK(c, hipMemcpyAsync(&hs[4], c->rq_err.p, 2 * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
        HIPCHK(c, hipStreamSynchronize(st));
        const uint32_t err = (uint32_t)hs[4], n_rreq = (uint32_t)(hs[4] >> 32);
        if (err)
            return c->fail(AD_E_INVAL, "Range-domain request: keys and ranges together, or ranges not normalised "
                                       "(start < end, ascending, disjoint)");
        np = hs[3];
        if (!ens<int64_t>(c->rq_keys, np) || !ens<int64_t>(c->rq_hi, np) || !ens<uint8_t>(c->rq_kind, np))
            return c->fail(AD_E_NOMEM, "range request probes");
        HIPCHK(c, run_range_fill(c->ds, n, q->key_off, q->keys, q->range_off, q->range_start, q->range_end,
                                 c->rq_off.as<uint64_t>(), c->rq_keys.as<int64_t>(), c->rq_hi.as<int64_t>(),
                                 c->rq_kind.as<uint8_t>(), c->rq_list.as<uint32_t>(), n_rreq, recovery_scan < 0, st));
    }
    // a batch with Range-domain requests keeps the lean / general path for its key-domain requests: k_prepare
    // marks the Range-domain ones, k_resolve hands them to the split kernels' list (resolved after the first
    // pack pass, like any request the fused kernels cannot take)
    const bool split_only = c->cfg.path == 1 || recovery_scan >= 0;
    // the lean kernel covers stores without redundant-before entries, elision on
    // (range commands only with their stabbing index)
    const bool lean = !split_only && np > 0 && (c->ds.n_rent == 0 || c->ds.cell_off != nullptr) && c->ds.n_rb == 0 &&
                      c->ds.elide && getenv("AD_NO_LEAN") == nullptr;
    BatchBufs b{};
    b.n_txns = n;
    b.n_probes = np;
    b.q_txn_msb = q->txn_msb; b.q_txn_lsb = q->txn_lsb; b.q_txn_node = q->txn_node;
    b.q_exec_msb = q->exec_msb; b.q_exec_lsb = q->exec_lsb; b.q_exec_node = q->exec_node;
    b.q_min_epoch = q->min_epoch; b.q_key_off = q->key_off; b.q_keys = q->keys;
    if (nr)
    {
        b.q_key_off = c->rq_off.as<uint64_t>();
        b.q_keys = c->rq_keys.as<int64_t>();
        b.q_keys_hi = c->rq_hi.as<int64_t>();
        b.p_kind = c->rq_kind.as<uint8_t>();
    }
    const uint64_t nb = (n + 1023) / 1024;
    if (!ens<uint32_t>(c->sz, 9 * n) || !ens<uint64_t>(c->off, 9 * (n + 1)) || !ens<uint64_t>(c->bsum, 9 * nb + 16) ||
        !ens<uint64_t>(c->t_reg, 3 * n) || !ens<BatchCtl>(c->ctl, 1) || !ens<uint32_t>(c->deferred, n) ||
        !ens<uint4>(c->q_rec, n) || !ens<uint32_t>(c->deferred1, n + DEFER_CHUNK * (uint64_t)device_cu_count() * 64) ||
        !ens<uint32_t>(c->deferred2, n + DEFER_CHUNK * (uint64_t)device_cu_count() * 64) || !ens<uint32_t>(c->big, n))
        return c->fail(AD_E_NOMEM, "batch buffers");
    b.big = c->big.as<uint32_t>();
    b.k2_big = K2_BIG;
    if (lean && !c->ds.n_rent)
    {
        if (!ens<uint32_t>(c->p_slot, std::max<uint64_t>(np, 1))) return c->fail(AD_E_NOMEM, "probe slots");
        b.p_slot = c->p_slot.as<uint32_t>();
        b.slots_by_prepare = getenv("AD_SLOTS_KERNEL") == nullptr;     // measurement switch: the separate launch
    }
    // lean pass 1 as gather + build (two requests per build wave, no range commands): AD_LEAN_GB=0 keeps
    // the single fused pass
    const bool gb = lean && !c->ds.n_rent && lean_rpw1(n, np) == 2 && lean_gb_on();
    if (gb)
    {
        if (!ens<uint32_t>(c->lg_stage, n * 64) || !ens<uint4>(c->lg_rec, n) || !ens<int64_t>(c->lg_keys, n * 8) ||
            !ens<uint64_t>(c->lg_dummy, (uint64_t)device_cu_count() * 64 * 16))
            return c->fail(AD_E_NOMEM, "lean stage");
        b.lg_dummy = c->lg_dummy.as<uint64_t>();
        b.lg_stage = c->lg_stage.as<uint32_t>();
        b.lg_rec = c->lg_rec.as<uint4>();
        b.lg_keys = c->lg_keys.as<int64_t>();
    }
    if (const char* e = getenv("AD_K2_BIG")) b.k2_big = (uint32_t)strtoul(e, nullptr, 10);   // tests: force k_build_big
    b.q_rec = c->q_rec.as<uint4>();
    b.deferred1 = c->deferred1.as<uint32_t>();
    b.deferred2 = c->deferred2.as<uint32_t>();
    b.sz = c->sz.as<uint32_t>(); b.off = c->off.as<uint64_t>(); b.bsum = c->bsum.as<uint64_t>();
    b.t_reg = c->t_reg.as<uint64_t>(); b.ctl = c->ctl.as<BatchCtl>(); b.deferred = c->deferred.as<uint32_t>();
    if (split_only && !bind_split(c->split, b, n, np, false)) return c->fail(AD_E_NOMEM, "split buffers");

    const uint64_t waves = (uint64_t)device_cu_count() * 8 * 4;
    const uint64_t k2_waves = (uint64_t)device_cu_count() * 16;
    const uint64_t np_split = split_only ? np : std::min<uint64_t>(np, 1u << 20);
    uint64_t want_key = std::max<uint64_t>(np_split * 4 + waves * 4096, 1u << 20);
    uint64_t want_rng = c->ds.n_rent ? std::max<uint64_t>(np_split * 2 + waves * 2048, 1u << 20) : 1;
    uint64_t want_scr = 64ull << 20;
    uint64_t want_reg = std::max<uint64_t>(n * 3 * 8 + np * 24 + k2_waves * (3ull << 16), 16ull << 20);
    if (c->key_cap < want_key) c->key_cap = want_key;
    if (c->rng_cap < want_rng) c->rng_cap = want_rng;
    if (c->scr_cap < want_scr) c->scr_cap = want_scr;
    if (c->reg_cap < want_reg) c->reg_cap = want_reg;
    constexpr uint64_t REG_CAP_MAX = (1ull << 35) - (1ull << 20);     // lean region offsets: 32-bit, 8-byte units
    c->reg_cap = std::min(c->reg_cap, REG_CAP_MAX);

    for (int attempt = 0; attempt < 8; ++attempt)
    {
        if (!c->arena.ensure(sizeof(uint32_t) * c->key_cap)) return c->fail(AD_E_NOMEM, "key arena %llu", (unsigned long long)c->key_cap);
        if (!c->rarena.ensure(sizeof(uint64_t) * c->rng_cap)) return c->fail(AD_E_NOMEM, "range arena");
        if (!c->scratch.ensure(c->scr_cap)) return c->fail(AD_E_NOMEM, "scratch");
        if (!c->reg.ensure(c->reg_cap)) return c->fail(AD_E_NOMEM, "region arena");
        b.arena = c->arena.as<uint32_t>();
        b.rarena = c->rarena.as<uint64_t>();
        b.scratch = c->scratch.as<uint8_t>();
        b.reg = c->reg.as<uint8_t>();
        BatchCtl h{};
        h.key_cap = c->key_cap;
        h.rng_cap = c->rng_cap;
        h.scr_cap = c->scr_cap;
        h.reg_cap = c->reg_cap;
        // the fused path's k_prepare writes the control block itself (one host copy less per batch);
        // every other path gets it copied
        if (recovery_scan < 0 && !split_only && n)
        {
            b.ctl_init = 1;
            b.init_cap[0] = h.key_cap;
            b.init_cap[1] = h.rng_cap;
            b.init_cap[2] = h.scr_cap;
            b.init_cap[3] = h.reg_cap;
        }
        else
            HIPCHK(c, h2d(b.ctl, &h, sizeof(h), st));
        HIPCHK(c, hipEventRecord(c->ev[0], st));
        uint64_t nd = 0;
        int rc;
        bool lean_track = false;    // this batch's lean pass 1 feeds lean_wide1_update
        uint32_t lean_rpw = 0, lean_fl = 0;   // the lean kernels that ran (ad_stats.lean_rpw1 / lean_flags)
        // the fused path's stage split (prepare, lean pass 1, pass 2, general kernel) costs three more
        // event records (~4 us of idle GPU each); without AD_STAGE_EVENTS=1 stage 0 holds the whole resolve
        const char* se = getenv("AD_STAGE_EVENTS");
        const bool split_stages = se && atoi(se) != 0;
        if (recovery_scan >= 0)
        {
            HIPCHK(c, run_recovery(c->ds, *rv, b, (uint32_t)recovery_scan, st));
            HIPCHK(c, hipEventRecord(c->ev[1], st));
        }
        else if (split_only)
        {
            if ((rc = run_split(c, b, st))) return rc;
            HIPCHK(c, hipEventRecord(c->ev[1], st));
        }
        else
        {
            if (!c->ev_slot) HIPCHK(c, timing_event(&c->ev_slot));
            if (!c->ev_lean) HIPCHK(c, timing_event(&c->ev_lean));
            HIPCHK(c, run_prepare(c->ds, b, st));
            b.ctl_init = 0;
            if (split_stages) HIPCHK(c, hipEventRecord(c->ev_slot, st));
            if (lean)
            {
                // lean kernel first (newest requests, 2 per wave); the general fused kernel then
                // takes only what it deferred (count read on the device, no host round trip)
                if (!c->ev_lean1) HIPCHK(c, timing_event(&c->ev_lean1));
                const uint32_t rpw1 = lean_rpw1(n, np);
                if (gb)
                {
                    // gather + build (k_lean_gather, k_lean_build): the rest to the general kernel
                    HIPCHK(c, run_lean_gb(c->ds, b, st));
                    if (split_stages) HIPCHK(c, hipEventRecord(c->ev_lean1, st));
                    if (split_stages) HIPCHK(c, hipEventRecord(c->ev_lean, st));
                }
                else
                {
                    const bool wide1 = rpw1 == 2 && !c->ds.n_rent && lean_wide1(c);
                    c->lean_ran_wide = wide1;
                    lean_track = rpw1 == 2 && !c->ds.n_rent;
                    lean_rpw = rpw1;
                    lean_fl = (wide1 ? AD_LEAN_WIDE1 : 0u) | (c->ds.n_rent ? AD_LEAN_RANGES : 0u) | (wide1 ? 0u : AD_LEAN_PASS2);
                    HIPCHK(c, run_resolve_lean(c->ds, b, 1, rpw1, wide1, st));
                    if (split_stages) HIPCHK(c, hipEventRecord(c->ev_lean1, st));
                    // after a wide pass 1 the pass-2 list is empty (it serves what pass 2 would, up to 64 raw
                    // emissions, and hands the rest straight to the general kernel): no launch
                    if (!wide1) HIPCHK(c, run_resolve_lean(c->ds, b, 2, rpw1, false, st));
                    if (split_stages) HIPCHK(c, hipEventRecord(c->ev_lean, st));
                }
                if (getenv("AD_DEFER_SPLIT"))
                    HIPCHK(c, run_defer_append(b, st));
                else
                {
                    BatchBufs b2 = b;
                    b2.req_list = b.deferred2;
                    b2.req_count = &b.ctl->n_deferred2;
                    HIPCHK(c, run_resolve(c->ds, b2, st));
                }
            }
            else
                HIPCHK(c, run_resolve(c->ds, b, st));
            HIPCHK(c, hipEventRecord(c->ev[1], st));
        }
        if (!c->h_ctl) HIPCHK(c, hipHostMalloc((void**)&c->h_ctl, sizeof(BatchCtl), hipHostMallocDefault));
        if (!c->ev_sp0) HIPCHK(c, timing_event(&c->ev_sp0));
        if (!c->ev_sp1) HIPCHK(c, timing_event(&c->ev_sp1));
        // offsets + totals + packed arrays (tile sums, their scan, streaming per-tile scan + pack), the
        // packed arrays sized beforehand (grown to the totals and packed again when too small): the
        // only host round trip of a batch is the final read of the control block
        const uint64_t tiles = lb_tiles(n);
        if (!ens<uint64_t>(c->lb_agg, 9 * tiles) || !ens<uint64_t>(c->lb_inc, 9 * tiles))
            return c->fail(AD_E_NOMEM, "tile sums");
        b.lb_agg = c->lb_agg.as<uint64_t>();
        b.lb_inc = c->lb_inc.as<uint64_t>();
        auto bind_outputs = [&]() -> int {
            for (int m = 0; m < 3; ++m)
            {
                if (!ens<int64_t>(c->o_keys[m], c->o_cap[3 * m]) || !ens<uint32_t>(c->o_txns[m], c->o_cap[3 * m + 1]) ||
                    !ens<int32_t>(c->o_k2t[m], c->o_cap[3 * m + 2]))
                    return c->fail(AD_E_NOMEM, "outputs");
                b.o_keys[m] = c->o_keys[m].as<int64_t>();
                b.o_txns[m] = c->o_txns[m].as<uint32_t>();
                b.o_k2t[m] = c->o_k2t[m].as<int32_t>();
            }
            for (int a = 0; a < 9; ++a) b.o_cap[a] = parts_only ? 0 : c->o_cap[a];
            return 0;
        };
        if (!parts_only)
        {
            // first use: keys <= probes per map; ids and keysToTxnIds a guess (grown on overflow)
            for (int m = 0; m < 3; ++m)
            {
                c->o_cap[3 * m] = std::max<uint64_t>(c->o_cap[3 * m], np);
                c->o_cap[3 * m + 1] = std::max<uint64_t>(c->o_cap[3 * m + 1], 2 * np);
                c->o_cap[3 * m + 2] = std::max<uint64_t>(c->o_cap[3 * m + 2], 4 * np);
            }
            if ((rc = bind_outputs())) return rc;
        }
        // stage events: the first pack pass is timed from ev[1] (the resolve's end; one event less per
        // batch -- each record still costs ~4 us of idle GPU), a re-run from its own ev[4]
        int n_pack = 0;
        auto pack_pass = [&]() -> int {
            if (n_pack++ > 0) HIPCHK(c, hipEventRecord(c->ev[4], st));
            HIPCHK(c, run_pack_lb(b, !parts_only, st));
            HIPCHK(c, hipEventRecord(c->ev[5], st));
            HIPCHK(c, d2h(c->h_ctl, b.ctl, sizeof(BatchCtl), st));
            HIPCHK(c, batch_wait(c, st));
            h = *c->h_ctl;
            return 0;
        };
        if ((rc = pack_pass())) return rc;
        double ms_split = 0;
        if (!split_only)
        {
            nd = h.n_deferred;
            if (nd && !h.error && !(h.overflow & 8u))
            {
                HIPCHK(c, hipEventRecord(c->ev_sp0, st));
                // deferred requests: gather a sub-batch, resolve it with the split kernels, scatter back
                if (!ens<uint32_t>(c->s_cnt, nd) || !ens<uint64_t>(c->s_ko, nd + 1))
                    return c->fail(AD_E_NOMEM, "deferred buffers");
                HIPCHK(c, run_defer_counts(b, b.deferred, nd, c->s_cnt.as<uint32_t>(), st));
                HIPCHK(c, run_scan_arrays(c->s_cnt.as<uint32_t>(), c->s_ko.as<uint64_t>(), nd, 1, b.bsum, st));
                uint64_t snp = 0;
                HIPCHK(c, d2h(&snp, c->s_ko.as<uint64_t>() + nd, sizeof(uint64_t), st));
                HIPCHK(c, hipStreamSynchronize(st));
                BatchBufs sb = b;
                sb.n_txns = nd;
                sb.n_probes = snp;
                if (!bind_split(c->sub, sb, nd, snp, true) || !ens<uint64_t>(c->s_tm, nd) || !ens<uint64_t>(c->s_tl, nd) ||
                    !ens<int32_t>(c->s_tn, nd) || !ens<uint64_t>(c->s_em, nd) || !ens<uint64_t>(c->s_el, nd) ||
                    !ens<int32_t>(c->s_en, nd) || !ens<int64_t>(c->s_me, nd) || !ens<int64_t>(c->s_k, snp) ||
                    (b.p_kind && (!ens<int64_t>(c->s_khi, snp) || !ens<uint8_t>(c->s_kind, snp))))
                    return c->fail(AD_E_NOMEM, "deferred buffers");
                uint64_t* sko = c->s_ko.as<uint64_t>();     // the scanned counts are the sub-batch key_off
                HIPCHK(c, run_defer_gather(b, b.deferred, nd, c->s_ko.as<uint64_t>(), sb, c->s_tm.as<uint64_t>(),
                                           c->s_tl.as<uint64_t>(), c->s_tn.as<int32_t>(), c->s_em.as<uint64_t>(),
                                           c->s_el.as<uint64_t>(), c->s_en.as<int32_t>(), c->s_me.as<int64_t>(), sko,
                                           c->s_k.as<int64_t>(), b.p_kind ? c->s_khi.as<int64_t>() : nullptr,
                                           b.p_kind ? c->s_kind.as<uint8_t>() : nullptr, st));
                sb.q_txn_msb = c->s_tm.as<uint64_t>(); sb.q_txn_lsb = c->s_tl.as<uint64_t>(); sb.q_txn_node = c->s_tn.as<int32_t>();
                sb.q_exec_msb = c->s_em.as<uint64_t>(); sb.q_exec_lsb = c->s_el.as<uint64_t>(); sb.q_exec_node = c->s_en.as<int32_t>();
                sb.q_min_epoch = b.q_min_epoch ? c->s_me.as<int64_t>() : nullptr;
                sb.q_key_off = sko;
                sb.q_keys = c->s_k.as<int64_t>();
                sb.q_keys_hi = b.p_kind ? c->s_khi.as<int64_t>() : nullptr;
                sb.p_kind = b.p_kind ? c->s_kind.as<uint8_t>() : nullptr;
                if ((rc = run_split(c, sb, st))) return rc;
                HIPCHK(c, run_defer_scatter(b, b.deferred, nd, sb.sz, sb.t_reg, st));
                // the requests are complete now: pack (k_pack_lb skips batches with split deferrals)
                HIPCHK(c, hipMemsetAsync(&b.ctl->n_deferred, 0, sizeof(unsigned long long), st));
                HIPCHK(c, hipEventRecord(c->ev_sp1, st));
                if ((rc = pack_pass())) return rc;
                float msp = 0;
                HIPCHK(c, hipEventElapsedTime(&msp, c->ev_sp0, c->ev_sp1));
                ms_split = msp;
            }
        }
        if (h.error)
        {
            if (h.error == ERR_STATE)
                return c->fail(AD_E_STATE, "reference would throw: prunedBefore set but no committed Write to substitute (CommandsForKey.java:955-962)");
            return c->fail(AD_E_INVAL, recovery_scan >= 0 ? "invalid Txn.Kind for witnessedBy() in a request (Txn.java:247-262)"
                                                          : "invalid Txn.Kind for witnesses() in a request (Txn.java:221-235)");
        }
        if (h.overflow & 15u)
        {
            if (h.overflow & 1u) c->key_cap = std::max<uint64_t>(c->key_cap * 2, h.key_top + (h.key_top >> 1));
            if (h.overflow & 2u) c->rng_cap = std::max<uint64_t>(c->rng_cap * 2, h.rng_top + (h.rng_top >> 1));
            if (h.overflow & 4u) c->scr_cap = std::max<uint64_t>(c->scr_cap * 2, h.scr_top + (h.scr_top >> 1));
            if (h.overflow & 8u)
            {
                if (c->reg_cap >= REG_CAP_MAX) return c->fail(AD_E_CAPACITY, "batch output beyond the 32 GB region arena");
                c->reg_cap = std::min<uint64_t>(std::max<uint64_t>(c->reg_cap * 2, h.reg_top + (h.reg_top >> 1)), REG_CAP_MAX);
            }
            continue;
        }
        if (h.overflow & OVF_PACK)
        {
            // packed arrays too small: grow them to the totals (with slack for the next batches), pack again
            for (int a = 0; a < 9; ++a) c->o_cap[a] = std::max<uint64_t>(c->o_cap[a], h.tot[a] + h.tot[a] / 4);
            if ((rc = bind_outputs())) return rc;
            HIPCHK(c, hipMemsetAsync(&b.ctl->overflow, 0, sizeof(unsigned int), st));
            if ((rc = pack_pass())) return rc;
            if (h.overflow) return c->fail(AD_E_DEVICE, "pack overflow after growing the outputs to the totals");
        }
        uint64_t tot[9];
        for (int a = 0; a < 9; ++a) tot[a] = h.tot[a];
        // the regions of this batch, for ad_parts_export of a parts-only result
        c->last_reg = b.reg;
        c->last_t_reg = b.t_reg;
        c->last_n = n;
        c->last_parts_only = parts_only;

        ad_stats& S = out->stats;
        memset(&S, 0, sizeof(S));
        S.n_txns = n;
        S.n_probes = np;
        S.n_deferred = nd;
        S.n_deferred_lean = lean ? h.n_real2 : 0;     // requests the lean passes left to the general kernel
        S.n_lean_pass2 = lean ? h.n_real1 : 0;        // requests lean pass 1 left to pass 2
        S.n_launches = lean_track && c->lean_ran_wide ? 1 : 0;   // lean pass 1 ran its wide kernel
        S.lean_rpw1 = lean_rpw;
        S.lean_flags = lean_fl;
        if (lean_track) lean_wide1_update(c, n, h);
        for (int m = 0; m < 3; ++m)
        {
            S.n_pairs[m] = tot[3 * m + 2] - tot[3 * m + 0];
            S.n_unique[m] = tot[3 * m + 1];
            S.n_keys[m] = tot[3 * m + 0];
        }
        float ms;
        // stage 0: the resolve (ev[0] -> ev[1]); 5: offsets + pack (the last pack pass); 1 and 4 (the gap
        // before the offsets scan, the scan itself inside the pack pass) are 0 since no event splits them
        double total = 0;
        HIPCHK(c, hipEventElapsedTime(&ms, c->ev[0], c->ev[1]));
        S.ms_stage[0] = ms;
        total += ms;
        HIPCHK(c, hipEventElapsedTime(&ms, c->ev[n_pack > 1 ? 4 : 1], c->ev[5]));
        S.ms_stage[5] = ms;
        total += ms;
        if (!split_only && split_stages)
        {
            // stage 2: k_prepare; stage 0: k_resolve_lean (or k_resolve when not lean);
            // stage 3: k_resolve over the lean kernel's deferrals
            HIPCHK(c, hipEventElapsedTime(&ms, c->ev[0], c->ev_slot));
            S.ms_stage[2] = ms;
            S.ms_stage[0] -= ms;
            if (lean)
            {
                // stage 0: lean pass 1 (k_resolve_lean<2>), 3: lean pass 2 (k_resolve_lean<1>),
                // 6: the general kernel on what both passes deferred
                float m1 = 0, m2 = 0;
                HIPCHK(c, hipEventElapsedTime(&m1, c->ev_slot, c->ev_lean1));
                HIPCHK(c, hipEventElapsedTime(&m2, c->ev_lean1, c->ev_lean));
                S.ms_stage[6] = S.ms_stage[0] - m1 - m2;
                S.ms_stage[0] = m1;
                S.ms_stage[3] = m2;
            }
        }
        S.ms_stage[1] += ms_split;           // split kernels on the fused kernels' deferrals (+ offsets re-run)
        total += ms_split;
        S.ms_device = total;
        S.ms_ingest = c->ms_ingest;
        out->n_txns = n;
        out->regions = b.reg;
        out->regions_bytes = h.reg_top;
        out->region_bytes = 0;
        for (int m = 0; m < 3; ++m)
        {
            out->region_off[m] = b.t_reg + (uint64_t)m * n;
            out->region_bytes += 8 * tot[3 * m + 0] + 4 * tot[3 * m + 1] + 4 * tot[3 * m + 2];
            out->keys_off[m] = b.off + (uint64_t)(3 * m + 0) * (n + 1);
            out->txn_off[m] = b.off + (uint64_t)(3 * m + 1) * (n + 1);
            out->k2t_off[m] = b.off + (uint64_t)(3 * m + 2) * (n + 1);
            out->keys[m] = parts_only ? nullptr : b.o_keys[m];
            out->txns[m] = parts_only ? nullptr : b.o_txns[m];
            out->k2t[m] = parts_only ? nullptr : b.o_k2t[m];
        }
        return 0;
    }
    return c->fail(AD_E_NOMEM, "arena growth did not converge");
}

template <class T>
static T* stage_q(ad_ctx* c, DevBuf& b, const T* src, uint64_t n, int* rc)
{
    if (!src) return nullptr;
    if (!b.ensure(sizeof(T) * std::max<uint64_t>(n, 1))) { *rc = c->fail(AD_E_NOMEM, "query staging"); return nullptr; }
    if (n && h2d(b.p, src, sizeof(T) * n, c->stream) != hipSuccess)
    {
        *rc = c->fail(AD_E_DEVICE, "query H2D");
        return nullptr;
    }
    return b.as<T>();
}

// A library-owned host result array (released by free() in ad_result_free). Large ones are 2 MB aligned
// and advised as transparent huge pages: the copy-out then first-touches a few hundred pages instead of
// ~90k 4 KB ones per config-2 batch (the page faults were most of ad_deps_batch's host time).
static void* host_result_alloc(size_t bytes)
{
    constexpr size_t HUGE = 2u << 20;
    if (bytes < 4 * HUGE) return malloc(bytes);
    void* p = nullptr;
    const size_t rounded = (bytes + HUGE - 1) & ~(HUGE - 1);
    if (posix_memalign(&p, HUGE, rounded) != 0) return nullptr;
    (void)madvise(p, rounded, MADV_HUGEPAGE);
    return p;
}

// one array of a device result into a library-owned host array (n elements, n <= bound), checked
template <class T>
static int d2h(ad_ctx* c, T** out, const T* src, uint64_t n, uint64_t bound, const char* what, int m)
{
    if (n > bound)
        return c->fail(AD_E_DEVICE, "result %s of map %d: %llu elements, beyond the batch total %llu", what, m,
                       (unsigned long long)n, (unsigned long long)bound);
    T* p = (T*)host_result_alloc(sizeof(T) * std::max<uint64_t>(n, 1));
    if (!p) return c->fail(AD_E_NOMEM, "result %s of map %d: %llu elements", what, m, (unsigned long long)n);
    *out = p;
    if (n)
    {
        const hipError_t e = copy_sync(p, src, sizeof(T) * n, hipMemcpyDeviceToHost);
        if (e != hipSuccess) return c->fail(AD_E_DEVICE, "result %s of map %d: %s", what, m, hipGetErrorString(e));
    }
    return 0;
}

// A device result (packed arrays) into a library-owned host result. Every copy is checked and every
// array length is bounded by the batch totals the pipeline reported (ad_stats); the offsets must start
// at 0 and end exactly at those totals, else AD_E_DEVICE names the map and the array (nothing is
// sized from a value the checks have not accepted).
static int result_to_host(ad_ctx* c, uint64_t n, const ad_deps_result& dev, ad_deps_result** out)
{
    ad_deps_result* r = (ad_deps_result*)calloc(1, sizeof(ad_deps_result));
    if (!r) return c->fail(AD_E_NOMEM, "result");
    r->n_txns = n;
    r->stats = dev.stats;
    auto run = [&]() -> int {
        for (int m = 0; m < 3; ++m)
        {
            const uint64_t tot[3] = {dev.stats.n_keys[m], dev.stats.n_unique[m], dev.stats.n_pairs[m] + dev.stats.n_keys[m]};
            const char* names[3] = {"keys", "txnIds", "keysToTxnIds"};
            uint64_t** offs[3] = {&r->keys_off[m], &r->txn_off[m], &r->k2t_off[m]};
            const uint64_t* src_off[3] = {dev.keys_off[m], dev.txn_off[m], dev.k2t_off[m]};
            for (int a = 0; a < 3; ++a)
            {
                if (int rc = d2h(c, offs[a], src_off[a], n + 1, n + 1, names[a], m)) return rc;
                const uint64_t* o = *offs[a];
                if (o[0] != 0 || o[n] != tot[a])
                    return c->fail(AD_E_DEVICE, "result offsets of %s, map %d: [0] = %llu, [n] = %llu, batch total %llu", names[a],
                                   m, (unsigned long long)o[0], (unsigned long long)o[n], (unsigned long long)tot[a]);
            }
            if (int rc = d2h(c, &r->keys[m], dev.keys[m], tot[0], tot[0], names[0], m)) return rc;
            if (int rc = d2h(c, &r->txns[m], dev.txns[m], tot[1], tot[1], names[1], m)) return rc;
            if (int rc = d2h(c, &r->k2t[m], dev.k2t[m], tot[2], tot[2], names[2], m)) return rc;
        }
        return 0;
    };
    if (int rc = run())
    {
        ad_result_free(r);
        return rc;
    }
    *out = r;
    return AD_OK;
}

static int check_query_host(ad_ctx* c, const ad_query_soa* q, uint32_t flags = 0)
{
    if (q->range_off && q->n_txns)
    {
        // Range-domain requests: ranges normalised (accord.primitives.Ranges), no keys beside them,
        // SNAPSHOT semantics only
        if (!q->range_start || !q->range_end)
            return c->fail(AD_E_INVAL, "range_off without range_start / range_end");
        for (uint64_t i = 0; i < q->n_txns; ++i)
        {
            const uint64_t r0 = q->range_off[i], r1 = q->range_off[i + 1];
            if (r1 < r0) return c->fail(AD_E_INVAL, "request %llu: range_off not monotone", (unsigned long long)i);
            if (r1 == r0) continue;
            if (q->key_off[i + 1] != q->key_off[i])
                return c->fail(AD_E_INVAL, "request %llu has keys and ranges (a request is key- or Range-domain)", (unsigned long long)i);
            for (uint64_t j = r0; j < r1; ++j)
                if (q->range_start[j] >= q->range_end[j] || (j > r0 && q->range_end[j - 1] > q->range_start[j]))
                    return c->fail(AD_E_INVAL, "request %llu: ranges not normalised (start < end, ascending, disjoint)",
                                   (unsigned long long)i);
        }
    }
    // host threads over request ranges; the lowest offending request is reported
    std::atomic<uint64_t> bad{~0ull};
    parallel_for(q->n_txns, [&](size_t a, size_t b) {
        for (uint64_t i = a; i < b; ++i)
        {
            bool ok = q->key_off[i] <= q->key_off[i + 1];
            for (uint64_t k = q->key_off[i] + 1; ok && k < q->key_off[i + 1]; ++k) ok = q->keys[k - 1] < q->keys[k];
            if (!ok)
            {
                uint64_t cur = bad.load();
                while (i < cur && !bad.compare_exchange_weak(cur, i)) {}
                return;
            }
        }
    }, 1 << 15);
    if (bad.load() != ~0ull)
        return c->fail(AD_E_INVAL, "request %llu: keys not strictly ascending", (unsigned long long)bad.load());
    return 0;
}

}  // namespace

// =======================================================================================
// C ABI
// =======================================================================================
extern "C" {

int ad_abi_version(void) { return AD_ABI_VERSION; }

static thread_local std::string g_create_err;

int ad_ctx_create(const ad_config* cfg, ad_ctx** out)
{
    if (!cfg || !out) return AD_E_INVAL;
    ad_ctx* c = new (std::nothrow) ad_ctx();
    if (!c) return AD_E_NOMEM;
    hipError_t e;
    c->cfg = *cfg;
    for (uint64_t i = 0; i < cfg->n_slices; ++i)
    {
        // the store's Ranges, normalised (start < end, ascending, disjoint): Range-domain requests are
        // sliced against them in order
        if (cfg->slice_start[i] >= cfg->slice_end[i] || (i > 0 && cfg->slice_end[i - 1] > cfg->slice_start[i]))
        {
            g_create_err = "ad_ctx_create: slices not normalised (start < end, ascending, disjoint)";
            delete c;
            return AD_E_INVAL;
        }
        c->slice_s.push_back(cfg->slice_start[i]);
        c->slice_e.push_back(cfg->slice_end[i]);
    }
    c->cfg.slice_start = nullptr;
    c->cfg.slice_end = nullptr;
    c->device = cfg->device;
    if ((e = hipSetDevice(c->device)) != hipSuccess || (e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking)) != hipSuccess)
    {
        g_create_err = std::string("ad_ctx_create: ") + hipGetErrorName(e) + ": " + hipGetErrorString(e);
        delete c;
        return AD_E_DEVICE;
    }
    for (auto& ev : c->ev)
        if ((e = timing_event(&ev)) != hipSuccess)
        {
            g_create_err = std::string("ad_ctx_create: hipEventCreate: ") + hipGetErrorString(e);
            delete c;
            return AD_E_DEVICE;
        }
    *out = c;
    return AD_OK;
}

void ad_ctx_destroy(ad_ctx* c)
{
    if (!c) return;
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    for (auto& e : c->ev)
        if (e) (void)hipEventDestroy(e);
    if (c->ev_slot) (void)hipEventDestroy(c->ev_slot);
    if (c->ev_lean) (void)hipEventDestroy(c->ev_lean);
    if (c->ev_lean1) (void)hipEventDestroy(c->ev_lean1);
    if (c->ev_done) (void)hipEventDestroy(c->ev_done);
    if (c->ev_sp0) (void)hipEventDestroy(c->ev_sp0);
    if (c->ev_sp1) (void)hipEventDestroy(c->ev_sp1);
    if (c->h_ctl) (void)hipHostFree(c->h_ctl);
    if (c->h_small) (void)hipHostFree(c->h_small);
    for (int k = 0; k < 2; ++k)
    {
        if (c->up_busy[k]) (void)hipEventSynchronize(c->ev_up[k]);     // a copy on a caller's stream
        if (c->ev_up[k]) (void)hipEventDestroy(c->ev_up[k]);
        if (c->h_up[k]) (void)hipHostFree(c->h_up[k]);
    }
    if (c->h_rb) (void)hipHostFree(c->h_rb);
    if (c->h_xtab) (void)hipHostFree(c->h_xtab);
    if (c->ev_ready) (void)hipEventDestroy(c->ev_ready);
    for (hipEvent_t e : c->ev_copied)
        if (e) (void)hipEventDestroy(e);
    if (c->cstream) (void)hipStreamDestroy(c->cstream);
    for (void* p : c->in_pin)
        if (p) (void)hipHostFree(p);
    for (auto& b : c->w_pin)
        for (void* p : b)
            if (p) (void)hipHostFree(p);
    for (hipEvent_t e : c->ev_h2d)
        if (e) (void)hipEventDestroy(e);
    if (c->hstream) (void)hipStreamDestroy(c->hstream);
    for (hipEvent_t e : c->x_ev)
        if (e) (void)hipEventDestroy(e);
    if (c->lv) levels_work_destroy(c->lv);
    if (c->cu) cfk_upd_work_destroy(c->cu);
    if (c->ing) ingest_work_destroy(c->ing);
    if (c->comm) (void)ncclCommDestroy(c->comm);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

const char* ad_last_error(const ad_ctx* c) { return c ? c->err.c_str() : g_create_err.c_str(); }

int ad_cfk_load(ad_ctx* c, const ad_cfk_soa* in)
{
    if (!c || !in) return AD_E_INVAL;
    auto& K = c->cfk;
    const uint64_t nk = in->n_keys, ne = in->n_entries;
    if ((nk && (!in->keys || !in->seg)) || (!nk && ne)) return c->fail(AD_E_INVAL, "bad cfk soa");
    if (nk && in->seg[nk] != ne) return c->fail(AD_E_INVAL, "seg[n_keys] != n_entries");
    K.keys.assign(in->keys, in->keys + nk);
    K.seg.assign(nk + 1, 0);
    if (nk) std::copy(in->seg, in->seg + nk + 1, K.seg.begin());
    for (uint64_t k = 0; k < nk; ++k)
        if (K.seg[k] > K.seg[k + 1]) return c->fail(AD_E_INVAL, "seg not monotone");
    K.status.assign(in->status, in->status + ne);
    K.pruned.clear();
    if (in->pruned_before) K.pruned.assign(in->pruned_before, in->pruned_before + nk);
    // the byId ids go to HBM as they are (the device ingest reads them there; the host copy is read
    // back only when a host path needs it); AD_INGEST_HOST keeps the host ingest
    c->raw_dev = false;
    if (getenv("AD_INGEST_HOST") == nullptr)
    {
        if (hipSetDevice(c->device) != hipSuccess) return c->fail(AD_E_DEVICE, "hipSetDevice");
        StreamScope scope_(c->stream, c->cstream);
        auto up = [&](DevBuf& b, const void* src, size_t bytes) -> int {
            if (!b.ensure(std::max<size_t>(bytes, 8))) return c->fail(AD_E_NOMEM, "hipMalloc %zu (snapshot columns)", bytes);
            // ordered on the ctx stream (non-blocking: a null-stream copy would not wait for its kernels)
            if (bytes) HIPCHK(c, h2d(b.p, src, bytes, c->stream));
            return 0;
        };
        int rc;
        if ((rc = up(c->d_keys, in->keys, 8 * nk)) || (rc = up(c->d_in_seg, in->seg, 8 * (nk + 1))) ||
            (rc = up(c->d_in_tm, in->txn_msb, 8 * ne)) || (rc = up(c->d_in_tl, in->txn_lsb, 8 * ne)) ||
            (rc = up(c->d_in_tn, in->txn_node, 4 * ne)) || (rc = up(c->d_in_em, in->exec_msb, 8 * ne)) ||
            (rc = up(c->d_in_el, in->exec_lsb, 8 * ne)) || (rc = up(c->d_in_en, in->exec_node, 4 * ne)) ||
            (rc = up(c->d_status, in->status, ne)) ||
            (in->pruned_before && (rc = up(c->d_in_pruned, in->pruned_before, 8 * nk))))
            return rc;
        HIPCHK(c, hipStreamSynchronize(c->stream));     // the caller's arrays are free to go on return
        K.txn.clear();
        K.exec.clear();
        c->raw_dev = true;
        c->raw_ne = ne;
    }
    else
    {
        K.txn.resize(ne);
        K.exec.resize(ne);
        parallel_for(ne, [&](size_t a, size_t b) {
            for (size_t e = a; e < b; ++e)
            {
                K.txn[e] = {in->txn_msb[e], in->txn_lsb[e], in->txn_node[e]};
                K.exec[e] = {in->exec_msb[e], in->exec_lsb[e], in->exec_node[e]};
            }
        });
    }
    K.miss_off.clear();
    K.miss.clear();
    K.miss_stale = false;
    K.ballot.clear();
    c->d_ballot.release();
    c->d_ballot2.release();
    c->dmiss_on = false;
    c->d_mref.release();
    c->d_mref2.release();
    K.loaded = true;
    c->host_stale = false;       // the load replaces whatever ad_cfk_update applied on the device
    c->host_moved = false;
    c->host_dict_stale = false;
    c->host_ingested = false;
    drop_global_dict(c);         // a new snapshot: the node-wide dictionary must be installed again
    c->dirty = true;
    return AD_OK;
}

int ad_range_cmds_load(ad_ctx* c, const ad_range_cmds_soa* in)
{
    if (!c || !in) return AD_E_INVAL;
    auto& R = c->cmds;
    const uint64_t n = in->n_cmds;
    R.txn.resize(n);
    for (uint64_t i = 0; i < n; ++i) R.txn[i] = {in->txn_msb[i], in->txn_lsb[i], in->txn_node[i]};
    R.erased.clear();
    R.historical.clear();
    if (in->erased) R.erased.assign(in->erased, in->erased + n);
    if (in->historical) R.historical.assign(in->historical, in->historical + n);
    R.off.assign(in->range_off, in->range_off + n + 1);
    const uint64_t nr = n ? in->range_off[n] : 0;
    R.start.assign(in->range_start, in->range_start + nr);
    R.end.assign(in->range_end, in->range_end + nr);
    R.rec = false;                  // recovery facts belong to the previous commands
    c->rv_gen = ~0ull;
    c->rv_rng_gen = ~0ull;
    drop_global_dict(c);         // a new snapshot: the node-wide dictionary must be installed again
    c->dirty = true;
    return AD_OK;
}

int ad_redundant_load(ad_ctx* c, const ad_redundant_soa* in)
{
    if (!c || !in) return AD_E_INVAL;
    auto& B = c->rb;
    const uint64_t n = in->n;
    B.start.assign(in->range_start, in->range_start + n);
    B.end.assign(in->range_end, in->range_end + n);
    B.e0.assign(in->start_epoch, in->start_epoch + n);
    B.e1.assign(in->end_epoch, in->end_epoch + n);
    B.wm.resize(n);
    for (uint64_t i = 0; i < n; ++i) B.wm[i] = {in->wm_msb[i], in->wm_lsb[i], in->wm_node[i]};
    drop_global_dict(c);         // a new snapshot: the node-wide dictionary must be installed again
    c->dirty = true;
    return AD_OK;
}

int ad_prepare(ad_ctx* c)
{
    if (!c) return AD_E_INVAL;
    if (!c->cfk.loaded) return c->fail(AD_E_NOT_LOADED, "ad_cfk_load not called");
    if (hipSetDevice(c->device) != hipSuccess) return c->fail(AD_E_DEVICE, "hipSetDevice");
    StreamScope scope_(c->stream, c->cstream);
    return c->dirty ? build_snapshot(c) : AD_OK;
}

static int cfk_update_run(ad_ctx* c, const CfkUpdIn& u, hipStream_t st, uint64_t* n_applied, ad_stats* stats);

// SEQUENTIAL PreAccepts as device-side CommandsForKey.update insertions (PREACCEPTED, executeAt =
// txnId) of every request into the CommandsForKey of each of its keys in the slice, as
// apply_preaccepts does on the host (keys without a CommandsForKey and older ids included). Returns
// 0 (applied), 1 (not applicable here: no built snapshot, or a batch the device path refuses) or an
// AD_E_* error.
static int sequential_on_device(ad_ctx* c, const ad_query_soa* q)
{
    if (c->dirty || getenv("AD_SEQ_HOST")) return 1;
    // Range-domain requests register as range commands, whose part of the snapshot is host-built: the
    // host route (apply_preaccepts + rebuild)
    if (q->n_txns && q->range_off && q->range_off[q->n_txns] > q->range_off[0]) return 1;
    std::vector<int64_t> keys;
    std::vector<uint64_t> tm, tl;
    std::vector<int32_t> tn;
    for (uint64_t i = 0; i < q->n_txns; ++i)
    {
        const Tid t{q->txn_msb[i], q->txn_lsb[i], q->txn_node[i]};
        const Tid x{q->exec_msb[i], q->exec_lsb[i], q->exec_node[i]};
        if (!(t.msb == x.msb && ((t.lsb ^ x.lsb) & 0xFFFFFFFFFFFF001EULL) == 0 && t.node == x.node))
            return c->fail(AD_E_INVAL, "SEQUENTIAL (PreAccept) requests need executeAt == txnId");
        if (i > 0)
        {
            const Tid p{q->txn_msb[i - 1], q->txn_lsb[i - 1], q->txn_node[i - 1]};
            if (norm_cmp(norm(p), norm(t)) >= 0) return c->fail(AD_E_INVAL, "SEQUENTIAL requests must be in ascending TxnId order");
        }
        const uint32_t kind = (uint32_t)((t.lsb >> 1) & 7);
        if (!((t.lsb & 1) == 0 && ((KINDS_ANY_GLOBALLY_VISIBLE >> kind) & 1))) continue;   // CommandsForKey.manages
        for (uint64_t k = q->key_off[i]; k < q->key_off[i + 1]; ++k)
        {
            const int64_t key = q->keys[k];
            bool in = c->slice_s.empty();
            for (size_t s = 0; s < c->slice_s.size() && !in; ++s)
                in = range_contains(c->cfg.range_start_inclusive, c->slice_s[s], c->slice_e[s], key);
            if (!in) continue;
            keys.push_back(key);
            tm.push_back(t.msb);
            tl.push_back(t.lsb);
            tn.push_back(t.node);
        }
    }
    if (keys.empty()) return 0;
    std::vector<uint8_t> st(keys.size(), AD_ST_PREACCEPTED_OR_ACCEPTED_INVALIDATE);
    const uint64_t n = keys.size();
    int rc = 0;
    CfkUpdIn in{n, stage_q(c, c->u_k, keys.data(), n, &rc), stage_q(c, c->u_tm, tm.data(), n, &rc),
                stage_q(c, c->u_tl, tl.data(), n, &rc), stage_q(c, c->u_tn, tn.data(), n, &rc), nullptr, nullptr, nullptr,
                stage_q(c, c->u_st, st.data(), n, &rc)};
    if (rc) return rc;
    in.exec_msb = in.txn_msb;
    in.exec_lsb = in.txn_lsb;
    in.exec_node = in.txn_node;
    rc = cfk_update_run(c, in, c->stream, nullptr, nullptr);
    if (rc == AD_E_INVAL || rc == AD_E_STATE) return 1;
    return rc;
}

int ad_deps_batch(ad_ctx* c, const ad_query_soa* q, uint32_t flags, ad_deps_result** out)
{
    if (!c || !q || !out) return AD_E_INVAL;
    if (!c->cfk.loaded) return c->fail(AD_E_NOT_LOADED, "ad_cfk_load not called");
    if (hipSetDevice(c->device) != hipSuccess) return c->fail(AD_E_DEVICE, "hipSetDevice");
    StreamScope scope_(c->stream, c->cstream);
    int rc = check_query_host(c, q, flags);
    if (rc) return rc;
    if (flags & AD_SEQUENTIAL)
    {
        // on the device when the snapshot holds every key and the batch only appends (§6e);
        // otherwise the host inserts and re-ingests
        rc = sequential_on_device(c, q);
        if (rc < 0) return rc;
        if (rc > 0)
        {
            // keep a copy so a failed batch leaves the snapshot untouched
            if ((rc = sync_host(c))) return rc;
            auto saved = c->cfk;
            auto saved_cmds = c->cmds;
            if ((rc = apply_preaccepts(c, q)))
            {
                c->cfk = saved;
                c->cmds = saved_cmds;
                return rc;
            }
        }
    }
    if (c->dirty && (rc = build_snapshot(c))) return rc;
    const uint64_t n = q->n_txns;
    const uint64_t np = n ? q->key_off[n] : 0;
    ad_query_soa d{};
    d.n_txns = n;
    rc = 0;
    d.txn_msb = stage_q(c, c->q_tm, q->txn_msb, n, &rc);
    d.txn_lsb = stage_q(c, c->q_tl, q->txn_lsb, n, &rc);
    d.txn_node = stage_q(c, c->q_tn, q->txn_node, n, &rc);
    d.exec_msb = stage_q(c, c->q_em, q->exec_msb, n, &rc);
    d.exec_lsb = stage_q(c, c->q_el, q->exec_lsb, n, &rc);
    d.exec_node = stage_q(c, c->q_en, q->exec_node, n, &rc);
    d.min_epoch = stage_q(c, c->q_me, q->min_epoch, n, &rc);
    d.key_off = stage_q(c, c->q_ko, q->key_off, n + 1, &rc);
    d.keys = stage_q(c, c->q_k, q->keys, np, &rc);
    if (n && q->range_off && q->range_off[n] > q->range_off[0])
    {
        const uint64_t r0 = q->range_off[0], nr = q->range_off[n] - r0;
        std::vector<uint64_t> ro(n + 1);
        for (uint64_t i = 0; i <= n; ++i) ro[i] = q->range_off[i] - r0;
        d.range_off = stage_q(c, c->q_ro, ro.data(), n + 1, &rc);
        d.range_start = stage_q(c, c->q_rs, q->range_start + r0, nr, &rc);
        d.range_end = stage_q(c, c->q_re, q->range_end + r0, nr, &rc);
        d.n_ranges = nr;
        if (!rc) HIPCHK(c, hipStreamSynchronize(c->stream));     // ro is a local
    }
    if (rc) return rc;
    ad_deps_result dev{};
    if ((rc = run_pipeline(c, &d, c->stream, &dev))) return rc;
    return result_to_host(c, n, dev, out);
}

int ad_host_register(ad_ctx* c, void* p, uint64_t bytes)
{
    if (!c || !p || !bytes) return AD_E_INVAL;
    if (hipSetDevice(c->device) != hipSuccess) return c->fail(AD_E_DEVICE, "hipSetDevice");
    StreamScope scope_(c->stream, c->cstream);
    HIPCHK(c, hipHostRegister(p, bytes, hipHostRegisterDefault));
    return AD_OK;
}

int ad_host_alloc(uint64_t bytes, void** p)
{
    if (!p) return AD_E_INVAL;
    *p = nullptr;
    if (!bytes) return AD_E_INVAL;
    if (hipHostMalloc(p, bytes, hipHostMallocPortable) != hipSuccess)
    {
        *p = nullptr;
        return AD_E_NOMEM;
    }
    return AD_OK;
}

int ad_host_free(void* p)
{
    if (!p) return AD_OK;
    // no copy may still be landing in the pages
    (void)hipDeviceSynchronize();
    return hipHostFree(p) == hipSuccess ? AD_OK : AD_E_DEVICE;
}

int ad_debug_guard_check(char* buf, uint64_t n)
{
    std::string rep;
    const int bad = dev_guard_check(&rep);
    if (buf && n)
    {
        const size_t k = std::min<size_t>(rep.size(), n - 1);
        memcpy(buf, rep.data(), k);
        buf[k] = 0;
    }
    return bad;
}

int ad_host_unregister(ad_ctx* c, void* p)
{
    if (!p) return AD_E_INVAL;
    if (!c)
    {
        // no ctx (it may be gone already): a registration is process-wide, nothing of a ctx is needed
        return hipHostUnregister(p) == hipSuccess ? AD_OK : AD_E_DEVICE;
    }
    if (hipSetDevice(c->device) != hipSuccess) return c->fail(AD_E_DEVICE, "hipSetDevice");
    StreamScope scope_(c->stream, c->cstream);
    // nothing of this ctx may still be copying into the pages
    if (c->cstream) HIPCHK(c, hipStreamSynchronize(c->cstream));
    HIPCHK(c, hipHostUnregister(p));
    return AD_OK;
}

// ---- ad_deps_batch_into, key-only SNAPSHOT batches: inputs packed by the host worker pool into pinned
// staging (one H2D per slice, the next slice packed while this one resolves; the key-order check is the
// same pass), results copied by a kernel straight into the caller's pinned arrays (CU stores over PCIe run
// beside the SDMA H2D: both directions at once), offsets of maps empty in a slice filled by the pool at
// the end. Pageable output arrays fall back to staged copies.
namespace {

// device-mapped address of pinned (registered or hipHostMalloc'd) host memory p; null: pageable
void* mapped_addr(void* p)
{
    if (!p) return nullptr;
    hipPointerAttribute_t a{};
    if (hipPointerGetAttributes(&a, p) != hipSuccess)
    {
        (void)hipGetLastError();
        return nullptr;
    }
    if (a.type != hipMemoryTypeHost || !a.devicePointer) return nullptr;
    if (a.hostPointer) return (char*)a.devicePointer + ((char*)p - (char*)a.hostPointer);
    return a.devicePointer;
}

struct InLayout {
    uint64_t tm, tl, tn, em, el, en, me, ko, k, bytes;
};

InLayout in_layout(uint64_t nc, uint64_t nk, bool me)
{
    auto al = [](uint64_t x) { return (x + 255) & ~uint64_t(255); };
    InLayout L{};
    uint64_t o = 0;
    L.tm = o; o = al(o + 8 * nc);
    L.tl = o; o = al(o + 8 * nc);
    L.tn = o; o = al(o + 4 * nc);
    L.em = o; o = al(o + 8 * nc);
    L.el = o; o = al(o + 8 * nc);
    L.en = o; o = al(o + 4 * nc);
    L.me = o; o = al(o + (me ? 8 * nc : 0));
    L.ko = o; o = al(o + 8 * (nc + 1));
    L.k = o; o = al(o + 8 * std::max<uint64_t>(nk, 1));
    L.bytes = o;
    return L;
}

// pack requests [lo, hi) into P (layout L) and check them (key_off monotone, keys strictly ascending per
// request): the lowest offending request into *bad
void stage_slice(const ad_query_soa* q, uint64_t lo, uint64_t hi, char* P, const InLayout& L, std::atomic<uint64_t>* bad)
{
    const uint64_t nc = hi - lo;
    const uint64_t k0 = q->key_off[lo], k1 = q->key_off[hi];
    if (k1 < k0)
    {
        uint64_t cur = bad->load();
        while (lo < cur && !bad->compare_exchange_weak(cur, lo)) {}
        return;
    }
    constexpr uint64_t CH = 1 << 14;
    const uint64_t tasks = (nc + CH - 1) / CH;
    host_parallel(tasks, [&](size_t t) {
        const uint64_t a = lo + t * CH, b = std::min(hi, a + CH), m = b - a, r = a - lo;
        memcpy(P + L.tm + 8 * r, q->txn_msb + a, 8 * m);
        memcpy(P + L.tl + 8 * r, q->txn_lsb + a, 8 * m);
        memcpy(P + L.tn + 4 * r, q->txn_node + a, 4 * m);
        memcpy(P + L.em + 8 * r, q->exec_msb + a, 8 * m);
        memcpy(P + L.el + 8 * r, q->exec_lsb + a, 8 * m);
        memcpy(P + L.en + 4 * r, q->exec_node + a, 4 * m);
        if (q->min_epoch) memcpy(P + L.me + 8 * r, q->min_epoch + a, 8 * m);
        uint64_t* ko = (uint64_t*)(P + L.ko) + r;
        uint64_t first_bad = ~0ull;
        for (uint64_t i = a; i <= b; ++i)
        {
            const uint64_t v = q->key_off[i];
            if (v < k0 || v > k1 || (i > a && v < q->key_off[i - 1]))
            {
                first_bad = i > a ? i - 1 : i;
                break;
            }
            if (i < b || b == hi) ko[i - a] = v - k0;
        }
        if (first_bad == ~0ull)
        {
            const uint64_t ka = q->key_off[a], kb = q->key_off[b];
            memcpy(P + L.k + 8 * (ka - k0), q->keys + ka, 8 * (kb - ka));
            for (uint64_t i = a; i < b && first_bad == ~0ull; ++i)
                for (uint64_t k = q->key_off[i] + 1; k < q->key_off[i + 1]; ++k)
                    if (q->keys[k - 1] >= q->keys[k])
                    {
                        first_bad = i;
                        break;
                    }
        }
        if (first_bad != ~0ull)
        {
            uint64_t cur = bad->load();
            while (first_bad < cur && !bad->compare_exchange_weak(cur, first_bad)) {}
        }
    });
}

}  // namespace

static int deps_into_fast(ad_ctx* c, const ad_query_soa* q, ad_deps_result* out, const uint64_t* cap, uint64_t* need,
                          uint32_t slices)
{
    const uint64_t n = q->n_txns;
    const bool trace = getenv("AD_INTO_TRACE") != nullptr;
    const double t_begin = trace ? now_ms() : 0.0;
    hipStream_t st = c->stream;
    if (slices == 0) slices = (uint32_t)std::min<uint64_t>(8, std::max<uint64_t>(1, n >> 17));
    slices = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(slices, std::max<uint64_t>(n, 1)));
    // staging sized for the largest slice
    const bool me = q->min_epoch != nullptr;
    uint64_t max_bytes = 0;
    for (uint32_t j = 0; j < slices; ++j)
    {
        const uint64_t lo = n * j / slices, hi = n * (j + 1) / slices;
        const uint64_t nk = q->key_off[hi] >= q->key_off[lo] ? q->key_off[hi] - q->key_off[lo] : 0;
        max_bytes = std::max(max_bytes, in_layout(hi - lo, nk, me).bytes);
    }
    for (int b = 0; b < 2; ++b)
        if (c->in_pin_cap[b] < max_bytes)
        {
            if (c->in_pin[b]) (void)hipHostFree(c->in_pin[b]);
            c->in_pin[b] = nullptr;
            c->in_pin_cap[b] = 0;
            const size_t want = max_bytes + max_bytes / 8;
            if (hipHostMalloc(&c->in_pin[b], want, hipHostMallocDefault) != hipSuccess)
                return c->fail(AD_E_NOMEM, "ad_deps_batch_into: pinned staging of %zu bytes", want);
            c->in_pin_cap[b] = want;
        }
    for (int b = 0; b < 2; ++b)
    {
        if (!c->in_dev[b].ensure(max_bytes)) return c->fail(AD_E_NOMEM, "ad_deps_batch_into: device staging");
        if (!c->ev_h2d[b]) HIPCHK(c, hipEventCreateWithFlags(&c->ev_h2d[b], hipEventDisableTiming));
    }
    if (!c->hstream) HIPCHK(c, hipStreamCreateWithFlags(&c->hstream, hipStreamNonBlocking));
    StreamScope hscope_(c->hstream, c->stream, c->cstream);
    // the caller's output arrays as device-mapped addresses (null: pageable, staged copies)
    void* dmap[3][6];
    for (int m = 0; m < 3; ++m)
    {
        void* hp[6] = {out->keys_off[m], out->txn_off[m], out->k2t_off[m], out->keys[m], out->txns[m], out->k2t[m]};
        for (int k = 0; k < 6; ++k) dmap[m][k] = mapped_addr(hp[k]);
    }
    struct Fill {
        int m;
        uint64_t lo, hi, b[3];
    };
    uint64_t base[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    bool fits = true;
    ad_stats agg{};
    uint64_t bytes_in = 0, bytes_out = 0;
    std::atomic<uint64_t> bad{~0ull};
    // slice 0 packed and sent here; slice j + 1 packed and sent by a helper thread (packing on the pool,
    // the H2D on hstream into the other device region) while slice j resolves
    auto layout_of = [&](uint32_t j, uint64_t* lo, uint64_t* hi) {
        *lo = n * j / slices;
        *hi = n * (j + 1) / slices;
        const uint64_t nk = q->key_off[*hi] >= q->key_off[*lo] ? q->key_off[*hi] - q->key_off[*lo] : 0;
        return in_layout(*hi - *lo, nk, me);
    };
    std::atomic<int> h2d_err{0};
    auto stage_and_send = [&](uint32_t j) {
        uint64_t lo, hi;
        const InLayout L = layout_of(j, &lo, &hi);
        // the pinned buffer's previous H2D (slice j - 2) must be done before it is rewritten
        if (j >= 2 && hipEventSynchronize(c->ev_h2d[j & 1]) != hipSuccess) h2d_err = 1;
        stage_slice(q, lo, hi, (char*)c->in_pin[j & 1], L, &bad);
        if (bad.load() != ~0ull) return;
        if (hipMemcpyAsync(c->in_dev[j & 1].p, c->in_pin[j & 1], L.bytes, hipMemcpyHostToDevice, c->hstream) != hipSuccess ||
            hipEventRecord(c->ev_h2d[j & 1], c->hstream) != hipSuccess)
            h2d_err = 1;
    };
    stage_and_send(0);
    std::thread stager;
    std::vector<std::thread> fillers;
    // the wire form (AD_INTO_WIRE=0: off): keyDeps keys as u8 indices into the request's query keys and
    // k2t as u16 cross PCIe; an expander thread per slice rebuilds the caller's arrays once its copy-out
    // has landed (beside the later slices' transfers)
    const char* we = getenv("AD_INTO_WIRE");
    const bool wire_on = !(we && atoi(we) == 0);
    std::thread expander[2];
    std::atomic<int> exp_err{0};
    struct JoinExp {
        std::thread* t;
        ~JoinExp()
        {
            for (int i = 0; i < 2; ++i)
                if (t[i].joinable()) t[i].join();
        }
    } join_exp_{expander};
    struct JoinAll {
        std::vector<std::thread>& v;
        ~JoinAll()
        {
            for (auto& t : v)
                if (t.joinable()) t.join();
        }
    } join_fill_{fillers};
    struct Join {
        std::thread& t;
        ~Join()
        {
            if (t.joinable()) t.join();
        }
    } join_{stager};
    for (uint32_t j = 0; j < slices; ++j)
    {
        const double t_s0 = trace ? now_ms() : 0.0;
        if (stager.joinable()) stager.join();
        if (bad.load() != ~0ull)
            return c->fail(AD_E_INVAL, "request %llu: key_off not monotone or keys not strictly ascending",
                           (unsigned long long)bad.load());
        if (h2d_err.load()) return c->fail(AD_E_DEVICE, "ad_deps_batch_into: query H2D");
        uint64_t lo, hi;
        const InLayout L = layout_of(j, &lo, &hi);
        const uint64_t nc = hi - lo, k0 = q->key_off[lo], k1 = q->key_off[hi];
        // this bank's last copy-out must be complete: the resolve below may grow (free and reallocate) it
        if (j >= 2) HIPCHK(c, hipEventSynchronize(c->ev_copied[j & 1]));
        char* R = c->in_dev[j & 1].as<char>();
        HIPCHK(c, hipStreamWaitEvent(st, c->ev_h2d[j & 1], 0));
        bytes_in += L.bytes;
        // the other device region was last read by slice j - 1's resolve, complete on its return
        if (j + 1 < slices) stager = std::thread([&stage_and_send, j] { stage_and_send(j + 1); });
        ad_query_soa d{};
        d.n_txns = nc;
        d.n_keys = k1 - k0;
        d.txn_msb = (const uint64_t*)(R + L.tm);
        d.txn_lsb = (const uint64_t*)(R + L.tl);
        d.txn_node = (const int32_t*)(R + L.tn);
        d.exec_msb = (const uint64_t*)(R + L.em);
        d.exec_lsb = (const uint64_t*)(R + L.el);
        d.exec_node = (const int32_t*)(R + L.en);
        d.min_epoch = me ? (const int64_t*)(R + L.me) : nullptr;
        d.key_off = (const uint64_t*)(R + L.ko);
        d.keys = (const int64_t*)(R + L.k);
        const double t_s1 = trace ? now_ms() : 0.0;
        ad_deps_result dev{};
        int rc = run_pipeline(c, &d, st, &dev, false, true);       // complete on return
        if (rc) return rc;
        const double t_s2 = trace ? now_ms() : 0.0;
        const ad_stats& S = dev.stats;
        uint64_t t[9];
        for (int m = 0; m < 3; ++m)
        {
            t[3 * m] = S.n_keys[m];
            t[3 * m + 1] = S.n_unique[m];
            t[3 * m + 2] = S.n_pairs[m] + S.n_keys[m];
        }
        for (int a = 0; a < 9; ++a) fits = fits && base[a] + t[a] <= cap[a];
        bool w_keys = false, w_k2t = false;
        if (fits && wire_on && t[0])
        {
            if (!ens<uint8_t>(c->w_idx, t[0]) || !ens<uint32_t>(c->w_flag, 1)) return c->fail(AD_E_NOMEM, "wire buffers");
            HIPCHK(c, run_key_index(nc, d.key_off, d.keys, c->off.as<uint64_t>(), dev.keys[0], c->w_idx.as<uint8_t>(),
                                    c->w_flag.as<uint32_t>(), st));
            uint32_t fl = 3;
            HIPCHK(c, d2h(&fl, c->w_flag.p, 4, st));
            HIPCHK(c, hipStreamSynchronize(st));
            w_keys = !(fl & 1u);
            w_k2t = !(fl & 2u) && t[2] > 0;
            // this bank's landing buffers: the expander of slice j - 2 reads them
            if (expander[j & 1].joinable()) expander[j & 1].join();
            const size_t want[2] = {(size_t)t[0], (size_t)2 * t[2]};
            const bool use[2] = {w_keys, w_k2t};
            for (int k = 0; k < 2; ++k)
                if (use[k] && c->w_pin_cap[j & 1][k] < want[k])
                {
                    if (c->w_pin[j & 1][k]) (void)hipHostFree(c->w_pin[j & 1][k]);
                    c->w_pin[j & 1][k] = nullptr;
                    c->w_pin_cap[j & 1][k] = 0;
                    const size_t sz = want[k] + want[k] / 4 + 4096;
                    if (hipHostMalloc(&c->w_pin[j & 1][k], sz, hipHostMallocDefault) != hipSuccess)
                        return c->fail(AD_E_NOMEM, "wire landing buffer");
                    c->w_pin_cap[j & 1][k] = sz;
                }
        }
        if (fits)
        {
            OutSegs g{};
            const uint64_t* off = c->off.as<uint64_t>();
            // any pageable offsets array: the bases are added on the device first (k_add_bases) and every
            // offsets segment is a plain copy; otherwise the copy kernel adds them
            bool off_mapped = true;
            for (int m = 0; m < 3; ++m)
                if (t[3 * m] || t[3 * m + 2])
                    for (int k = 0; k < 3; ++k) off_mapped = off_mapped && dmap[m][k] != nullptr;
            if (!off_mapped) HIPCHK(c, run_add_bases(c->off.as<uint64_t>(), nc + 1, base, st));
            HIPCHK(c, hipEventRecord(c->ev_ready, st));
            HIPCHK(c, hipStreamWaitEvent(c->cstream, c->ev_ready, 0));
            for (int m = 0; m < 3; ++m)
            {
                if (!t[3 * m] && !t[3 * m + 2])
                {
                    // offsets of a map empty in this slice: its bases, written by a host thread
                    const Fill F{m, lo, hi, {base[3 * m], base[3 * m + 1], base[3 * m + 2]}};
                    fillers.emplace_back([F, out] {
                        uint64_t* offs[3] = {out->keys_off[F.m], out->txn_off[F.m], out->k2t_off[F.m]};
                        for (int k = 0; k < 3; ++k) std::fill(offs[k] + F.lo, offs[k] + F.hi + 1, F.b[k]);
                    });
                    continue;
                }
                uint64_t* offs[3] = {out->keys_off[m], out->txn_off[m], out->k2t_off[m]};
                for (int k = 0; k < 3; ++k)
                {
                    const uint64_t* src = off + (uint64_t)(3 * m + k) * (nc + 1);
                    if (dmap[m][k])
                        g.s[g.n++] = OutSeg{src, (uint64_t*)dmap[m][k] + lo, 8 * (nc + 1), off_mapped ? base[3 * m + k] : 0,
                                            off_mapped ? 1u : 0u, 0u};
                    else
                        HIPCHK(c, d2h(offs[k] + lo, src, 8 * (nc + 1), c->cstream));
                    bytes_out += 8 * (nc + 1);
                }
                const void* srcs[3] = {dev.keys[m], dev.txns[m], dev.k2t[m]};
                const uint64_t el[3] = {8, 4, 4};
                void* hdst[3] = {(char*)out->keys[m] + 8 * base[3 * m], (char*)out->txns[m] + 4 * base[3 * m + 1],
                                 (char*)out->k2t[m] + 4 * base[3 * m + 2]};
                for (int k = 0; k < 3; ++k)
                {
                    const uint64_t bytes = el[k] * t[3 * m + k];
                    if (!bytes) continue;
                    if (m == 0 && k == 0 && w_keys)
                    {
                        g.s[g.n++] = OutSeg{c->w_idx.p, mapped_addr(c->w_pin[j & 1][0]), t[0], 0, 0u, 0u};
                        bytes_out += t[0];
                        continue;
                    }
                    if (m == 0 && k == 2 && w_k2t)
                    {
                        g.s[g.n++] = OutSeg{srcs[2], mapped_addr(c->w_pin[j & 1][1]), bytes, 0, 2u, 0u};
                        bytes_out += bytes / 2;
                        continue;
                    }
                    if (dmap[m][3 + k])
                        g.s[g.n++] = OutSeg{srcs[k], (char*)dmap[m][3 + k] + el[k] * base[3 * m + k], bytes, 0, 0u, 0u};
                    else
                        HIPCHK(c, d2h(hdst[k], srcs[k], bytes, c->cstream));
                    bytes_out += bytes;
                }
            }
            HIPCHK(c, run_copy_out(g, c->cstream));
            HIPCHK(c, hipEventRecord(c->ev_copied[j & 1], c->cstream));
            if (w_keys || w_k2t)
            {
                if (expander[j & 1].joinable()) expander[j & 1].join();
                const uint8_t* widx = (const uint8_t*)c->w_pin[j & 1][0];
                const uint16_t* wk2t = (const uint16_t*)c->w_pin[j & 1][1];
                const uint64_t kb = base[0], tb = base[2], nk2t = t[2];
                hipEvent_t ev = c->ev_copied[j & 1];
                const int dev_id = c->device;
                expander[j & 1] = std::thread([=, &exp_err] {
                    (void)hipSetDevice(dev_id);
                    if (hipEventSynchronize(ev) != hipSuccess)
                    {
                        exp_err = 1;
                        return;
                    }
                    constexpr uint64_t RCH = 1 << 13, ECH = 1 << 18;
                    const uint64_t nr = w_keys ? (nc + RCH - 1) / RCH : 0, ne = w_k2t ? (nk2t + ECH - 1) / ECH : 0;
                    host_parallel(nr + ne, [&](size_t x) {
                        if (x < nr)
                        {
                            const uint64_t a = lo + x * RCH, b = std::min(hi, a + RCH);
                            const uint64_t* ko = out->keys_off[0];
                            int64_t* ok = out->keys[0];
                            for (uint64_t i = a; i < b; ++i)
                            {
                                const int64_t* qk = q->keys + q->key_off[i];
                                for (uint64_t k = ko[i]; k < ko[i + 1]; ++k) ok[k] = qk[widx[k - kb]];
                            }
                        }
                        else
                        {
                            const uint64_t e0 = (x - nr) * ECH, e1 = std::min(nk2t, e0 + ECH);
                            int32_t* dst = out->k2t[0] + tb;
                            for (uint64_t e = e0; e < e1; ++e) dst[e] = wk2t[e];
                        }
                    });
                });
            }
            auto sw = [](DevBuf& a, DevBuf& b) { std::swap(a.p, b.p); std::swap(a.cap, b.cap); };
            sw(c->off, c->off_b);
            for (int m = 0; m < 3; ++m)
            {
                sw(c->o_keys[m], c->o_keys_b[m]);
                sw(c->o_txns[m], c->o_txns_b[m]);
                sw(c->o_k2t[m], c->o_k2t_b[m]);
            }
        }
        for (int a = 0; a < 9; ++a) base[a] += t[a];
        agg.n_txns += S.n_txns;
        agg.n_probes += S.n_probes;
        agg.n_deferred += S.n_deferred;
        agg.n_deferred_lean += S.n_deferred_lean;
        agg.n_lean_pass2 += S.n_lean_pass2;
        for (int m = 0; m < 3; ++m)
        {
            agg.n_pairs[m] += S.n_pairs[m];
            agg.n_unique[m] += S.n_unique[m];
            agg.n_keys[m] += S.n_keys[m];
        }
        for (int i = 0; i < 7; ++i) agg.ms_stage[i] += S.ms_stage[i];
        agg.ms_device += S.ms_device;
        if (trace)
            fprintf(stderr, "[into] slice %u: %llu txns, stage-wait+h2d %.3f ms, resolve %.3f ms, enqueue %.3f ms (at %.3f)\n",
                    j, (unsigned long long)nc, t_s1 - t_s0, t_s2 - t_s1, now_ms() - t_s2, t_s0 - t_begin);
    }
    const double t_f0 = trace ? now_ms() : 0.0;
    for (auto& t : fillers) t.join();
    for (auto& t : expander)
        if (t.joinable()) t.join();
    if (exp_err.load()) return c->fail(AD_E_DEVICE, "ad_deps_batch_into: copy-out");
    const double t_d0 = trace ? now_ms() : 0.0;
    HIPCHK(c, hipStreamSynchronize(c->cstream));
    if (trace)
        fprintf(stderr, "[into] fills %.3f ms, drain %.3f ms, total %.3f ms; %.1f MB in (H2D), %.1f MB out (D2H)\n",
                t_d0 - t_f0, now_ms() - t_d0, now_ms() - t_begin, bytes_in / 1e6, bytes_out / 1e6);
    for (int a = 0; a < 9; ++a) need[a] = base[a];
    agg.ms_ingest = c->ms_ingest;
    out->n_txns = n;
    out->stats = agg;
    if (n == 0)
        for (int m = 0; m < 3; ++m) out->keys_off[m][0] = out->txn_off[m][0] = out->k2t_off[m][0] = 0;
    if (!fits)
        return c->fail(AD_E_SPACE, "ad_deps_batch_into: output capacities too small (needed sizes in need[])");
    return AD_OK;
}

int ad_deps_batch_into(ad_ctx* c, const ad_query_soa* q, uint32_t flags, ad_deps_result* out, const uint64_t* cap,
                       uint64_t* need, uint32_t slices)
{
    if (!c || !q || !out || !cap || !need) return AD_E_INVAL;
    if (!c->cfk.loaded) return c->fail(AD_E_NOT_LOADED, "ad_cfk_load not called");
    if (hipSetDevice(c->device) != hipSuccess) return c->fail(AD_E_DEVICE, "hipSetDevice");
    StreamScope scope_(c->stream, c->cstream);
    const uint64_t n = q->n_txns;
    for (int m = 0; m < 3; ++m)
        if (!out->keys_off[m] || !out->txn_off[m] || !out->k2t_off[m] || (cap[3 * m] && !out->keys[m]) ||
            (cap[3 * m + 1] && !out->txns[m]) || (cap[3 * m + 2] && !out->k2t[m]))
            return c->fail(AD_E_INVAL, "ad_deps_batch_into: output arrays missing for map %d", m);
    // key-only SNAPSHOT batches take the pipelined path (its staging pass checks the keys)
    const bool fast = !(flags & AD_SEQUENTIAL) && !(n && q->range_off && q->range_off[n] > q->range_off[0]) &&
                      getenv("AD_INTO_LEGACY") == nullptr;
    int rc = fast ? 0 : check_query_host(c, q, flags);
    if (rc) return rc;
    if (flags & AD_SEQUENTIAL)
    {
        rc = sequential_on_device(c, q);
        if (rc < 0) return rc;
        if (rc > 0)
        {
            if ((rc = sync_host(c))) return rc;
            auto saved = c->cfk;
            auto saved_cmds = c->cmds;
            if ((rc = apply_preaccepts(c, q)))
            {
                c->cfk = saved;
                c->cmds = saved_cmds;
                return rc;
            }
        }
        slices = 1;        // the inserted requests are part of one snapshot
    }
    if (c->dirty && (rc = build_snapshot(c))) return rc;
    if (!c->cstream) HIPCHK(c, hipStreamCreateWithFlags(&c->cstream, hipStreamNonBlocking));
    scope_.add(c->cstream);
    // every return -- errors inside the slice loop included -- waits for the copy-outs already queued
    // into the caller's arrays: the caller may unregister and free them as soon as this returns
    struct CopyDrain {
        hipStream_t s;
        ~CopyDrain() { (void)hipStreamSynchronize(s); }
    } drain_{c->cstream};
    if (!c->ev_ready) HIPCHK(c, hipEventCreateWithFlags(&c->ev_ready, hipEventDisableTiming));
    for (hipEvent_t& e : c->ev_copied)
        if (!e) HIPCHK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
    if (fast) return deps_into_fast(c, q, out, cap, need, slices);
    // slices of >= 128k requests (SNAPSHOT requests are independent): slice j's result is copied out on
    // the copy stream while slice j + 1 resolves into the other result bank
    if (slices == 0) slices = (uint32_t)std::min<uint64_t>(4, std::max<uint64_t>(1, n >> 17));
    slices = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(slices, std::max<uint64_t>(n, 1)));
    auto swap_bank = [&]() {
        auto sw = [](DevBuf& a, DevBuf& b) { std::swap(a.p, b.p); std::swap(a.cap, b.cap); };
        sw(c->off, c->off_b);
        for (int m = 0; m < 3; ++m)
        {
            sw(c->o_keys[m], c->o_keys_b[m]);
            sw(c->o_txns[m], c->o_txns_b[m]);
            sw(c->o_k2t[m], c->o_k2t_b[m]);
        }
    };
    uint64_t base[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    bool fits = true;
    ad_stats agg{};
    std::vector<uint64_t> ko, ro;
    hipStream_t st = c->stream;
    // AD_INTO_TRACE=1: per-slice host timeline on stderr (staging, resolve, copy-out enqueue, final drain)
    const bool trace = getenv("AD_INTO_TRACE") != nullptr;
    auto tnow = []() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
    const double t_begin = trace ? tnow() : 0.0;
    uint64_t bytes_in = 0, bytes_out = 0;
    for (uint32_t j = 0; j < slices; ++j)
    {
        const double t_s0 = trace ? tnow() : 0.0;
        const uint64_t lo = n * j / slices, hi = n * (j + 1) / slices, nc = hi - lo;
        const uint64_t k0 = n ? q->key_off[lo] : 0, k1 = n ? q->key_off[hi] : 0;
        // this bank's last copy-out must be complete on the host side too: the resolve below may grow
        // (free and reallocate) the bank's buffers, which a stream-side wait would not protect
        if (j >= 2) HIPCHK(c, hipEventSynchronize(c->ev_copied[j & 1]));
        ko.resize(nc + 1);
        for (uint64_t i = 0; i <= nc; ++i) ko[i] = n ? q->key_off[lo + i] - k0 : 0;
        ad_query_soa d{};
        d.n_txns = nc;
        d.n_keys = k1 - k0;
        rc = 0;
        d.txn_msb = stage_q(c, c->q_tm, q->txn_msb + lo, nc, &rc);
        d.txn_lsb = stage_q(c, c->q_tl, q->txn_lsb + lo, nc, &rc);
        d.txn_node = stage_q(c, c->q_tn, q->txn_node + lo, nc, &rc);
        d.exec_msb = stage_q(c, c->q_em, q->exec_msb + lo, nc, &rc);
        d.exec_lsb = stage_q(c, c->q_el, q->exec_lsb + lo, nc, &rc);
        d.exec_node = stage_q(c, c->q_en, q->exec_node + lo, nc, &rc);
        d.min_epoch = q->min_epoch ? stage_q(c, c->q_me, q->min_epoch + lo, nc, &rc) : nullptr;
        d.key_off = stage_q(c, c->q_ko, ko.data(), nc + 1, &rc);
        d.keys = stage_q(c, c->q_k, q->keys + k0, k1 - k0, &rc);
        if (nc && q->range_off && q->range_off[hi] > q->range_off[lo])
        {
            const uint64_t r0 = q->range_off[lo], nr = q->range_off[hi] - r0;
            ro.resize(nc + 1);
            for (uint64_t i = 0; i <= nc; ++i) ro[i] = q->range_off[lo + i] - r0;
            d.range_off = stage_q(c, c->q_ro, ro.data(), nc + 1, &rc);
            d.range_start = stage_q(c, c->q_rs, q->range_start + r0, nr, &rc);
            d.range_end = stage_q(c, c->q_re, q->range_end + r0, nr, &rc);
            d.n_ranges = nr;
        }
        if (rc) return rc;
        const double t_s1 = trace ? tnow() : 0.0;
        if (trace)
            bytes_in += nc * (3 * 20 + 8) + 8 * (k1 - k0) + (q->min_epoch ? 8 * nc : 0);
        ad_deps_result dev{};
        if ((rc = run_pipeline(c, &d, st, &dev, false, true))) return rc;      // complete on return
        const double t_s2 = trace ? tnow() : 0.0;
        const ad_stats& S = dev.stats;
        uint64_t t[9];
        for (int m = 0; m < 3; ++m)
        {
            t[3 * m] = S.n_keys[m];
            t[3 * m + 1] = S.n_unique[m];
            t[3 * m + 2] = S.n_pairs[m] + S.n_keys[m];
        }
        for (int a = 0; a < 9; ++a) fits = fits && base[a] + t[a] <= cap[a];
        if (fits)
        {
            // offsets relative to the whole batch, then the copy-out of this slice
            HIPCHK(c, run_add_bases(c->off.as<uint64_t>(), nc + 1, base, st));
            HIPCHK(c, hipEventRecord(c->ev_ready, st));
            HIPCHK(c, hipStreamWaitEvent(c->cstream, c->ev_ready, 0));
            for (int m = 0; m < 3; ++m)
            {
                uint64_t* offs[3] = {out->keys_off[m], out->txn_off[m], out->k2t_off[m]};
                if (!t[3 * m] && !t[3 * m + 2])
                {
                    // a map empty in this slice: its offsets are the bases (host fill, no transfer)
                    for (int k = 0; k < 3; ++k) std::fill(offs[k] + lo, offs[k] + hi + 1, base[3 * m + k]);
                    continue;
                }
                for (int k = 0; k < 3; ++k)
                    HIPCHK(c, d2h(offs[k] + lo, c->off.as<uint64_t>() + (uint64_t)(3 * m + k) * (nc + 1),
                                             8 * (nc + 1), c->cstream));
                if (t[3 * m])
                    HIPCHK(c, d2h(out->keys[m] + base[3 * m], dev.keys[m], 8 * t[3 * m], c->cstream));
                if (t[3 * m + 1])
                    HIPCHK(c, d2h(out->txns[m] + base[3 * m + 1], dev.txns[m], 4 * t[3 * m + 1],
                                             c->cstream));
                if (t[3 * m + 2])
                    HIPCHK(c, d2h(out->k2t[m] + base[3 * m + 2], dev.k2t[m], 4 * t[3 * m + 2],
                                             c->cstream));
            }
            HIPCHK(c, hipEventRecord(c->ev_copied[j & 1], c->cstream));
            swap_bank();
            if (trace)
                for (int m = 0; m < 3; ++m)
                    bytes_out += (t[3 * m] || t[3 * m + 2] ? 24 * (nc + 1) : 0) + 8 * t[3 * m] + 4 * t[3 * m + 1] + 4 * t[3 * m + 2];
        }
        if (trace)
            fprintf(stderr, "[into] slice %u: %llu txns, stage %.3f ms, resolve %.3f ms, enqueue %.3f ms (at %.3f)\n", j,
                    (unsigned long long)nc, t_s1 - t_s0, t_s2 - t_s1, tnow() - t_s2, t_s0 - t_begin);
        for (int a = 0; a < 9; ++a) base[a] += t[a];
        agg.n_txns += S.n_txns;
        agg.n_probes += S.n_probes;
        agg.n_deferred += S.n_deferred;
        agg.n_deferred_lean += S.n_deferred_lean;
        agg.n_lean_pass2 += S.n_lean_pass2;
        for (int m = 0; m < 3; ++m)
        {
            agg.n_pairs[m] += S.n_pairs[m];
            agg.n_unique[m] += S.n_unique[m];
            agg.n_keys[m] += S.n_keys[m];
        }
        for (int i = 0; i < 7; ++i) agg.ms_stage[i] += S.ms_stage[i];
        agg.ms_device += S.ms_device;
    }
    const double t_d0 = trace ? tnow() : 0.0;
    HIPCHK(c, hipStreamSynchronize(c->cstream));
    if (trace)
        fprintf(stderr, "[into] drain %.3f ms, total %.3f ms; %.1f MB in (H2D), %.1f MB out (D2H)\n", tnow() - t_d0,
                tnow() - t_begin, bytes_in / 1e6, bytes_out / 1e6);
    for (int a = 0; a < 9; ++a) need[a] = base[a];
    agg.ms_ingest = c->ms_ingest;
    out->n_txns = n;
    out->stats = agg;
    if (n == 0)
        for (int m = 0; m < 3; ++m) out->keys_off[m][0] = out->txn_off[m][0] = out->k2t_off[m][0] = 0;
    if (!fits)
        return c->fail(AD_E_SPACE, "ad_deps_batch_into: output capacities too small (needed sizes in need[])");
    return AD_OK;
}

int ad_deps_batch_device(ad_ctx* c, const ad_query_soa* q, uint32_t flags, void* stream, ad_deps_result* out)
{
    if (!c || !q || !out) return AD_E_INVAL;
    if (!c->cfk.loaded) return c->fail(AD_E_NOT_LOADED, "ad_cfk_load not called");
    if (flags & AD_SEQUENTIAL) return c->fail(AD_E_INVAL, "device-resident batches are SNAPSHOT only");
    if (hipSetDevice(c->device) != hipSuccess) return c->fail(AD_E_DEVICE, "hipSetDevice");
    StreamScope scope_(c->stream, c->cstream);
    int rc;
    if (c->dirty && (rc = build_snapshot(c))) return rc;
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    scope_.add(st);
    // AD_REGIONS and AD_PARTS_ONLY: no packed copy (the regions are the result)
    return run_pipeline(c, q, st, out, (flags & (AD_PARTS_ONLY | AD_REGIONS)) != 0, (flags & AD_N_KEYS) != 0);
}

// device view of the snapshot for mapReduceFull: entries in load order with executeAt ranks,
// status, kind and their TxnInfo.missing() lists as ranks (built once per snapshot / missing load)
// The live range commands of the view: per range entry of the snapshot its command, the commands'
// recovery facts normalised. Host-built from the loaded commands; rebuilt when ranks change.
static int build_rv_ranges(ad_ctx* c, bool live_cmds)
{
    if (int rc = host_dict(c)) return rc;
    int rc;
        const auto& R = c->cmds;
        const size_t nc = R.txn.size(), nre = c->h_rtxw.size();
        std::vector<uint32_t> r_cmd(std::max<size_t>(nre, 1), ~0u), flags(std::max<size_t>(nc, 1), 0), dep_off(nc + 1, 0);
        std::vector<uint64_t> ex_hi(std::max<size_t>(nc, 1)), ex_lo(std::max<size_t>(nc, 1)), dhi, dlo;
        std::vector<int32_t> ex_node(std::max<size_t>(nc, 1)), dnode;
        std::vector<std::pair<uint32_t, uint32_t>> by_rank;       // (rank, command) of the live commands
        for (size_t i = 0; i < nc; ++i)
        {
            const bool live = (R.historical.empty() || !R.historical[i]) && (R.erased.empty() || !R.erased[i]);
            if (live) by_rank.push_back({c->h_cmd_rank[i], (uint32_t)i});
            if (R.rec)
            {
                flags[i] = (R.rec_status[i] & 3u) | (R.rec_has_deps[i] ? 4u : 0u);
                const NormTid x = norm(R.rec_exec[i]);
                ex_hi[i] = x.hi; ex_lo[i] = x.lo; ex_node[i] = x.node;
                for (uint64_t j = R.rec_dep_off[i]; j < R.rec_dep_off[i + 1]; ++j)
                {
                    const NormTid d = norm(R.rec_deps[j]);
                    dhi.push_back(d.hi); dlo.push_back(d.lo); dnode.push_back(d.node);
                }
            }
            dep_off[i + 1] = (uint32_t)dhi.size();
        }
        std::sort(by_rank.begin(), by_rank.end());
        for (size_t e = 0; e < nre; ++e)
        {
            if (!c->h_rlive[e]) continue;
            const uint32_t rk = c->h_rtxw[e] & RANK_MASK;
            auto it = std::lower_bound(by_rank.begin(), by_rank.end(), std::make_pair(rk, 0u));
            if (it != by_rank.end() && it->first == rk) r_cmd[e] = it->second;
        }
        if (dhi.empty()) { dhi.push_back(0); dlo.push_back(0); dnode.push_back(0); }
        if ((rc = upload(c, c->rv_rcmd, r_cmd)) || (rc = upload(c, c->rv_rflags, flags)) ||
            (rc = upload(c, c->rv_rex_hi, ex_hi)) || (rc = upload(c, c->rv_rex_lo, ex_lo)) ||
            (rc = upload(c, c->rv_rex_node, ex_node)) || (rc = upload(c, c->rv_rdep_off, dep_off)) ||
            (rc = upload(c, c->rv_rdep_hi, dhi)) || (rc = upload(c, c->rv_rdep_lo, dlo)) ||
            (rc = upload(c, c->rv_rdep_node, dnode)))
            return rc;
        c->rv_ranges = live_cmds && nre > 0;
    c->rv_rng_gen = c->rank_gen;
    return 0;
}

// The view from the device state (a live store: ad_cfk_update / ad_cfk_prune keep it current, nothing
// goes through the host): entries, segments, prunedBefore, trees and the inverted missing() index.
static int build_recovery_view_device(ad_ctx* c)
{
    const uint64_t ne = c->ds.n_ent, nk = c->ds.n_keys;
    hipStream_t st = c->stream;
    RvDevIn in{ne, nk, c->ds.ent, c->ds.krec, c->d_status.as<uint8_t>(), c->d_xrank.as<uint32_t>(), c->d_ekey.as<uint32_t>(),
               c->dmiss_on ? c->d_mref.as<uint32_t>() : nullptr, c->d_moff.as<uint64_t>(), c->d_mids.as<uint32_t>()};
    int nl = 1;
    std::vector<uint64_t> lvl_n(1, ne);
    while (lvl_n.back() > 1 && nl < MAX_LEVELS)
    {
        lvl_n.push_back((lvl_n.back() + 63) / 64);
        ++nl;
    }
    if (nl < 2)
    {
        lvl_n.push_back(1);
        nl = 2;
    }
    std::vector<uint64_t> lvl_at(nl + 1, 0);
    for (int l = 1; l < nl; ++l) lvl_at[l + 1] = lvl_at[l] + lvl_n[l];
    const uint64_t per_set = lvl_at[nl];
    if (!ens<uint4>(c->rv_ent, ne) || !ens<uint32_t>(c->rv_seg, nk + 1) || !ens<uint32_t>(c->rv_pruned, nk) ||
        !ens<uint32_t>(c->rv_cnt, ne) || !ens<uint64_t>(c->rv_eoff, ne + 1) || !ens<uint64_t>(c->rv_bsum, (ne + 1023) / 1024 + 16) ||
        !ens<uint32_t>(c->rv_err, 1) || !ens<uint32_t>(c->rv_tree, 2 * per_set) || !ens<uint64_t>(c->rv_inv_off, nk + 1))
        return c->fail(AD_E_NOMEM, "recovery view");
    uint32_t* tree = c->rv_tree.as<uint32_t>();
    std::vector<uint32_t*> l0(nl, nullptr), l1(nl, nullptr);
    for (int l = 1; l < nl; ++l)
    {
        l0[l] = tree + lvl_at[l];
        l1[l] = tree + per_set + lvl_at[l];
    }
    HIPCHK(c, hipMemsetAsync(c->rv_err.p, 0, 4, st));
    HIPCHK(c, run_rv_entries(in, c->rv_ent.as<uint4>(), c->rv_seg.as<uint32_t>(), c->rv_pruned.as<uint32_t>(),
                             c->rv_cnt.as<uint32_t>(), c->rv_err.as<uint32_t>(), st));
    HIPCHK(c, run_rv_trees(in, l0.data(), l1.data(), lvl_n.data(), nl, st));
    HIPCHK(c, run_scan_arrays(c->rv_cnt.as<uint32_t>(), c->rv_eoff.as<uint64_t>(), ne, 1, c->rv_bsum.as<uint64_t>(), st));
    uint64_t np = 0;
    uint32_t err = 0;
    HIPCHK(c, d2h(&np, c->rv_eoff.as<uint64_t>() + ne, 8, st));
    HIPCHK(c, d2h(&err, c->rv_err.p, 4, st));
    HIPCHK(c, hipStreamSynchronize(st));
    if (err) return c->fail(AD_E_CAPACITY, "more than %u missing ids on one entry", RV_MAX_MISS);
    // per key, its (missing() id, entry) pairs sorted by id (entries ascending within): a stable radix
    // sort of (key index << 32 | id rank) over the pairs written in entry order
    if (!ens<uint64_t>(c->rv_pk, np) || !ens<uint32_t>(c->rv_pv, np) || !ens<uint64_t>(c->rv_pk2, np) ||
        !ens<uint32_t>(c->rv_pv2, np) || !ens<uint2>(c->rv_inv, np))
        return c->fail(AD_E_NOMEM, "recovery view");
    uint64_t* ks = c->rv_pk.as<uint64_t>();
    uint32_t* vs = c->rv_pv.as<uint32_t>();
    HIPCHK(c, run_rv_inv_pairs(in, c->rv_eoff.as<uint64_t>(), ks, vs, st));
    if (np > 1)
    {
        auto nbytes = [](uint64_t v) { uint32_t b = 0; while (v) { ++b; v >>= 8; } return b; };
        uint32_t mask = 0;
        for (uint32_t b = 0; b < nbytes(2 * c->ds.n_dict + 1) && b < 4; ++b) mask |= 1u << b;
        for (uint32_t b = 0; b < nbytes(nk ? nk - 1 : 0) && b < 4; ++b) mask |= 1u << (4 + b);
        const uint64_t hn = radix_hist_entries(np);
        if (!ens<uint32_t>(c->rv_hist, hn) || !ens<uint64_t>(c->rv_hoff, hn + 1) ||
            !ens<uint64_t>(c->rv_bsum, (std::max(hn, np) + 1023) / 1024 + 16))
            return c->fail(AD_E_NOMEM, "recovery view");
        HIPCHK(c, radix_sort_pairs(ks, vs, c->rv_pk2.as<uint64_t>(), c->rv_pv2.as<uint32_t>(), np, mask, c->rv_hist.as<uint32_t>(),
                                   c->rv_hoff.as<uint64_t>(), c->rv_bsum.as<uint64_t>(), st, &ks, &vs));
    }
    HIPCHK(c, run_rv_inv_finish(in, c->rv_eoff.as<uint64_t>(), ks, vs, np, c->rv_inv_off.as<uint64_t>(), c->rv_inv.as<uint2>(), st));
    HIPCHK(c, hipStreamSynchronize(st));
    c->rv_levels = nl;
    c->rv_lvl_at.assign(lvl_at.begin(), lvl_at.end());
    c->rv_per_set = per_set;
    c->rv_dev_miss = c->dmiss_on;
    return 0;
}

static int build_recovery_view(ad_ctx* c, RecoveryView* v)
{
    auto& K = c->cfk;
    // a live store (lists on the device, or none at all): the view from the device state
    const bool dev = !c->dirty && !getenv("AD_RV_HOST") && (c->dmiss_on || (K.miss_off.empty() && !K.miss_stale));
    if (!dev)
        if (int rc0 = sync_host(c)) return rc0;
    bool live_cmds = false;
    for (size_t i = 0; i < c->cmds.txn.size(); ++i)
        live_cmds |= (c->cmds.historical.empty() || !c->cmds.historical[i]) && (c->cmds.erased.empty() || !c->cmds.erased[i]);
    if (live_cmds && !c->cmds.rec)
        return c->fail(AD_E_STATE, "recovery scans of range commands need their recovery facts (ad_range_cmds_recovery_load)");
    if (!dev && K.miss_stale) return c->fail(AD_E_STATE, "missing lists predate SEQUENTIAL insertions: load them again");
    const uint64_t ne = K.status.size(), nk = K.keys.size();
    if (dev && c->rv_gen != c->snap_gen)
    {
        if (int rc = build_recovery_view_device(c)) return rc;
        c->rv_gen = c->snap_gen;
    }
    if (dev && c->rv_rng_gen != c->rank_gen)
    {
        if (int rc = build_rv_ranges(c, live_cmds)) return rc;
        HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    if (!dev && c->rv_gen != c->snap_gen)
    {
        std::vector<uint4> ent(ne);
        std::vector<uint32_t> seg(nk + 1), miss;
        for (uint64_t k = 0; k <= nk; ++k) seg[k] = (uint32_t)K.seg[k];
        // rank of an id: member i of the dictionary -> 2i+1, else 2 * lower bound (as encode_rank)
        auto rank_of = [&](const Tid& t) -> uint32_t {
            const NormTid x = norm(t);
            uint64_t lo = 0, hi = c->dict_msb.size();
            while (lo < hi)
            {
                const uint64_t mid = (lo + hi) >> 1;
                if (norm_cmp(norm_tid(c->dict_msb[mid], c->dict_lsb[mid], c->dict_node[mid]), x) < 0) lo = mid + 1;
                else hi = mid;
            }
            if (lo < c->dict_msb.size() && norm_cmp(norm_tid(c->dict_msb[lo], c->dict_lsb[lo], c->dict_node[lo]), x) == 0)
                return (uint32_t)(2 * lo + 1);
            return (uint32_t)(2 * lo);
        };
        for (uint64_t e = 0; e < ne; ++e)
        {
            const uint32_t kind = (uint32_t)((K.txn[e].lsb >> 1) & 7);
            uint32_t nm = 0, mo = (uint32_t)miss.size();
            if (!K.miss_off.empty())
            {
                const uint64_t a = K.miss_off[e], b = K.miss_off[e + 1];
                if (b - a > RV_MAX_MISS) return c->fail(AD_E_CAPACITY, "more than %u missing ids on one entry", RV_MAX_MISS);
                for (uint64_t j = a; j < b; ++j) miss.push_back(rank_of(K.miss[j]));
                nm = (uint32_t)(b - a);
            }
            ent[e] = make_uint4(c->h_txn_rank[e], c->h_exec_rank[e], K.status[e] | (kind << 8) | (nm << RV_MISS_SHIFT), mo);
        }
        // per status set (ACCEPTED/COMMITTED, STABLE/APPLIED) a 64-ary max tree of the entries' executeAt
        // ranks: every scan wants executeAt > testTxnId (:861-866), so a subtree at or below it is skipped
        int nl = 1;
        std::vector<uint64_t> lvl_n(1, ne);
        while (lvl_n.back() > 1 && nl < MAX_LEVELS)
        {
            lvl_n.push_back((lvl_n.back() + 63) / 64);
            ++nl;
        }
        if (nl < 2)
        {
            lvl_n.push_back(1);
            nl = 2;
        }
        std::vector<uint64_t> lvl_at(nl + 1, 0);      // offset of level l (>= 1) in the per-set array
        for (int l = 1; l < nl; ++l) lvl_at[l + 1] = lvl_at[l] + lvl_n[l];
        const uint64_t per_set = lvl_at[nl];
        std::vector<uint32_t> tree(2 * per_set, 0);
        for (uint64_t e = 0; e < ne; ++e)
        {
            const uint32_t st = K.status[e];
            const int set = (st == 3 || st == 4) ? 0 : (st == 5 || st == 6) ? 1 : -1;
            if (set >= 0)
            {
                uint32_t& x = tree[set * per_set + lvl_at[1] + e / 64];
                x = std::max(x, c->h_exec_rank[e]);
            }
        }
        for (int set = 0; set < 2; ++set)
            for (int l = 2; l < nl; ++l)
                for (uint64_t j = 0; j < lvl_n[l - 1]; ++j)
                {
                    uint32_t& x = tree[set * per_set + lvl_at[l] + j / 64];
                    x = std::max(x, tree[set * per_set + lvl_at[l - 1] + j]);
                }
        // per key, the (missing() id, entry) pairs sorted: a WITHOUT scan of a known testTxnId wants
        // exactly the entries whose missing() holds it (:868-872)
        std::vector<uint64_t> inv_off(nk + 1, 0);
        for (uint64_t k = 0; k < nk; ++k)
        {
            uint64_t cnt = 0;
            for (uint64_t e = K.seg[k]; e < K.seg[k + 1]; ++e) cnt += ent[e].z >> RV_MISS_SHIFT;
            inv_off[k + 1] = inv_off[k] + cnt;
        }
        std::vector<uint2> inv(inv_off[nk]);
        parallel_for(nk, [&](size_t ka, size_t kb) {
            for (size_t k = ka; k < kb; ++k)
            {
                uint64_t at = inv_off[k];
                for (uint64_t e = K.seg[k]; e < K.seg[k + 1]; ++e)
                {
                    const uint32_t nm = ent[e].z >> RV_MISS_SHIFT;
                    for (uint32_t j = 0; j < nm; ++j) inv[at++] = make_uint2(miss[ent[e].w + j], (uint32_t)e);
                }
                std::sort(inv.begin() + inv_off[k], inv.begin() + at,
                          [](const uint2& x, const uint2& y) { return x.x < y.x || (x.x == y.x && x.y < y.y); });
            }
        });
        int rc;
        if ((rc = upload(c, c->rv_ent, ent)) || (rc = upload(c, c->rv_seg, seg)) || (rc = upload(c, c->rv_pruned, c->h_pruned)) ||
            (rc = upload(c, c->rv_miss, miss)) || (rc = upload(c, c->rv_tree, tree)) || (rc = upload(c, c->rv_inv_off, inv_off)) ||
            (rc = upload(c, c->rv_inv, inv)))
            return rc;
        c->rv_levels = nl;
        c->rv_lvl_at.assign(lvl_at.begin(), lvl_at.end());
        c->rv_per_set = per_set;
        if ((rc = build_rv_ranges(c, live_cmds))) return rc;
        HIPCHK(c, hipStreamSynchronize(c->stream));
        c->rv_gen = c->snap_gen;
        c->rv_dev_miss = false;
    }
    v->ent = c->rv_ent.as<uint4>();
    v->seg = c->rv_seg.as<uint32_t>();
    v->pruned = c->rv_pruned.as<uint32_t>();
    v->miss = c->rv_dev_miss ? c->d_mids.as<uint32_t>() : c->rv_miss.as<uint32_t>();
    for (int set = 0; set < 2; ++set)
        for (int l = 0; l < MAX_LEVELS; ++l)
            v->lvl[set][l] = (l >= 1 && l < c->rv_levels) ? c->rv_tree.as<uint32_t>() + set * c->rv_per_set + c->rv_lvl_at[l]
                                                          : nullptr;
    v->n_levels = c->rv_levels;
    v->inv_off = c->rv_inv_off.as<uint64_t>();
    v->inv = c->rv_inv.as<uint2>();
    v->r_cmd = c->rv_rcmd.as<uint32_t>();
    v->rc_flags = c->rv_rflags.as<uint32_t>();
    v->rc_ex_hi = c->rv_rex_hi.as<uint64_t>();
    v->rc_ex_lo = c->rv_rex_lo.as<uint64_t>();
    v->rc_ex_node = c->rv_rex_node.as<int32_t>();
    v->rc_dep_off = c->rv_rdep_off.as<uint32_t>();
    v->rc_dep_hi = c->rv_rdep_hi.as<uint64_t>();
    v->rc_dep_lo = c->rv_rdep_lo.as<uint64_t>();
    v->rc_dep_node = c->rv_rdep_node.as<int32_t>();
    v->ranges = c->rv_ranges;
    return 0;
}

int ad_cfk_missing_load(ad_ctx* c, const ad_cfk_missing_soa* m)
{
    if (c && c->host_stale)
        if (int rc0 = sync_host(c)) return rc0;
    if (!c || !m) return AD_E_INVAL;
    auto& K = c->cfk;
    if (!K.loaded) return c->fail(AD_E_NOT_LOADED, "ad_cfk_load not called");
    const uint64_t ne = K.status.size();
    if (m->n_entries != ne) return c->fail(AD_E_INVAL, "missing lists for %llu entries, snapshot has %llu",
                                           (unsigned long long)m->n_entries, (unsigned long long)ne);
    for (uint64_t e = 0; e < ne; ++e)
    {
        const uint64_t a = m->off[e], b = m->off[e + 1];
        if (b < a) return c->fail(AD_E_INVAL, "missing offsets not monotone");
        if (b > a && !(K.status[e] >= AD_ST_ACCEPTED && K.status[e] <= AD_ST_APPLIED))
            return c->fail(AD_E_INVAL, "missing ids on an entry without deps (CommandsForKey.java:278)");
        for (uint64_t j = a + 1; j < b; ++j)
        {
            const NormTid x = norm_tid(m->msb[j - 1], m->lsb[j - 1], m->node[j - 1]), y = norm_tid(m->msb[j], m->lsb[j], m->node[j]);
            if (norm_cmp(x, y) >= 0) return c->fail(AD_E_INVAL, "missing ids not strictly ascending");
        }
    }
    K.miss_off.assign(m->off, m->off + ne + 1);
    const uint64_t nm = m->off[ne];
    K.miss.resize(nm);
    for (uint64_t j = 0; j < nm; ++j) K.miss[j] = {m->msb[j], m->lsb[j], m->node[j]};
    K.miss_stale = false;
    c->rv_gen = ~0ull;
    c->rv_rng_gen = ~0ull;
    return AD_OK;
}

int ad_range_cmds_recovery_load(ad_ctx* c, const ad_range_cmds_recovery_soa* in)
{
    if (!c || !in) return AD_E_INVAL;
    auto& R = c->cmds;
    const uint64_t n = in->n_cmds;
    if (n != R.txn.size())
        return c->fail(AD_E_INVAL, "recovery facts for %llu range commands, %llu loaded", (unsigned long long)n,
                       (unsigned long long)R.txn.size());
    if (n && (!in->status || !in->has_deps || !in->exec_msb || !in->exec_lsb || !in->exec_node || !in->dep_off))
        return AD_E_INVAL;
    for (uint64_t i = 0; i < n; ++i)
    {
        if (in->status[i] > 3) return c->fail(AD_E_INVAL, "range command %llu: status class %u", (unsigned long long)i, in->status[i]);
        if (in->dep_off[i + 1] < in->dep_off[i]) return c->fail(AD_E_INVAL, "range command deps offsets not monotone");
        for (uint64_t j = in->dep_off[i] + 1; j < in->dep_off[i + 1]; ++j)
            if (norm_cmp(norm_tid(in->dep_msb[j - 1], in->dep_lsb[j - 1], in->dep_node[j - 1]),
                         norm_tid(in->dep_msb[j], in->dep_lsb[j], in->dep_node[j])) >= 0)
                return c->fail(AD_E_INVAL, "range command deps not strictly ascending");
    }
    R.rec_status.assign(in->status, in->status + n);
    R.rec_has_deps.assign(in->has_deps, in->has_deps + n);
    R.rec_exec.resize(n);
    for (uint64_t i = 0; i < n; ++i) R.rec_exec[i] = {in->exec_msb[i], in->exec_lsb[i], in->exec_node[i]};
    R.rec_dep_off.assign(in->dep_off, in->dep_off + n + 1);
    const uint64_t nd = n ? in->dep_off[n] : 0;
    R.rec_deps.resize(nd);
    for (uint64_t j = 0; j < nd; ++j) R.rec_deps[j] = {in->dep_msb[j], in->dep_lsb[j], in->dep_node[j]};
    R.rec = true;
    c->rv_gen = ~0ull;
    c->rv_rng_gen = ~0ull;
    return AD_OK;
}

int ad_recovery_batch_device(ad_ctx* c, const ad_query_soa* q, uint32_t scan, void* stream, ad_deps_result* out)
{
    if (!c || !q || !out) return AD_E_INVAL;
    if (!c->cfk.loaded) return c->fail(AD_E_NOT_LOADED, "ad_cfk_load not called");
    if (scan > AD_RECOVER_EXECUTES_AFTER_STABLE_NO_WITNESS) return c->fail(AD_E_INVAL, "unknown recovery scan %u", scan);
    if (hipSetDevice(c->device) != hipSuccess) return c->fail(AD_E_DEVICE, "hipSetDevice");
    StreamScope scope_(c->stream, c->cstream);
    int rc;
    if (c->dirty && (rc = build_snapshot(c))) return rc;
    RecoveryView v{};
    if ((rc = build_recovery_view(c, &v))) return rc;
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    scope_.add(st);
    return run_pipeline(c, q, st, out, false, false, (int)scan, &v);
}

int ad_recovery_batch(ad_ctx* c, const ad_query_soa* q, uint32_t scan, ad_deps_result** out)
{
    if (!c || !q || !out) return AD_E_INVAL;
    if (!c->cfk.loaded) return c->fail(AD_E_NOT_LOADED, "ad_cfk_load not called");
    if (hipSetDevice(c->device) != hipSuccess) return c->fail(AD_E_DEVICE, "hipSetDevice");
    StreamScope scope_(c->stream, c->cstream);
    int rc = check_query_host(c, q);
    if (rc) return rc;
    const uint64_t n = q->n_txns;
    const uint64_t np = n ? q->key_off[n] : 0;
    ad_query_soa d{};
    d.n_txns = n;
    d.txn_msb = stage_q(c, c->q_tm, q->txn_msb, n, &rc);
    d.txn_lsb = stage_q(c, c->q_tl, q->txn_lsb, n, &rc);
    d.txn_node = stage_q(c, c->q_tn, q->txn_node, n, &rc);
    d.key_off = stage_q(c, c->q_ko, q->key_off, n + 1, &rc);
    d.keys = stage_q(c, c->q_k, q->keys, np, &rc);
    std::vector<uint64_t> ro;
    if (n && q->range_off && q->range_off[n] > q->range_off[0])
    {
        // Range-domain requests: a recovering sync point or range txn over its Ranges (BeginRecovery
        // passes partialTxn.keys(), Seekables, to mapReduceFull: BeginRecovery.java:334,348,365,378)
        const uint64_t r0 = q->range_off[0], nr = q->range_off[n] - r0;
        ro.resize(n + 1);
        for (uint64_t i = 0; i <= n; ++i) ro[i] = q->range_off[i] - r0;
        d.range_off = stage_q(c, c->q_ro, ro.data(), n + 1, &rc);
        d.range_start = stage_q(c, c->q_rs, q->range_start + r0, nr, &rc);
        d.range_end = stage_q(c, c->q_re, q->range_end + r0, nr, &rc);
        d.n_ranges = nr;
        if (!rc) HIPCHK(c, hipStreamSynchronize(c->stream));     // ro is a local
    }
    if (rc) return rc;
    ad_deps_result dev{};
    if ((rc = ad_recovery_batch_device(c, &d, scan, c->stream, &dev))) return rc;
    return result_to_host(c, n, dev, out);
}

void ad_result_free(ad_deps_result* r)
{
    if (!r) return;
    for (int m = 0; m < 3; ++m)
    {
        free(r->keys_off[m]); free(r->keys[m]); free(r->txn_off[m]); free(r->txns[m]); free(r->k2t_off[m]); free(r->k2t[m]);
    }
    free(r);
}

int ad_dict(const ad_ctx* c, uint64_t* n, const uint64_t** msb, const uint64_t** lsb, const int32_t** node)
{
    if (c && host_dict(const_cast<ad_ctx*>(c))) return AD_E_DEVICE;
    if (!c || !n) return AD_E_INVAL;
    *n = c->dict_msb.size();
    if (msb) *msb = c->dict_msb.data();
    if (lsb) *lsb = c->dict_lsb.data();
    if (node) *node = c->dict_node.data();
    return AD_OK;
}

int ad_range_table(const ad_ctx* c, uint64_t* n, const int64_t** start, const int64_t** end)
{
    if (!c || !n) return AD_E_INVAL;
    *n = c->rt_start.size();
    if (start) *start = c->rt_start.data();
    if (end) *end = c->rt_end.data();
    return AD_OK;
}

static int load_range_map(ad_ctx* c, const ad_range_map_soa* m, ad_ctx::RangeMapBufs& B, const char* what)
{
    B.n = 0;
    B.has_present = false;
    if (!m || m->n_values == 0) return AD_OK;
    const uint64_t n = m->n_values;
    if (!m->starts || !m->msb || !m->lsb || !m->node) return c->fail(AD_E_INVAL, "%s: NULL array", what);
    for (uint64_t i = 0; i < n; ++i)
        if (m->starts[i] >= m->starts[i + 1]) return c->fail(AD_E_INVAL, "%s: starts not strictly ascending at %llu", what, (unsigned long long)i);
    if (!B.starts.ensure(8 * (n + 1)) || !B.msb.ensure(8 * n) || !B.lsb.ensure(8 * n) || !B.node.ensure(4 * n) ||
        (m->present && !B.present.ensure(n)))
        return c->fail(AD_E_NOMEM, "%s", what);
    HIPCHK(c, copy_sync(B.starts.p, m->starts, 8 * (n + 1), hipMemcpyHostToDevice));
    HIPCHK(c, copy_sync(B.msb.p, m->msb, 8 * n, hipMemcpyHostToDevice));
    HIPCHK(c, copy_sync(B.lsb.p, m->lsb, 8 * n, hipMemcpyHostToDevice));
    HIPCHK(c, copy_sync(B.node.p, m->node, 4 * n, hipMemcpyHostToDevice));
    if (m->present) HIPCHK(c, copy_sync(B.present.p, m->present, n, hipMemcpyHostToDevice));
    B.n = n;
    B.inclusive_ends = m->inclusive_ends ? 1u : 0u;
    B.has_present = m->present != nullptr;
    return AD_OK;
}

static DevRangeMap dev_range_map(ad_ctx::RangeMapBufs& B)
{
    DevRangeMap d{};
    d.n = B.n;
    if (B.n)
    {
        d.starts = B.starts.as<int64_t>();
        d.msb = B.msb.as<uint64_t>();
        d.lsb = B.lsb.as<uint64_t>();
        d.node = B.node.as<int32_t>();
        d.present = B.has_present ? B.present.as<uint8_t>() : nullptr;
    }
    d.inclusive_ends = B.inclusive_ends;
    return d;
}

int ad_preaccept_maps_load(ad_ctx* c, const ad_range_map_soa* max_conflicts, const ad_range_map_soa* reject_before)
{
    if (!c) return AD_E_INVAL;
    if (hipSetDevice(c->device) != hipSuccess) return c->fail(AD_E_DEVICE, "hipSetDevice");
    StreamScope scope_(c->stream, c->cstream);
    ++c->pa_gen;
    int rc = load_range_map(c, max_conflicts, c->pa_mc, "ad_preaccept_maps_load: maxConflicts");
    return rc ? rc : load_range_map(c, reject_before, c->pa_rb, "ad_preaccept_maps_load: rejectBefore");
}

int ad_preaccept_device(ad_ctx* c, const ad_query_soa* q, uint32_t permit_fast_path, uint64_t node_epoch, void* stream,
                        uint64_t* out_msb, uint64_t* out_lsb, int32_t* out_node, uint8_t* out_flags, ad_stats* stats)
{
    if (!c || !q) return AD_E_INVAL;
    if (q->n_txns && (!q->txn_msb || !q->txn_lsb || !q->txn_node || !q->key_off || !out_msb || !out_lsb || !out_node ||
                      !out_flags))
        return c->fail(AD_E_INVAL, "ad_preaccept_device: NULL array");
    if (hipSetDevice(c->device) != hipSuccess) return c->fail(AD_E_DEVICE, "hipSetDevice");
    StreamScope scope_(c->stream, c->cstream);
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    scope_.add(st);
    PreacceptArgs a{};
    a.n = q->n_txns;
    a.txn_msb = q->txn_msb; a.txn_lsb = q->txn_lsb; a.txn_node = q->txn_node;
    a.key_off = q->key_off; a.keys = q->keys;
    a.mc = dev_range_map(c->pa_mc);
    a.rb = dev_range_map(c->pa_rb);
    a.permit_fast_path = permit_fast_path ? 1u : 0u;
    a.node_epoch = node_epoch;
    a.out_msb = out_msb; a.out_lsb = out_lsb; a.out_node = out_node; a.out_flags = out_flags;
    if (c->cfk.loaded && !c->dirty && c->ds.n_keys && c->ds.khash)
    {
        // per snapshot key, its values in both maps (once per snapshot and maps)
        if (c->pa_iv_gen[0] != c->pa_gen || c->pa_iv_gen[1] != c->snap_gen)
        {
            if (!c->pa_key_val.ensure(2 * sizeof(PaValue) * c->ds.n_keys)) return c->fail(AD_E_NOMEM, "preaccept key values");
            HIPCHK(c, run_preaccept_key_values(a.mc, a.rb, c->ds.keys, c->ds.n_keys, c->pa_key_val.as<PaValue>(), st));
            c->pa_iv_gen[0] = c->pa_gen;
            c->pa_iv_gen[1] = c->snap_gen;
        }
        a.khash = c->ds.khash;
        a.khash_mask = c->ds.khash_mask;
        a.key_val = c->pa_key_val.as<PaValue>();
    }
    HIPCHK(c, hipEventRecord(c->ev[6], st));
    HIPCHK(c, run_preaccept(a, st));
    HIPCHK(c, hipEventRecord(c->ev[7], st));
    HIPCHK(c, hipStreamSynchronize(st));
    if (stats)
    {
        float ms = 0;
        HIPCHK(c, hipEventElapsedTime(&ms, c->ev[6], c->ev[7]));
        memset(stats, 0, sizeof(*stats));
        stats->n_txns = q->n_txns;
        stats->ms_device = ms;
        stats->ms_stage[0] = ms;
    }
    return AD_OK;
}

int ad_set_global_dict(ad_ctx* c, uint64_t n, const uint64_t* msb, const uint64_t* lsb, const int32_t* node)
{
    if (!c || (n && (!msb || !lsb || !node))) return AD_E_INVAL;
    if (n >= (1ull << 31)) return c->fail(AD_E_CAPACITY, "ad_set_global_dict: more than 2^31 ids");
    if (!c->cfk.loaded) return c->fail(AD_E_NOT_LOADED, "ad_cfk_load not called");
    if (hipSetDevice(c->device) != hipSuccess) return c->fail(AD_E_DEVICE, "hipSetDevice");
    StreamScope scope_(c->stream, c->cstream);
    for (uint64_t i = 1; i < n; ++i)
        if (norm_cmp(norm_tid(msb[i - 1], lsb[i - 1], node[i - 1]), norm_tid(msb[i], lsb[i], node[i])) >= 0)
            return c->fail(AD_E_INVAL, "ad_set_global_dict: ids not ascending and unique at %llu", (unsigned long long)i);
    // the snapshot is rebuilt over the node-wide dictionary (ingest work): its ranks become global
    c->gd_msb.assign(msb, msb + n);
    c->gd_lsb.assign(lsb, lsb + n);
    c->gd_node.assign(node, node + n);
    c->gd_set = true;
    c->gd_strict = true;
    c->dirty = true;
    const int rc = build_snapshot(c);
    c->gd_strict = false;
    if (rc)
    {
        drop_global_dict(c);
        c->dirty = true;
        return rc;
    }
    return AD_OK;
}

}  // extern "C"

// Export, phase 1 (ad_parts_export, ad_exchange, ad_exchange_local): validate, bind the export
// arguments and enqueue the size pass; c->x_cnt then holds the cumulative [n_dest + 1][4] bounds
// {parts, key words, ids, k2t} of the destinations. Nothing is read back.
static int export_sizes(ad_ctx* c, const ad_deps_result* res, const int64_t* txn_index, uint32_t n_dest,
                        const uint64_t* dest_first, uint32_t id_format, hipStream_t st, ExportArgs* pa)
{
    if (int rc = host_dict(c)) return rc;
    if (!res || !dest_first || n_dest == 0) return c->fail(AD_E_INVAL, "export: result, dest_first and n_dest are required");
    if (c->dirty) return c->fail(AD_E_NOT_LOADED, "export: no prepared snapshot");
    const uint64_t n = res->n_txns;
    if (n && !txn_index) return c->fail(AD_E_INVAL, "export: txn_index is NULL");
    if (dest_first[0] != 0 || dest_first[n_dest] != n) return c->fail(AD_E_INVAL, "export: dest_first must span [0, n)");
    for (uint32_t d = 0; d < n_dest; ++d)
        if (dest_first[d] > dest_first[d + 1]) return c->fail(AD_E_INVAL, "export: dest_first not ascending");
    // the id format is the caller's: its ids buffer was sized for it (cap_ids counts ids of that format)
    if (id_format != AD_IDS_RANK && id_format != AD_IDS_TRIPLET)
        return c->fail(AD_E_INVAL, "export: unknown id_format %u", id_format);
    if (id_format == AD_IDS_RANK && !c->global_ok)
        return c->fail(AD_E_STATE, "export: rank-format parts need a global dictionary covering this store's "
                                   "ids (ad_set_global_dict after the last snapshot load or dictionary append)");
    if (hipSetDevice(c->device) != hipSuccess) return c->fail(AD_E_DEVICE, "hipSetDevice");
    StreamScope scope_(c->stream, c->cstream);
    if (!ens<uint32_t>(c->x_sz, std::max<uint64_t>(n, 1)) || !ens<uint64_t>(c->x_off, n + 1) ||
        !ens<uint64_t>(c->x_bsum, (n + 1023) / 1024 + 16) || !ens<uint64_t>(c->x_df, n_dest + 1) ||
        !ens<uint64_t>(c->x_cnt, 4 * (n_dest + 1)))
        return c->fail(AD_E_NOMEM, "export buffers");
    ExportArgs a{};
    a.n = n;
    for (int m = 0; m < 3; ++m)
    {
        a.keys_off[m] = res->keys_off[m]; a.keys[m] = res->keys[m];
        a.txn_off[m] = res->txn_off[m]; a.txns[m] = res->txns[m];
        a.k2t_off[m] = res->k2t_off[m]; a.k2t[m] = res->k2t[m];
    }
    a.txn_index = txn_index;
    a.ids_per_req = n ? (res->stats.n_unique[0] + res->stats.n_unique[1] + res->stats.n_unique[2]) / n : 0;
    if (!res->keys[0] || !res->txns[0] || !res->k2t[0])
    {
        // a parts-only result: read the batch's regions (still valid: no batch since)
        if (!c->last_parts_only || c->last_n != n)
            return c->fail(AD_E_INVAL, "export: result without packed arrays is not the ctx's last batch");
        a.reg = c->last_reg;
        a.t_reg = c->last_t_reg;
    }
    a.dict_msb = c->d_dict_hi.as<uint64_t>();
    a.dict_lsb = c->d_dict_lsb_raw.as<uint64_t>();
    a.dict_node = c->d_dict_node.as<int32_t>();
    a.rt_start = c->d_rt_start.as<int64_t>();
    a.rt_end = c->d_rt_end.as<int64_t>();
    a.rank_ids = id_format == AD_IDS_RANK;      // the dictionary is the global one: ids are global ranks
    a.sz = c->x_sz.as<uint32_t>();
    a.off = c->x_off.as<uint64_t>();
    HIPCHK(c, up_small(c, 0, c->x_df.p, dest_first, sizeof(uint64_t) * (n_dest + 1), st));
    HIPCHK(c, run_export_sizes(a, st));
    HIPCHK(c, run_scan_arrays(a.sz, a.off, n, 1, c->x_bsum.as<uint64_t>(), st));
    HIPCHK(c, run_export_bounds(a, c->x_df.as<uint64_t>(), n_dest, c->x_cnt.as<uint64_t>(), st));
    *pa = a;
    return AD_OK;
}

// Export, phase 2: the parts into arrays sized from phase 1's bounds (grouped by destination)
static int export_emit(ad_ctx* c, ExportArgs& a, int64_t* hdr, int64_t* keys, int64_t* ids, int32_t* k2t, hipStream_t st)
{
    a.hdr = hdr; a.okeys = keys; a.oids = ids; a.ok2t = k2t;
    HIPCHK(c, run_export_emit(a, st));
    return AD_OK;
}

extern "C" {

int ad_parts_export(ad_ctx* c, const ad_deps_result* res, const int64_t* txn_index, uint32_t n_dest,
                    const uint64_t* dest_first, void* stream, ad_parts* out, uint64_t* dest_counts)
{
    if (!c || !res || !out || !dest_first || !dest_counts || n_dest == 0) return AD_E_INVAL;
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    StreamScope scope_(st, c->stream, c->cstream);
    ExportArgs a{};
    if (int rc = export_sizes(c, res, txn_index, n_dest, dest_first, out->id_format, st, &a)) return rc;
    std::vector<uint64_t> cnt(4 * (n_dest + 1));
    HIPCHK(c, d2h(cnt.data(), c->x_cnt.p, sizeof(uint64_t) * cnt.size(), st));
    HIPCHK(c, hipStreamSynchronize(st));
    out->n_parts = cnt[4 * n_dest + 0];
    out->n_key_words = cnt[4 * n_dest + 1];
    out->n_ids = cnt[4 * n_dest + 2];
    out->n_k2t = cnt[4 * n_dest + 3];
    for (uint32_t d = 0; d < n_dest; ++d)
        for (int k = 0; k < 4; ++k) dest_counts[4 * d + k] = cnt[4 * (d + 1) + k] - cnt[4 * d + k];
    if (out->n_parts > out->cap_parts || out->n_key_words > out->cap_key_words || out->n_ids > out->cap_ids ||
        out->n_k2t > out->cap_k2t)
    {
        c->fail(AD_E_SPACE, "ad_parts_export: buffers too small (need %llu parts, %llu key words, %llu ids, %llu k2t)",
                (unsigned long long)out->n_parts, (unsigned long long)out->n_key_words,
                (unsigned long long)out->n_ids, (unsigned long long)out->n_k2t);
        return AD_E_SPACE;
    }
    return export_emit(c, a, out->hdr, out->keys, out->ids, out->k2t, st);
}

// The end of a merge once its kernels and read-backs are queued: one synchronisation, then the result's
// views (parts_merge with a MergeTail returns before it, so that ad_exchange_local's owners merge at once)
struct MergeTail {
    hipStream_t st;
    MergeArgs a;
    bool by_request, rank_ids;
    uint64_t n_owned, txn_base;
};

static int merge_malformed(ad_ctx* c, uint32_t e)
{
    return c->fail(AD_E_INVAL, "ad_parts_merge: malformed parts (%s)",
                   e & 1  ? "request outside the owned range or bad map" :
                   e & 2  ? "two parts of one request and map from one source" :
                   e & 4  ? "keys of different stores overlap or are out of slice order" :
                   e & 16 ? "id rank outside the global dictionary" :
                            "ids of a part not sorted and unique");
}

static int merge_tail(ad_ctx* c, const MergeTail& t, ad_merged* out)
{
    const MergeArgs& a = t.a;
    const uint64_t n_owned = t.n_owned;
    uint64_t bases[12];
    uint32_t err = 0;
    uint64_t* rb = c->h_rb;             // filled by parts_merge's last copies
    if (hipSetDevice(c->device) != hipSuccess) return c->fail(AD_E_DEVICE, "hipSetDevice");
    HIPCHK(c, hipStreamSynchronize(t.st));
    memcpy(bases, rb, sizeof(bases));
    memcpy(&err, rb + 12, sizeof(err));
    if (err) return merge_malformed(c, err);
    float ms = 0;
    HIPCHK(c, hipEventElapsedTime(&ms, c->ev[6], c->ev[7]));
    memset(out, 0, sizeof(*out));
    out->n_txns = n_owned;
    out->txn_base = t.txn_base;
    out->ms_device = ms;
    out->id_format = t.rank_ids ? AD_IDS_RANK : AD_IDS_TRIPLET;
    for (int m = 0; m < 3; ++m)
    {
        if (t.by_request)
        {
            // the scan of the size pass is the merged CSR: [k*3 + m][n_owned + 1]
            out->keys_off[m] = a.goff + (uint64_t)(0 * 3 + m) * (n_owned + 1);
            out->txn_off[m] = a.goff + (uint64_t)(1 * 3 + m) * (n_owned + 1);
            out->k2t_off[m] = a.goff + (uint64_t)(2 * 3 + m) * (n_owned + 1);
        }
        else
        {
            out->keys_off[m] = a.o_keys_off + (uint64_t)m * (n_owned + 1);
            out->txn_off[m] = a.o_txn_off + (uint64_t)m * (n_owned + 1);
            out->k2t_off[m] = a.o_k2t_off + (uint64_t)m * (n_owned + 1);
        }
        out->keys[m] = a.o_keys + bases[3 * m + 0];
        out->txns[m] = t.rank_ids ? reinterpret_cast<int64_t*>(reinterpret_cast<uint32_t*>(a.o_ids) + bases[3 * m + 1])
                                  : a.o_ids + 3 * bases[3 * m + 1];
        out->k2t[m] = a.o_k2t + bases[3 * m + 2];
        out->n_keys[m] = (bases[3 * (m + 1) + 0] - bases[3 * m + 0]) / (m == AD_MAP_RANGE ? 2 : 1);
        out->n_ids[m] = bases[3 * (m + 1) + 1] - bases[3 * m + 1];
        out->n_k2t[m] = bases[3 * (m + 1) + 2] - bases[3 * m + 2];
    }
    return AD_OK;
}

static int parts_merge(ad_ctx* c, const ad_parts* in, uint32_t n_src, const uint64_t* src_parts, uint64_t txn_base,
                       uint64_t n_owned, void* stream, ad_merged* out, bool union_keys, MergeTail* defer = nullptr)
{
    if (!c || !in || !src_parts || !out || n_src == 0 || n_src > 64) return AD_E_INVAL;
    if (union_keys && in->id_format != AD_IDS_RANK)
        return c->fail(AD_E_INVAL, "ad_parts_union: parts must carry global ranks (ad_set_global_dict)");
    uint64_t tot = 0;
    std::vector<uint64_t> first(n_src + 1, 0);
    for (uint32_t s = 0; s < n_src; ++s) first[s + 1] = (tot += src_parts[s]);
    if (tot != in->n_parts) return c->fail(AD_E_INVAL, "ad_parts_merge: src_parts do not sum to n_parts");
    if (hipSetDevice(c->device) != hipSuccess) return c->fail(AD_E_DEVICE, "hipSetDevice");
    StreamScope scope_(c->stream, c->cstream);
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    scope_.add(st);
    const uint64_t P = in->n_parts, G = 3 * n_owned;
    const bool rank_ids = in->id_format == AD_IDS_RANK;
    if (in->id_format != AD_IDS_TRIPLET && !rank_ids) return c->fail(AD_E_INVAL, "ad_parts_merge: unknown id_format");
    // rank-format merge of a node's stores: one 16-lane group per owned request (K3 fast path)
    const bool by_request = rank_ids && !union_keys && n_src <= RM_MAX_SRC && in->n_key_words < (1ull << 32) &&
                            in->n_ids < (1ull << 32) && in->n_k2t < (1ull << 32) && n_owned < (1ull << 30) &&
                            in->n_parts < (1ull << 30);
    if (rank_ids && !c->global_ok)
        return c->fail(AD_E_INVAL, "ad_parts_merge: rank-format parts need ad_set_global_dict on this ctx");
    if (rank_ids && (!ens<uint32_t>(c->m_u, in->n_ids) || !ens<uint32_t>(c->m_ppre, 4 * std::max<uint64_t>(P, 1))))
        return c->fail(AD_E_NOMEM, "merge buffers");
    if (union_keys && (!ens<uint32_t>(c->m_kdp, in->n_key_words) || !ens<uint32_t>(c->m_kuk, in->n_key_words) ||
                       !ens<uint32_t>(c->m_khead, in->n_key_words) || !ens<uint32_t>(c->m_pdp, in->n_k2t) ||
                       !ens<uint32_t>(c->m_ppos, in->n_k2t)))
        return c->fail(AD_E_NOMEM, "union buffers");
    if (!ens<uint64_t>(c->m_src, n_src + 1) || !ens<uint32_t>(c->m_psz, 3 * P) || !ens<uint64_t>(c->m_poff, 3 * (P + 1)) ||
        !ens<int32_t>(c->m_slot, G * n_src) || !ens<uint32_t>(c->m_dup, in->n_ids) || !ens<uint32_t>(c->m_gsz, 3 * G) ||
        !ens<uint64_t>(c->m_goff, 3 * (G + 1) + 9) ||
        !ens<uint64_t>(c->m_bsum, 3 * ((std::max(P, G) + 1023) / 1024) + 16) || !ens<uint32_t>(c->m_err, 1) ||
        !ens<uint64_t>(c->m_bases, 16) || !ens<uint64_t>(c->m_ko, 3 * (n_owned + 1)) ||
        !ens<uint64_t>(c->m_to, 3 * (n_owned + 1)) || !ens<uint64_t>(c->m_oo, 3 * (n_owned + 1)) ||
        (by_request && (!ens<uint32_t>(c->m_pinfo, 8 * std::max<uint64_t>(P, 1)) ||
                        !ens<uint32_t>(c->m_heavy, 3 * std::max<uint64_t>(n_owned, 1) + 1) ||
                        !ens<uint64_t>(c->m_bsum, 9 * ((n_owned + 1023) / 1024) + 16))))
        return c->fail(AD_E_NOMEM, "merge buffers");
    // a merged map is never larger than what it merges: the by-request path sizes its outputs by the
    // received totals and needs no host round trip before the emit pass
    if (by_request && (!ens<int64_t>(c->m_keys, in->n_key_words) || !ens<int64_t>(c->m_ids, (in->n_ids + 1) / 2) ||
                       !ens<int32_t>(c->m_k2t, in->n_k2t)))
        return c->fail(AD_E_NOMEM, "merge outputs");
    MergeArgs a{};
    a.n_parts = P;
    a.n_elems = in->n_key_words + in->n_ids + in->n_k2t;
    a.n_owned = n_owned;
    a.txn_base = txn_base;
    a.n_src = n_src;
    a.src_first = c->m_src.as<uint64_t>();
    a.hdr = in->hdr; a.keys = in->keys; a.ids = in->ids; a.k2t = in->k2t;
    a.psz = c->m_psz.as<uint32_t>();
    a.poff = c->m_poff.as<uint64_t>();
    a.slot = c->m_slot.as<int32_t>();
    a.dup = c->m_dup.as<uint32_t>();
    a.pinfo = by_request ? c->m_pinfo.as<uint32_t>() : nullptr;
    a.heavy = by_request ? c->m_heavy.as<uint32_t>() + 1 : nullptr;
    a.n_heavy = by_request ? c->m_heavy.as<uint32_t>() : nullptr;
    a.gsz = c->m_gsz.as<uint32_t>();
    a.goff = c->m_goff.as<uint64_t>();
    a.error = c->m_err.as<uint32_t>();
    a.o_keys_off = c->m_ko.as<uint64_t>();
    a.o_txn_off = c->m_to.as<uint64_t>();
    a.o_k2t_off = c->m_oo.as<uint64_t>();
    if (rank_ids)
    {
        a.u = c->m_u.as<uint32_t>();
        a.ppre = c->m_ppre.as<uint32_t>();
        a.n_global = c->n_global;
    }
    if (union_keys)
    {
        a.kdp = c->m_kdp.as<uint32_t>(); a.kuk = c->m_kuk.as<uint32_t>(); a.khead = c->m_khead.as<uint32_t>();
        a.pdp = c->m_pdp.as<uint32_t>(); a.ppos = c->m_ppos.as<uint32_t>();
    }
    HIPCHK(c, hipEventRecord(c->ev[6], st));
    HIPCHK(c, up_small(c, 1, c->m_src.p, first.data(), sizeof(uint64_t) * (n_src + 1), st));
    HIPCHK(c, hipMemsetAsync(a.error, 0, sizeof(uint32_t), st));
    HIPCHK(c, hipMemsetAsync(a.slot, 0xFF, sizeof(int32_t) * std::max<uint64_t>((by_request ? n_owned : G) * n_src, 1), st));
    HIPCHK(c, run_merge_prepare(a, st));
    HIPCHK(c, run_scan_arrays(a.psz, a.poff, P, 3, c->m_bsum.as<uint64_t>(), st));
    if (by_request)
    {
        HIPCHK(c, run_rmerge_slots(a, st));
        HIPCHK(c, run_rmerge_size(a, st));
        // per map and array: offsets of the owned requests' merged maps, each map from 0
        HIPCHK(c, run_scan_arrays(a.gsz, a.goff, n_owned, 9, c->m_bsum.as<uint64_t>(), st));
    }
    else
    {
        HIPCHK(c, run_merge_slots(a, st));
        HIPCHK(c, union_keys ? run_union_rank(a, st) : rank_ids ? run_merge_rank(a, st) : run_merge_count(a, st));
        HIPCHK(c, run_scan_arrays(a.gsz, a.goff, G, 3, c->m_bsum.as<uint64_t>(), st));
        HIPCHK(c, run_merge_bases(a, c->m_bases.as<uint64_t>(), st));
    }
    uint64_t bases[12];
    uint32_t err = 0;
    if (n_owned == 0 && !by_request)
        for (DevBuf* b : {&c->m_ko, &c->m_to, &c->m_oo}) HIPCHK(c, hipMemsetAsync(b->p, 0, sizeof(uint64_t) * 3, st));
    if (!by_request)
    {
        // outputs sized from the scanned group sizes (one round trip)
        uint64_t* rb = rb_slot(c);
        if (!rb) return c->fail(AD_E_NOMEM, "pinned read-back words");
        HIPCHK(c, hipMemcpyAsync(rb, c->m_bases.p, sizeof(bases), hipMemcpyDeviceToHost, st));
        HIPCHK(c, hipMemcpyAsync(rb + 12, a.error, sizeof(err), hipMemcpyDeviceToHost, st));
        HIPCHK(c, hipStreamSynchronize(st));
        memcpy(bases, rb, sizeof(bases));
        memcpy(&err, rb + 12, sizeof(err));
        if (err) return merge_malformed(c, err);
        // bases[3*m + k]: offset of map m's first group in array k (m = 3: totals)
        if (!ens<int64_t>(c->m_keys, bases[9]) || !ens<int64_t>(c->m_ids, rank_ids ? (bases[10] + 1) / 2 : 3 * bases[10]) ||
            !ens<int32_t>(c->m_k2t, bases[11]))
            return c->fail(AD_E_NOMEM, "merge outputs");
    }
    a.o_keys = c->m_keys.as<int64_t>();
    a.o_ids = c->m_ids.as<int64_t>();
    a.o_k2t = c->m_k2t.as<int32_t>();
    HIPCHK(c, by_request ? run_rmerge_copy(a, c->m_bases.as<uint64_t>(), st)
                         : union_keys ? run_union_emit(a, st) : rank_ids ? run_merge_emit_rank(a, st) : run_merge_emit(a, st));
    HIPCHK(c, hipEventRecord(c->ev[7], st));
    uint64_t* rb = rb_slot(c);
    if (!rb) return c->fail(AD_E_NOMEM, "pinned read-back words");
    // the bases (by request: the device's; else the host's, as the emit used them) and the error word
    if (by_request) HIPCHK(c, hipMemcpyAsync(rb, c->m_bases.p, sizeof(bases), hipMemcpyDeviceToHost, st));
    else memcpy(rb, bases, sizeof(bases));
    HIPCHK(c, hipMemcpyAsync(rb + 12, a.error, sizeof(err), hipMemcpyDeviceToHost, st));
    const MergeTail t{st, a, by_request, rank_ids, n_owned, txn_base};
    if (defer)
    {
        *defer = t;
        return AD_OK;
    }
    return merge_tail(c, t, out);
}

int ad_parts_merge(ad_ctx* c, const ad_parts* in, uint32_t n_src, const uint64_t* src_parts, uint64_t txn_base,
                   uint64_t n_owned, void* stream, ad_merged* out)
{
    return parts_merge(c, in, n_src, src_parts, txn_base, n_owned, stream, out, false);
}

int ad_parts_union(ad_ctx* c, const ad_parts* in, uint32_t n_src, const uint64_t* src_parts, uint64_t txn_base,
                   uint64_t n_owned, void* stream, ad_merged* out)
{
    return parts_merge(c, in, n_src, src_parts, txn_base, n_owned, stream, out, true);
}

int ad_copy_to_host(ad_ctx* c, void* dst, const void* src, uint64_t bytes)
{
    if (!c || (!dst && bytes) || (!src && bytes)) return AD_E_INVAL;
    if (!bytes) return AD_OK;
    if (hipSetDevice(c->device) != hipSuccess) return c->fail(AD_E_DEVICE, "hipSetDevice");
    StreamScope scope_(c->stream, c->cstream);
    HIPCHK(c, copy_sync(dst, src, bytes, hipMemcpyDeviceToHost));
    return AD_OK;
}

static int levels_run(ad_ctx* c, const LevelsIn& in, uint32_t* out_dev, hipStream_t st, ad_stats* stats)
{
    if (!c->lv) c->lv = levels_work_create();
    LevelsOut lo;
    std::string err;
    const int rc = run_levels(c->lv, in, out_dev, st, &lo, &err);
    if (rc) return c->fail(rc, "%s", err.c_str());
    if (stats)
    {
        std::memset(stats, 0, sizeof(*stats));
        stats->n_txns = in.n;
        stats->n_probes = lo.n_occ;
        stats->ms_device = lo.ms_total;
        stats->ms_stage[0] = lo.ms_build;
        stats->ms_stage[1] = lo.ms_frontier;
        stats->n_levels = lo.n_levels;
        stats->n_edges = lo.n_edges;
        stats->n_launches = lo.n_launch;
        stats->n_deferred = lo.packed ? 1 : 0;
        // algorithmic bytes: nodes x (8 B executeAt + 4 B offset + 4 B level)
        // + edges x 4 B; the build additionally reads the key occurrences (8 B each) once
        stats->bytes_stage[0] = in.n * 16 + lo.n_occ * 8;
        stats->bytes_stage[1] = in.n * 8 + lo.n_edges * 4;
    }
    return AD_OK;
}

int ad_levels_device(ad_ctx* c, const ad_graph_soa* g, uint32_t* level_out, void* stream, ad_stats* stats)
{
    if (!c || !g) return AD_E_INVAL;
    if (g->n_txns && (!g->exec_msb || !g->exec_lsb || !g->exec_node || !g->kind || !g->key_off || !level_out))
        return c->fail(AD_E_INVAL, "ad_levels_device: null array");
    if (hipSetDevice(c->device) != hipSuccess) return c->fail(AD_E_DEVICE, "hipSetDevice");
    StreamScope scope_(c->stream, c->cstream);
    scope_.add((hipStream_t)stream);
    LevelsIn in{g->n_txns, g->exec_msb, g->exec_lsb, g->exec_node, g->kind, g->key_off, g->keys, g->dep_off, g->deps};
    return levels_run(c, in, level_out, stream ? (hipStream_t)stream : c->stream, stats);
}

int ad_levels(ad_ctx* c, const ad_graph_soa* g, uint32_t* level_out, ad_stats* stats)
{
    if (!c || !g) return AD_E_INVAL;
    const uint64_t n = g->n_txns;
    if (n && (!g->exec_msb || !g->exec_lsb || !g->exec_node || !g->kind || !g->key_off || !level_out))
        return c->fail(AD_E_INVAL, "ad_levels: null array");
    if (n && g->key_off[0] != 0) return c->fail(AD_E_INVAL, "ad_levels: key_off must start at 0");
    if (hipSetDevice(c->device) != hipSuccess) return c->fail(AD_E_DEVICE, "hipSetDevice");
    StreamScope scope_(c->stream, c->cstream);
    if (n == 0)
    {
        if (stats) std::memset(stats, 0, sizeof(*stats));
        return AD_OK;
    }
    const uint64_t nk = g->key_off[n];
    if (nk && !g->keys) return c->fail(AD_E_INVAL, "ad_levels: null keys");
    const uint64_t nd = g->dep_off ? g->dep_off[n] : 0;
    if (g->dep_off && nd && !g->deps) return c->fail(AD_E_INVAL, "ad_levels: null deps");
    auto up = [&](DevBuf& b, const void* src, size_t bytes) -> int {
        if (!b.ensure(std::max<size_t>(bytes, 8))) return c->fail(AD_E_NOMEM, "hipMalloc %zu", bytes);
        if (bytes) HIPCHK(c, h2d(b.p, src, bytes, c->stream));
        return 0;
    };
    int rc;
    if ((rc = up(c->g_em, g->exec_msb, 8 * n)) || (rc = up(c->g_el, g->exec_lsb, 8 * n)) ||
        (rc = up(c->g_en, g->exec_node, 4 * n)) || (rc = up(c->g_kind, g->kind, n)) ||
        (rc = up(c->g_ko, g->key_off, 8 * (n + 1))) || (rc = up(c->g_k, g->keys, 8 * nk)))
        return rc;
    if (g->dep_off && ((rc = up(c->g_do, g->dep_off, 8 * (n + 1))) || (rc = up(c->g_d, g->deps, 4 * nd)))) return rc;
    if (!c->g_out.ensure(4 * n)) return c->fail(AD_E_NOMEM, "hipMalloc levels");
    LevelsIn in{n, c->g_em.as<uint64_t>(), c->g_el.as<uint64_t>(), c->g_en.as<int32_t>(), c->g_kind.as<uint8_t>(),
                c->g_ko.as<uint64_t>(), c->g_k.as<int64_t>(), g->dep_off ? c->g_do.as<uint64_t>() : nullptr,
                g->dep_off ? c->g_d.as<uint32_t>() : nullptr};
    if ((rc = levels_run(c, in, c->g_out.as<uint32_t>(), c->stream, stats))) return rc;
    HIPCHK(c, d2h(level_out, c->g_out.p, 4 * n, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return AD_OK;
}

// ---- device-resident CommandsForKey maintenance ----------------------------
static int cfk_need_bufs(void* vc, uint64_t n_cand, uint64_t n_cwr, uint64_t n_w, CfkDerivedBufs* b)
{
    ad_ctx* c = (ad_ctx*)vc;
    if (!c->d_cand.ensure(4 * std::max<uint64_t>(n_cand, 1)) || !c->d_cwr.ensure(4 * std::max<uint64_t>(n_cwr, 1)) ||
        !c->d_w.ensure(8 * std::max<uint64_t>(n_w, 1)))
        return AD_E_NOMEM;
    b->cand = c->d_cand.as<uint32_t>();
    b->cwr = c->d_cwr.as<uint32_t>();
    b->w = c->d_w.as<uint2>();
    return 0;
}

// DevBuf growth keeping the first `keep` bytes (slack for the next batches)
static bool grow_keep(DevBuf& b, size_t keep, size_t need)
{
    if (b.p && need <= b.cap) return true;
    const size_t cap = std::max<size_t>(need + need / 2, 64);
    void* p = dev_alloc(cap);
    if (!p) return false;
    // the kept bytes were written on the call's stream: the copy is ordered after them there
    const hipStream_t st = dev_scope_stream();
    if (keep && (hipMemcpyAsync(p, b.p, keep, hipMemcpyDeviceToDevice, st) != hipSuccess ||
                 (st ? hipStreamSynchronize(st) : hipDeviceSynchronize()) != hipSuccess))
    {
        dev_free(p);
        return false;
    }
    b.release();
    b.p = p;
    b.cap = cap;
    return true;
}

static int cfk_grow_dict(void* vc, uint64_t n_old, uint64_t n_new, uint64_t** hi, uint64_t** lo, int32_t** node, uint64_t** raw)
{
    ad_ctx* c = (ad_ctx*)vc;
    if (!grow_keep(c->d_dict_hi, 8 * n_old, 8 * n_new) || !grow_keep(c->d_dict_lo, 8 * n_old, 8 * n_new) ||
        !grow_keep(c->d_dict_node, 4 * n_old, 4 * n_new) || !grow_keep(c->d_dict_lsb_raw, 8 * n_old, 8 * n_new))
        return AD_E_NOMEM;
    *hi = c->d_dict_hi.as<uint64_t>();
    *lo = c->d_dict_lo.as<uint64_t>();
    *node = c->d_dict_node.as<int32_t>();
    *raw = c->d_dict_lsb_raw.as<uint64_t>();
    return 0;
}

static int cfk_grow_entries(void* vc, uint64_t ne, uint2** ent, uint8_t** st, uint32_t** xr, uint32_t** ek, Bal** bal,
                            uint32_t** mref)
{
    ad_ctx* c = (ad_ctx*)vc;
    const uint64_t padded = std::max<uint64_t>(64, (ne + 63) / 64 * 64);
    if (!grow_keep(c->d_ent2, 0, 8 * padded) || !grow_keep(c->d_status2, 0, ne) || !grow_keep(c->d_xrank2, 0, 4 * ne) ||
        !grow_keep(c->d_ekey2, 0, 4 * ne))
        return AD_E_NOMEM;
    *bal = nullptr;
    if (c->d_ballot.p)
    {
        if (!grow_keep(c->d_ballot2, 0, sizeof(Bal) * ne)) return AD_E_NOMEM;
        *bal = c->d_ballot2.as<Bal>();
    }
    *mref = nullptr;
    if (c->dmiss_on)
    {
        if (!grow_keep(c->d_mref2, 0, 4 * ne)) return AD_E_NOMEM;
        *mref = c->d_mref2.as<uint32_t>();
    }
    *ent = c->d_ent2.as<uint2>();
    *st = c->d_status2.as<uint8_t>();
    *xr = c->d_xrank2.as<uint32_t>();
    *ek = c->d_ekey2.as<uint32_t>();
    return 0;
}

static void swap_buf(DevBuf& a, DevBuf& b)
{
    std::swap(a.p, b.p);
    std::swap(a.cap, b.cap);
}

static int size_cfk_trees(ad_ctx* c, uint64_t ne)
{
    DevSnapshot& s = c->ds;
    s.n_ent = ne;
    s.ent = c->d_ent.as<uint2>();
    s.lvl_n[0] = ne;
    int L = 1;
    while (s.lvl_n[L - 1] > 64 && L < MAX_LEVELS)
    {
        s.lvl_n[L] = (s.lvl_n[L - 1] + 63) / 64;
        ++L;
    }
    s.n_levels = L;
    for (int l = 1; l < L; ++l)
        for (int cl = 0; cl < NCLASS; ++cl)
        {
            if (!c->d_lvl[cl][l].ensure(sizeof(uint32_t) * ((s.lvl_n[l] + 63) / 64 * 64))) return AD_E_NOMEM;
            s.lvl[cl][l] = c->d_lvl[cl][l].as<uint32_t>();
        }
    return 0;
}

static int cfk_swap_entries(void* vc, uint64_t ne, uint2** ent, uint8_t** st, uint32_t** xr, uint32_t** ek, Bal** bal,
                            uint32_t** mref)
{
    ad_ctx* c = (ad_ctx*)vc;
    swap_buf(c->d_ent, c->d_ent2);
    swap_buf(c->d_status, c->d_status2);
    swap_buf(c->d_xrank, c->d_xrank2);
    swap_buf(c->d_ekey, c->d_ekey2);
    if (c->d_ballot.p) swap_buf(c->d_ballot, c->d_ballot2);
    if (c->dmiss_on) swap_buf(c->d_mref, c->d_mref2);
    *mref = c->dmiss_on ? c->d_mref.as<uint32_t>() : nullptr;
    *bal = c->d_ballot.as<Bal>();
    *ent = c->d_ent.as<uint2>();
    *st = c->d_status.as<uint8_t>();
    *xr = c->d_xrank.as<uint32_t>();
    *ek = c->d_ekey.as<uint32_t>();
    return size_cfk_trees(c, ne);
}

static int cfk_ballot_init(void* vc, uint64_t ne, Bal** bal)
{
    ad_ctx* c = (ad_ctx*)vc;
    if (!c->d_ballot.ensure(sizeof(Bal) * ne + sizeof(Bal) * (ne / 4))) return AD_E_NOMEM;
    if (dev_zero_sync(c->d_ballot.p, sizeof(Bal) * ne) != hipSuccess) return AD_E_DEVICE;
    *bal = c->d_ballot.as<Bal>();
    return 0;
}

static int cfk_keys_spare(void* vc, uint64_t nk, KeyBufs* b)
{
    ad_ctx* c = (ad_ctx*)vc;
    uint64_t hcap = 16;
    while (hcap < 2 * nk) hcap <<= 1;
    const uint64_t slack = nk / 8;
    if (!c->d_keys2.ensure(8 * (nk + slack)) || !c->d_krec2.ensure(sizeof(KeyRec) * (nk + slack)) ||
        !c->d_kcell2.ensure(4 * (nk + slack)) || !c->d_khash2.ensure(sizeof(KeySlot) * hcap) ||
        !c->d_kent2.ensure(sizeof(KeyEntry) * (nk + slack)))
        return AD_E_NOMEM;
    *b = KeyBufs{c->d_keys2.as<int64_t>(), c->d_krec2.as<KeyRec>(), c->d_kcell2.as<uint32_t>(), c->d_khash2.as<KeySlot>(),
                 c->d_kent2.as<KeyEntry>(), hcap};
    return 0;
}

static int cfk_keys_swap(void* vc, KeyBufs* b)
{
    ad_ctx* c = (ad_ctx*)vc;
    swap_buf(c->d_keys, c->d_keys2);
    swap_buf(c->d_krec, c->d_krec2);
    swap_buf(c->d_kcell, c->d_kcell2);
    swap_buf(c->d_khash, c->d_khash2);
    swap_buf(c->d_kent, c->d_kent2);
    b->keys = c->d_keys.as<int64_t>();
    b->krec = c->d_krec.as<KeyRec>();
    b->kcell = c->d_kcell.as<uint32_t>();
    b->khash = c->d_khash.as<KeySlot>();
    b->kent = c->d_kent.as<KeyEntry>();
    return 0;
}

// After new keys on the device: the KeyLine perfect hash takes them (incrementally on the host),
// displacements uploaded, every key's line recomputed on the device.
static int cfk_after_new_keys(ad_ctx* c, const CfkUpdOut& o, hipStream_t st)
{
    const uint64_t nk = c->ds.n_keys, U = o.n_new_keys;
    std::vector<int64_t> nkeys(U);
    HIPCHK(c, d2h(nkeys.data(), o.new_keys, 8 * U, st));
    HIPCHK(c, hipStreamSynchronize(st));
    bool rebuild = false;
    if (int rc = kl_add_keys(c, nkeys, nk, &rebuild)) return rc;
    if (rebuild)
    {
        // the whole table again, half full (every key of the store, from the device)
        std::vector<int64_t> all(nk);
        HIPCHK(c, copy_sync(all.data(), c->d_keys.p, 8 * nk, hipMemcpyDeviceToHost));
        if (int rc = kl_place_all(c, all, std::max<uint64_t>(1, nk / 4), true)) return c->fail(rc, "key perfect hash did not converge");
    }
    if (int rc = upload(c, c->d_kl_disp, c->kl_disp_h)) return rc;
    if (!c->d_kslot.ensure(4 * nk + 4 * (nk / 8))) return c->fail(AD_E_NOMEM, "key slots");
    if (!c->d_kline.ensure(kline_table_bytes(c->kline_slots))) return c->fail(AD_E_NOMEM, "key lines");
    DevSnapshot& s = c->ds;
    s.kline = c->d_kline.as<KeyLine>();
    s.kl_lines = c->kline_slots;
    s.kquad = kline_quads(s.kline, c->kline_slots);
    s.kl_buckets = c->kl_nb_h;
    s.kl_disp = c->d_kl_disp.as<uint32_t>();
    HIPCHK(c, run_key_slots(c->d_keys.as<int64_t>(), nk, c->d_kl_disp.as<uint32_t>(), c->kl_nb_h, c->kline_slots,
                            c->d_kslot.as<uint32_t>(), st));
    return 0;
}

static int cfk_dict_spare(void* vc, uint64_t n, uint64_t** hi, uint64_t** lo, int32_t** node, uint64_t** raw)
{
    ad_ctx* c = (ad_ctx*)vc;
    if (!c->d_dict_hi2.ensure(8 * n + 8 * (n / 8)) || !c->d_dict_lo2.ensure(8 * n + 8 * (n / 8)) ||
        !c->d_dict_node2.ensure(4 * n + 4 * (n / 8)) || !c->d_dict_raw2.ensure(8 * n + 8 * (n / 8)))
        return AD_E_NOMEM;
    *hi = c->d_dict_hi2.as<uint64_t>();
    *lo = c->d_dict_lo2.as<uint64_t>();
    *node = c->d_dict_node2.as<int32_t>();
    *raw = c->d_dict_raw2.as<uint64_t>();
    return 0;
}

static int cfk_dict_swap(void* vc, uint64_t** hi, uint64_t** lo, int32_t** node, uint64_t** raw)
{
    ad_ctx* c = (ad_ctx*)vc;
    swap_buf(c->d_dict_hi, c->d_dict_hi2);
    swap_buf(c->d_dict_lo, c->d_dict_lo2);
    swap_buf(c->d_dict_node, c->d_dict_node2);
    swap_buf(c->d_dict_lsb_raw, c->d_dict_raw2);
    *hi = c->d_dict_hi.as<uint64_t>();
    *lo = c->d_dict_lo.as<uint64_t>();
    *node = c->d_dict_node.as<int32_t>();
    *raw = c->d_dict_lsb_raw.as<uint64_t>();
    return 0;
}

// After a dictionary merge on the device: the host dictionary copy and the host-side rank arrays
// (r = 2i+1 -> 2(i + #{pos <= i}) + 1, the device remap)
static int cfk_after_merge(ad_ctx* c, const uint64_t* pos_dev, uint64_t U, hipStream_t st)
{
    // (the whole dictionary is read back below; host rank copies that are stale -- host_moved -- are
    // rebuilt from the device later, their remap here is then moot)
    c->host_dict_stale = false;
    const uint64_t nd = c->ds.n_dict;
    std::vector<uint64_t> pos(U);
    c->dict_msb.resize(nd);
    c->dict_lsb.resize(nd);
    c->dict_node.resize(nd);
    HIPCHK(c, d2h(pos.data(), pos_dev, 8 * U, st));
    HIPCHK(c, d2h(c->dict_msb.data(), c->d_dict_hi.p, 8 * nd, st));
    HIPCHK(c, d2h(c->dict_lsb.data(), c->d_dict_lsb_raw.p, 8 * nd, st));
    HIPCHK(c, d2h(c->dict_node.data(), c->d_dict_node.p, 4 * nd, st));
    HIPCHK(c, hipStreamSynchronize(st));
    auto remap = [&](uint32_t r) -> uint32_t {
        if (r == 0) return 0;
        const uint64_t i = (r - 1) / 2;
        return (uint32_t)(2 * (i + (uint64_t)(std::upper_bound(pos.begin(), pos.end(), i) - pos.begin())) + 1);
    };
    auto remap_txw = [&](uint32_t y) -> uint32_t { return (y & ~RANK_MASK) | remap(y & RANK_MASK); };
    for (auto& r : c->h_txn_rank) r = remap(r);
    for (auto& r : c->h_exec_rank) r = remap(r);
    for (auto& r : c->h_pruned) r = remap(r);
    for (auto& r : c->h_cmd_rank) r = remap(r);
    for (auto& y : c->h_rtxw) y = remap_txw(y);
    ++c->rank_gen;
    return 0;
}

static int cfk_miss_spare(void* vc, uint64_t n, uint64_t n_ids, uint64_t** off, uint32_t** ids)
{
    ad_ctx* c = (ad_ctx*)vc;
    if (!c->d_moff2.ensure(8 * (n + 1) + 8 * (n / 8)) || !c->d_mids2.ensure(4 * std::max<uint64_t>(n_ids, 1) + 4 * (n_ids / 8)))
        return AD_E_NOMEM;
    *off = c->d_moff2.as<uint64_t>();
    *ids = c->d_mids2.as<uint32_t>();
    c->dmiss_lists = n;
    c->dmiss_ids = n_ids;
    return 0;
}

static int cfk_miss_swap(void* vc, uint64_t** off, uint32_t** ids)
{
    ad_ctx* c = (ad_ctx*)vc;
    swap_buf(c->d_moff, c->d_moff2);
    swap_buf(c->d_mids, c->d_mids2);
    *off = c->d_moff.as<uint64_t>();
    *ids = c->d_mids.as<uint32_t>();
    return 0;
}

// Start maintaining TxnInfo.missing() on the device: the host lists (NO_TXNIDS everywhere without a
// load) as rank CSR, every entry its own list. 1: the lists cannot go to the device (stale, or an
// id outside the dictionary): they are then marked stale by updates as before.
static int dmiss_enable(ad_ctx* c, hipStream_t st)
{
    if (int rc = sync_host(c)) return rc;
    auto& K = c->cfk;
    if (K.miss_stale) return 1;
    const uint64_t ne = K.status.size();
    std::vector<uint64_t> off(ne + 1, 0);
    std::vector<uint32_t> ids;
    if (!K.miss_off.empty())
    {
        off.assign(K.miss_off.begin(), K.miss_off.end());
        ids.resize(K.miss.size());
        for (size_t j = 0; j < K.miss.size(); ++j)
        {
            const NormTid x = norm(K.miss[j]);
            uint64_t lo = 0, hi = c->dict_msb.size();
            while (lo < hi)
            {
                const uint64_t mid = (lo + hi) >> 1;
                if (norm_cmp(norm_tid(c->dict_msb[mid], c->dict_lsb[mid], c->dict_node[mid]), x) < 0) lo = mid + 1;
                else hi = mid;
            }
            if (lo >= c->dict_msb.size() || norm_cmp(norm_tid(c->dict_msb[lo], c->dict_lsb[lo], c->dict_node[lo]), x) != 0)
                return 1;
            ids[j] = (uint32_t)(2 * lo + 1);
        }
    }
    std::vector<uint32_t> mref(ne);
    for (uint64_t e = 0; e < ne; ++e) mref[e] = (uint32_t)e;
    if (int rc = upload(c, c->d_moff, off)) return rc;
    if (int rc = upload(c, c->d_mids, ids.empty() ? std::vector<uint32_t>(1, 0) : ids)) return rc;
    if (int rc = upload(c, c->d_mref, mref.empty() ? std::vector<uint32_t>(1, 0) : mref)) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->dmiss_lists = ne;
    c->dmiss_ids = ids.size();
    c->dmiss_on = true;
    (void)st;
    return 0;
}

static int cfk_update_follow(ad_ctx* c, const CfkUpdOut& o, int rc, hipStream_t st);

static int cfk_update_run(ad_ctx* c, const CfkUpdIn& u, hipStream_t st, uint64_t* n_applied, ad_stats* stats)
{
    StreamScope scope_(st, c->stream, c->cstream);
    c->upd_applied = false;
    c->upd_failed = -1;
    if (c->dirty)
        if (int rc = build_snapshot(c)) return rc;
    // missing() on the device while batches bring their deps; a batch without deps hands the lists
    // back to the host, where updates mark them stale (recovery then asks for a reload)
    if (u.dep_off && !c->dmiss_on)
    {
        const int rc = dmiss_enable(c, st);
        if (rc < 0) return rc;
    }
    else if (!u.dep_off && c->dmiss_on)
    {
        if (int rc = sync_host(c)) return rc;
        if (c->host_stale == false && c->dmiss_on) { if (int rc = pull_missing(c)) return rc; }
        c->dmiss_on = false;
    }
    if (!c->cu) c->cu = cfk_upd_work_create();
    CfkDevState d{c->d_status.as<uint8_t>(), c->d_xrank.as<uint32_t>(), c->d_ekey.as<uint32_t>(),
                  c->d_dict_lsb_raw.as<uint64_t>(), c->d_ballot.p ? c->d_ballot.as<Bal>() : nullptr,
                  c->dmiss_on ? c->d_mref.as<uint32_t>() : nullptr,
                  c->d_ent.as<uint2>(), c->d_krec.as<KeyRec>(), c->d_kent.as<KeyEntry>()};
    CfkDerivedBufs b{c->d_cand.as<uint32_t>(), c->d_cand.cap / 4, c->d_cwr.as<uint32_t>(), c->d_cwr.cap / 4,
                     c->d_w.as<uint2>(), c->d_w.cap / 8};
    CfkUpdOut o;
    std::string e;
    const CfkGrow grow{c, cfk_grow_dict, cfk_grow_entries, cfk_swap_entries, cfk_ballot_init, cfk_dict_spare, cfk_dict_swap,
                       c->d_rtxw.as<uint32_t>(), c->ds.n_rent, c->d_cell_ent.as<uint64_t>(), c->ds.cell_ent ? c->n_cell_ent : 0,
                       c->d_rb_wm.as<uint32_t>(), c->ds.n_rb, c->dmiss_on ? c->d_mids.as<uint32_t>() : nullptr,
                       c->dmiss_on ? c->dmiss_ids : 0, cfk_keys_spare, cfk_keys_swap,
                       c->d_kcell.p ? c->d_kcell.as<uint32_t>() : nullptr};
    if (int rc = host_dict(c)) return rc;
    CfkMiss miss;
    miss.on = c->dmiss_on && u.dep_off;
    miss.n_lists = c->dmiss_lists;
    miss.off = c->d_moff.as<uint64_t>();
    miss.ids = c->d_mids.as<uint32_t>();
    miss.ctx = c;
    miss.spare = cfk_miss_spare;
    miss.swap = cfk_miss_swap;
    c->lp_upd.clear(); c->lp_keys.clear(); c->lp_msb.clear(); c->lp_lsb.clear(); c->lp_node.clear();
    const int rc = run_cfk_update(c->cu, c->ds, d, u, &b, cfk_need_bufs, c, grow, st, &o, &e, &miss);
    // what the batch left is known here, before any follow-up copy can fail: a caller reading the status after
    // an error must never take a batch that stands for one that did not (and apply it twice)
    c->upd_applied = rc == AD_OK || o.batch_stood;
    c->upd_failed = o.failed_update;
    if (const int frc = cfk_update_follow(c, o, rc, st))
    {
        // the host copies and the derived arrays may be half refreshed: rebuilt from the entries at the next use
        c->host_stale = true;
        c->dirty = true;
        if (c->upd_applied) return c->fail(AD_E_PARTIAL, "explicit updates applied, their follow-up failed: %s", c->err.c_str());
        return frc;
    }
    if (rc && o.batch_stood)
    {
        // the explicit batch stands but what follows it (additions, missing() lists) failed: the entries
        // changed, the device lists are not this batch's -- the host copies follow on demand and the
        // lists ask for a reload (as after a batch without deps)
        c->host_stale = true;
        ++c->snap_gen;
        if (c->dmiss_on)
        {
            c->dmiss_on = false;
            c->cfk.miss_stale = true;
        }
    }
    if ((rc == AD_E_NOMEM || rc == AD_E_DEVICE) && !o.rolled_back && !o.rederived && !o.batch_stood)
    {
        // the derived arrays may be half built: rebuild them from the entries at the next use
        c->host_stale = true;
        c->dirty = true;
    }
    // a failure after the explicit batch stood is AD_E_PARTIAL: a caller must not take it for "nothing
    // applied" and retry the batch
    if (rc && o.batch_stood) return c->fail(AD_E_PARTIAL, "explicit updates applied, deps-derived part failed: %s", e.c_str());
    if (rc) return c->fail(rc, "%s", e.c_str());
    if (u.n)
    {
        c->host_stale = true;
        ++c->snap_gen;            // device views built from the host state (recovery) are stale
    }
    if (n_applied) *n_applied = o.n_applied;
    if (stats)
    {
        *stats = ad_stats{};
        stats->n_txns = u.n;
        stats->ms_device = o.ms_total;
        stats->ms_stage[0] = o.ms_locate;
        stats->ms_stage[1] = o.ms_derive;
        stats->n_keys[0] = o.n_inserted;         // entries inserted
        stats->n_keys[1] = o.n_new_ids;          // ids appended to the dictionary
        stats->n_keys[2] = o.n_additions;        // TRANSITIVELY_KNOWN entries from deps
    }
    return AD_OK;
}

// The host-side follow-up of an update batch (run_cfk_update returned rc): the LoadPruned hand-back, the
// KeyLine hash of new keys, the host dictionary after a merge or an append, the sampled dictionary index and
// the KeyLines. Nonzero: a device failure (the message is set).
static int cfk_update_follow(ad_ctx* c, const CfkUpdOut& o, int rc, hipStream_t st)
{
    const uint64_t nd0 = c->dict_msb.size();
    if (rc == AD_OK && o.n_load_pruned)
    {
        const uint64_t m = o.n_load_pruned;
        c->lp_upd.resize(m); c->lp_keys.resize(m); c->lp_msb.resize(m); c->lp_lsb.resize(m); c->lp_node.resize(m);
        HIPCHK(c, copy_sync(c->lp_upd.data(), o.lp_update, 8 * m, hipMemcpyDeviceToHost));
        HIPCHK(c, copy_sync(c->lp_keys.data(), o.lp_keys, 8 * m, hipMemcpyDeviceToHost));
        HIPCHK(c, copy_sync(c->lp_msb.data(), o.lp_msb, 8 * m, hipMemcpyDeviceToHost));
        HIPCHK(c, copy_sync(c->lp_lsb.data(), o.lp_lsb, 8 * m, hipMemcpyDeviceToHost));
        HIPCHK(c, copy_sync(c->lp_node.data(), o.lp_node, 4 * m, hipMemcpyDeviceToHost));
    }
    if (o.n_new_keys)
    {
        // keys created on the device (they stay when the batch then failed): KeyLines, host copies
        if (int rc2 = cfk_after_new_keys(c, o, st)) return rc2;
        c->host_moved = true;
        c->host_ingested = false;     // entries moved after the ingest
        c->host_stale = true;
        ++c->snap_gen;
    }
    if (o.merged)
    {
        // ids merged into the device dictionary (they stay when the batch then failed): host copies
        if (int rc2 = cfk_after_merge(c, o.merge_pos, o.n_new_ids, st)) return rc2;
        drop_global_dict(c);
        c->host_moved = true;        // entry ranks changed: host copies rebuilt from the device
        c->host_ingested = false;     // entries moved after the ingest
        c->host_stale = true;
        ++c->snap_gen;
    }
    if (c->ds.n_dict > nd0)
    {
        // ids appended to the device dictionary (kept even when the batch then failed): host copy
        const uint64_t add = c->ds.n_dict - nd0;
        c->dict_msb.resize(nd0 + add);
        c->dict_lsb.resize(nd0 + add);
        c->dict_node.resize(nd0 + add);
        HIPCHK(c, copy_sync(c->dict_msb.data() + nd0, c->d_dict_hi.as<uint64_t>() + nd0, 8 * add, hipMemcpyDeviceToHost));
        HIPCHK(c, copy_sync(c->dict_lsb.data() + nd0, c->d_dict_lsb_raw.as<uint64_t>() + nd0, 8 * add, hipMemcpyDeviceToHost));
        HIPCHK(c, copy_sync(c->dict_node.data() + nd0, c->d_dict_node.as<int32_t>() + nd0, 4 * add, hipMemcpyDeviceToHost));
        drop_global_dict(c);         // global ranks of the multi-store exchange no longer cover the dictionary
        // the sampled index over the grown dictionary (a stale one is still correct, only slower)
        // (a buffer that could not grow may have been released: then no sample, the searches span the
        // whole dictionary)
        const uint64_t ns = dict_samples(c->ds.n_dict), ne = dict_sample_entries(c->ds.n_dict);
        const bool ok = c->d_ds_hi.ensure(8 * ne + 8 * ne / 4) && c->d_ds_lo.ensure(8 * ne + 8 * ne / 4) &&
                        c->d_ds_node.ensure(4 * ne + 4 * ne / 4);
        c->ds.ds_hi = c->d_ds_hi.as<uint64_t>();
        c->ds.ds_lo = c->d_ds_lo.as<uint64_t>();
        c->ds.ds_node = c->d_ds_node.as<int32_t>();
        c->ds.n_samp = ok ? ns : 0;
        c->ds.n_samp2 = ok ? dict_samples2(c->ds.n_dict) : 0;
        if (ok) HIPCHK(c, run_dict_sample(c->ds, c->d_ds_hi.as<uint64_t>(), c->d_ds_lo.as<uint64_t>(), c->d_ds_node.as<int32_t>(), st));
    }
    if (o.n_inserted) { c->host_moved = true; c->host_ingested = false; }
    if ((rc == 0 || o.rolled_back || o.rederived || o.batch_stood) && c->kline_slots)
        HIPCHK(c, run_build_klines(c->ds, c->d_kslot.as<uint32_t>(), c->d_kcell.as<uint32_t>(), c->d_kline.as<KeyLine>(),
                                   c->kline_slots, st));
    return 0;
}

static int check_update_soa(ad_ctx* c, const ad_cfk_update_soa* u)
{
    // the status describes this call from here on, whatever rejects it below (ad_cfk_update_status)
    c->upd_applied = false;
    c->upd_failed = -1;
    if (!u) return c->fail(AD_E_INVAL, "null update batch");
    if (u->n && (!u->keys || !u->txn_msb || !u->txn_lsb || !u->txn_node || !u->exec_msb || !u->exec_lsb ||
                 !u->exec_node || !u->status))
        return c->fail(AD_E_INVAL, "update batch with null arrays");
    if (u->dep_off && (!u->dep_msb || !u->dep_lsb || !u->dep_node))
        return c->fail(AD_E_INVAL, "update batch with dep_off but null dep arrays");
    if ((u->ballot_msb != nullptr) != (u->ballot_lsb != nullptr) || (u->ballot_msb != nullptr) != (u->ballot_node != nullptr))
        return c->fail(AD_E_INVAL, "update batch ballots: ballot_msb, ballot_lsb and ballot_node must be all set or all NULL");
    if (!c->cfk.loaded) return c->fail(AD_E_NOT_LOADED, "ad_cfk_load not called");
    if (hipSetDevice(c->device) != hipSuccess) return c->fail(AD_E_DEVICE, "hipSetDevice");
    StreamScope scope_(c->stream, c->cstream);
    return 0;
}

int ad_cfk_update_status(const ad_ctx* c, int* applied, int64_t* failed_update)
{
    if (!c) return AD_E_INVAL;
    if (applied) *applied = c->upd_applied ? 1 : 0;
    if (failed_update) *failed_update = c->upd_failed;
    return AD_OK;
}

int ad_cfk_update_device(ad_ctx* c, const ad_cfk_update_soa* u, void* stream, uint64_t* n_applied, ad_stats* stats)
{
    if (!c) return AD_E_INVAL;
    if (int rc = check_update_soa(c, u)) return rc;
    CfkUpdIn in{u->n, u->keys, u->txn_msb, u->txn_lsb, u->txn_node, u->exec_msb, u->exec_lsb, u->exec_node, u->status,
                u->ballot_msb, u->ballot_lsb, u->ballot_node, u->dep_off, u->dep_msb, u->dep_lsb, u->dep_node};
    return cfk_update_run(c, in, stream ? (hipStream_t)stream : c->stream, n_applied, stats);
}

int ad_cfk_update(ad_ctx* c, const ad_cfk_update_soa* u, uint64_t* n_applied, ad_stats* stats)
{
    if (!c) return AD_E_INVAL;
    if (int rc = check_update_soa(c, u)) return rc;
    const uint64_t n = u->n;
    int rc = 0;
    CfkUpdIn in{n, stage_q(c, c->u_k, u->keys, n, &rc), stage_q(c, c->u_tm, u->txn_msb, n, &rc),
                stage_q(c, c->u_tl, u->txn_lsb, n, &rc), stage_q(c, c->u_tn, u->txn_node, n, &rc),
                stage_q(c, c->u_em, u->exec_msb, n, &rc), stage_q(c, c->u_el, u->exec_lsb, n, &rc),
                stage_q(c, c->u_en, u->exec_node, n, &rc), stage_q(c, c->u_st, u->status, n, &rc), nullptr, nullptr, nullptr,
                nullptr, nullptr, nullptr, nullptr};
    if (u->dep_off)
    {
        const uint64_t nd = u->dep_off[n];
        in.dep_off = stage_q(c, c->u_do, u->dep_off, n + 1, &rc);
        in.dep_msb = stage_q(c, c->u_dm, u->dep_msb, nd, &rc);
        in.dep_lsb = stage_q(c, c->u_dl, u->dep_lsb, nd, &rc);
        in.dep_node = stage_q(c, c->u_dn, u->dep_node, nd, &rc);
    }
    if (u->ballot_msb)
    {
        in.bal_msb = stage_q(c, c->u_bm, u->ballot_msb, n, &rc);
        in.bal_lsb = stage_q(c, c->u_bl, u->ballot_lsb, n, &rc);
        in.bal_node = stage_q(c, c->u_bn, u->ballot_node, n, &rc);
    }
    if (rc) return rc;
    return cfk_update_run(c, in, c->stream, n_applied, stats);
}

int ad_cfk_entries(ad_ctx* c, uint64_t* n_entries, const uint8_t** status, const uint64_t** exec_msb,
                   const uint64_t** exec_lsb, const int32_t** exec_node)
{
    if (!c || !n_entries || !status || !exec_msb || !exec_lsb || !exec_node) return AD_E_INVAL;
    if (!c->cfk.loaded) return c->fail(AD_E_NOT_LOADED, "ad_cfk_load not called");
    if (hipSetDevice(c->device) != hipSuccess) return c->fail(AD_E_DEVICE, "hipSetDevice");
    StreamScope scope_(c->stream, c->cstream);
    if (int rc = sync_host(c)) return rc;
    auto& K = c->cfk;
    const uint64_t ne = K.status.size();
    c->x_msb.resize(ne);
    c->x_lsb.resize(ne);
    c->x_node.resize(ne);
    for (uint64_t e = 0; e < ne; ++e)
    {
        c->x_msb[e] = K.exec[e].msb;
        c->x_lsb[e] = K.exec[e].lsb;
        c->x_node[e] = K.exec[e].node;
    }
    *n_entries = ne;
    *status = K.status.data();
    *exec_msb = c->x_msb.data();
    *exec_lsb = c->x_lsb.data();
    *exec_node = c->x_node.data();
    return AD_OK;
}

int ad_cfk_load_pruned(ad_ctx* c, uint64_t* n, const uint64_t** update, const int64_t** keys, const uint64_t** msb,
                       const uint64_t** lsb, const int32_t** node)
{
    if (!c || !n || !update || !keys || !msb || !lsb || !node) return AD_E_INVAL;
    *n = c->lp_upd.size();
    *update = c->lp_upd.data();
    *keys = c->lp_keys.data();
    *msb = c->lp_msb.data();
    *lsb = c->lp_lsb.data();
    *node = c->lp_node.data();
    return AD_OK;
}

int ad_cfk_ballots_load(ad_ctx* c, uint64_t n_entries, const uint64_t* msb, const uint64_t* lsb, const int32_t* node)
{
    if (!c || (n_entries && (!msb || !lsb || !node))) return AD_E_INVAL;
    if (!c->cfk.loaded) return c->fail(AD_E_NOT_LOADED, "ad_cfk_load not called");
    if (hipSetDevice(c->device) != hipSuccess) return c->fail(AD_E_DEVICE, "hipSetDevice");
    StreamScope scope_(c->stream, c->cstream);
    if (int rc = sync_host(c)) return rc;
    auto& K = c->cfk;
    if (n_entries != K.status.size()) return c->fail(AD_E_INVAL, "%llu ballots for %zu entries", (unsigned long long)n_entries, K.status.size());
    K.ballot.resize(n_entries);
    std::vector<Bal> bl(n_entries);
    for (uint64_t e = 0; e < n_entries; ++e)
    {
        K.ballot[e] = Tid{msb[e], lsb[e], node[e]};
        bl[e] = Bal{msb[e], lsb[e], node[e], 0};
    }
    if (!c->dirty)
    {
        if (int rc = upload(c, c->d_ballot, bl)) return rc;
        HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    return AD_OK;
}

int ad_cfk_ballots(ad_ctx* c, uint64_t* n_entries, const uint64_t** msb, const uint64_t** lsb, const int32_t** node)
{
    if (!c || !n_entries || !msb || !lsb || !node) return AD_E_INVAL;
    if (!c->cfk.loaded) return c->fail(AD_E_NOT_LOADED, "ad_cfk_load not called");
    if (hipSetDevice(c->device) != hipSuccess) return c->fail(AD_E_DEVICE, "hipSetDevice");
    StreamScope scope_(c->stream, c->cstream);
    if (int rc = sync_host(c)) return rc;
    auto& K = c->cfk;
    const uint64_t ne = K.status.size();
    c->x_msb.assign(ne, 0);
    c->x_lsb.assign(ne, 0);
    c->x_node.assign(ne, 0);
    for (uint64_t e = 0; e < ne && !K.ballot.empty(); ++e)
    {
        c->x_msb[e] = K.ballot[e].msb;
        c->x_lsb[e] = K.ballot[e].lsb;
        c->x_node[e] = K.ballot[e].node;
    }
    *n_entries = ne;
    *msb = c->x_msb.data();
    *lsb = c->x_lsb.data();
    *node = c->x_node.data();
    return AD_OK;
}

}  // extern "C"

// =======================================================================================
// Node exchange (SURVEY §8 e): the per-store PartialDeps of a node batch combined
// on the store that owns each request -- CommandStores.mapReduce's reduce (CommandStores.java:576-593)
// with PartialDeps.with (PreAccept.reduce, PreAccept.java:140-156) -- as export -> move -> K3 merge.
// Two transports of one protocol: device copies between the contexts of one process
// (ad_exchange_local: the Java host's one process per node, hipMemcpyPeerAsync over xGMI between
// GPUs) and RCCL grouped send/recv between processes (ad_exchange).
// =======================================================================================
namespace {

constexpr int XA = 4;                                  // hdr, keys, ids, k2t
static size_t x_unit_bytes(int a, uint32_t fmt)       // bytes per counted unit of array a
{
    switch (a)
    {
        case 0: return 32;                             // 4 int64 per part
        case 1: return 8;                              // key words
        case 2: return fmt == AD_IDS_RANK ? 4 : 24;    // ids
        default: return 4;                             // k2t
    }
}
static DevBuf* x_send(ad_ctx* c, int a) { DevBuf* b[XA] = {&c->xs_hdr, &c->xs_keys, &c->xs_ids, &c->xs_k2t}; return b[a]; }
static DevBuf* x_recv(ad_ctx* c, int a) { DevBuf* b[XA] = {&c->xr_hdr, &c->xr_keys, &c->xr_ids, &c->xr_k2t}; return b[a]; }
static uint32_t x_format(const ad_ctx* c) { return c->global_ok ? AD_IDS_RANK : AD_IDS_TRIPLET; }

// The plan of `R` from an agreed exchange table (layout: accord_deps.h, ad_exchange_plan). Every rank
// runs it on the same table, so every verdict -- failure, id formats, growth round -- is collective.
// bad: the rank whose row failed a check (-1: none).
static int x_plan(const uint64_t* table, uint32_t W, uint32_t R, ad_xfer* xf, uint64_t* recv_units, uint64_t* src_parts,
                  uint32_t* flags, int* bad)
{
    const size_t RW = AD_XROW_WORDS(W);
    auto row = [&](uint32_t s) { return table + RW * s; };
    *bad = -1;
    for (uint32_t s = 0; s < W; ++s)
        if (row(s)[4 * W] != AD_XROW_MAGIC || row(s)[4 * W + 3] != 0) { *bad = (int)s; return AD_E_INVAL; }
    for (uint32_t s = 0; s < W; ++s)
        if (row(s)[4 * W + 2] != 0) { *bad = (int)s; return AD_E_PEER; }
    const uint64_t fmt = row(0)[4 * W + 1];
    if (fmt != AD_IDS_RANK && fmt != AD_IDS_TRIPLET) { *bad = 0; return AD_E_INVAL; }
    for (uint32_t s = 1; s < W; ++s)
        if (row(s)[4 * W + 1] != fmt) { *bad = (int)s; return AD_E_STATE; }
    uint32_t fl = 0;
    for (int a = 0; a < XA; ++a)
    {
        const uint64_t ub = x_unit_bytes(a, (uint32_t)fmt);
        uint64_t soff = 0, roff = 0;
        for (uint32_t p = 0; p < W; ++p)
        {
            const uint64_t sc = row(R)[4 * p + a], rc = row(p)[4 * R + a];
            xf[(size_t)a * W + p] = ad_xfer{ub * soff, ub * sc, ub * roff, ub * rc};
            soff += sc;      // R's parts for p follow those for the lower ranks (grouped by owner)
            roff += rc;      // p's parts for R follow the lower ranks' (source = slice order for K3)
        }
        recv_units[a] = roff;
        // every rank's totals against the capacities it published
        for (uint32_t s = 0; s < W; ++s)
        {
            uint64_t snd = 0, rcv = 0;
            for (uint32_t p = 0; p < W; ++p)
            {
                snd += row(s)[4 * p + a];
                rcv += row(p)[4 * s + a];
            }
            if (snd > row(s)[4 * W + 4 + a] || rcv > row(s)[4 * W + 8 + a]) fl |= AD_XPLAN_GROW;
        }
    }
    for (uint32_t p = 0; p < W; ++p) src_parts[p] = row(p)[4 * R + 0];
    *flags = fl;
    return AD_OK;
}

// header words of c's row: format, status (-code of a failure before the move), buffer capacities in units
static XRowHdr x_row_hdr(ad_ctx* c, uint32_t fmt, int status)
{
    XRowHdr h{};
    h.w[0] = AD_XROW_MAGIC;
    h.w[1] = fmt;
    h.w[2] = status ? (uint64_t)(-(int64_t)status) : 0;
    h.w[3] = 0;
    for (int a = 0; a < XA; ++a)
    {
        h.w[4 + a] = x_send(c, a)->cap / x_unit_bytes(a, fmt);
        h.w[8 + a] = x_recv(c, a)->cap / x_unit_bytes(a, fmt);
    }
    return h;
}

// send / receive buffers of c for the units of a step (25 % headroom when they grow)
static int x_grow(ad_ctx* c, const uint64_t* send_units, const uint64_t* recv_units, uint32_t fmt)
{
    for (int a = 0; a < XA; ++a)
    {
        const uint64_t ub = x_unit_bytes(a, fmt);
        if (ub * send_units[a] > x_send(c, a)->cap && !x_send(c, a)->ensure(ub * (send_units[a] + send_units[a] / 4 + 64)))
            return c->fail(AD_E_NOMEM, "exchange send buffers");
        if (ub * recv_units[a] > x_recv(c, a)->cap && !x_recv(c, a)->ensure(ub * (recv_units[a] + recv_units[a] / 4 + 64)))
            return c->fail(AD_E_NOMEM, "exchange receive buffers");
    }
    return AD_OK;
}

// the parts of requests [lo, hi) stay on this store (it owns them): written by the export straight to
// their place in its receive arrays (plan entry `self` of each array), not copied there afterwards
static void x_keep_self(ad_ctx* c, ExportArgs& a, const ad_xfer* xf, uint32_t W, uint32_t self, uint64_t lo, uint64_t hi,
                        uint32_t fmt)
{
    a.self_lo = lo;
    a.self_hi = hi;
    for (int k = 0; k < XA; ++k)
    {
        const ad_xfer& x = xf[(size_t)k * W + self];
        const int64_t ub = (int64_t)x_unit_bytes(k, fmt);
        a.self_delta[k] = ((int64_t)x.recv_off - (int64_t)x.send_off) / ub;
    }
    a.rhdr = c->xr_hdr.as<int64_t>();
    a.rkeys = c->xr_keys.as<int64_t>();
    a.rids = c->xr_ids.as<int64_t>();
    a.rk2t = c->xr_k2t.as<int32_t>();
}

static int x_emit(ad_ctx* c, ExportArgs& a, hipStream_t st)
{
    return export_emit(c, a, c->xs_hdr.as<int64_t>(), c->xs_keys.as<int64_t>(), c->xs_ids.as<int64_t>(),
                       c->xs_k2t.as<int32_t>(), st);
}

// K3 on c over its receive buffers: sources in slice (= rank / context) order
static int x_merge(ad_ctx* c, uint32_t n_src, const uint64_t* src_parts, const uint64_t* recv_units, uint32_t fmt,
                   uint64_t txn_base, uint64_t n_owned, hipStream_t st, ad_merged* out, MergeTail* defer = nullptr)
{
    ad_parts in{};
    in.hdr = c->xr_hdr.as<int64_t>();
    in.keys = c->xr_keys.as<int64_t>();
    in.ids = c->xr_ids.as<int64_t>();
    in.k2t = c->xr_k2t.as<int32_t>();
    in.n_parts = recv_units[0];
    in.n_key_words = recv_units[1];
    in.n_ids = recv_units[2];
    in.n_k2t = recv_units[3];
    in.id_format = fmt;
    for (int a = 0; a < XA; ++a) c->xr_total[a] = recv_units[a];
    return parts_merge(c, &in, n_src, src_parts, txn_base, n_owned, st, out, false, defer);
}

// an error after the table was agreed: the peers are (or will be) inside the grouped send/recv, so the
// communicator is torn down -- this rank returns at once and its process exits instead of waiting
static int x_abort(ad_ctx* c, int code)
{
    if (c->comm) (void)ncclCommAbort(c->comm);
    c->comm = nullptr;
    return code;
}

static int nccl_fail(ad_ctx* c, ncclResult_t r, const char* what)
{
    return c->fail(AD_E_DEVICE, "%s: %s", what, ncclGetErrorString(r));
}
#define NCCLCHK(ctx, expr)                                                                         \
    do {                                                                                           \
        ncclResult_t _r = (expr);                                                                  \
        if (_r != ncclSuccess) return nccl_fail((ctx), _r, #expr);                                 \
    } while (0)

static float ev_ms(hipEvent_t a, hipEvent_t b)
{
    float ms = 0;
    return hipEventElapsedTime(&ms, a, b) == hipSuccess ? ms : 0.f;
}

}  // namespace

extern "C" {

int ad_exchange_plan(const uint64_t* table, uint32_t world, uint32_t rank, ad_xfer* xfers, uint64_t* recv_units,
                     uint64_t* src_parts, uint32_t* flags)
{
    if (!table || world == 0 || rank >= world || !xfers || !recv_units || !src_parts || !flags) return AD_E_INVAL;
    int bad = -1;
    return x_plan(table, world, rank, xfers, recv_units, src_parts, flags, &bad);
}

static int exchange_local_run(ad_ctx* const* ctxs, uint32_t n, const ad_deps_result* const* res, const int64_t* const* txn_index,
                              const uint64_t* const* dest_first, const uint64_t* txn_base, const uint64_t* n_owned,
                              ad_merged* out, ad_exchange_stats* stats);

int ad_exchange_local(ad_ctx* const* ctxs, uint32_t n, const ad_deps_result* const* res, const int64_t* const* txn_index,
                      const uint64_t* const* dest_first, const uint64_t* txn_base, const uint64_t* n_owned,
                      ad_merged* out, ad_exchange_stats* stats)
{
    if (!ctxs || n == 0 || !res || !txn_index || !dest_first || !txn_base || !n_owned || !out) return AD_E_INVAL;
    for (uint32_t i = 0; i < n; ++i)
        if (!ctxs[i] || !res[i]) return AD_E_INVAL;
    const int rc = exchange_local_run(ctxs, n, res, txn_index, dest_first, txn_base, n_owned, out, stats);
    if (rc)
    {
        // whatever an earlier store or owner had queued (exports, copies, merges, pinned read-backs) completes
        // before the call returns, and no owner's result looks valid
        for (uint32_t i = 0; i < n; ++i)
            if (hipSetDevice(ctxs[i]->device) == hipSuccess) (void)hipStreamSynchronize(ctxs[i]->stream);
        for (uint32_t i = 0; i < n; ++i) out[i] = ad_merged{};
    }
    return rc;
}

static int exchange_local_run(ad_ctx* const* ctxs, uint32_t n, const ad_deps_result* const* res, const int64_t* const* txn_index,
                              const uint64_t* const* dest_first, const uint64_t* txn_base, const uint64_t* n_owned,
                              ad_merged* out, ad_exchange_stats* stats)
{
    const uint32_t fmt = x_format(ctxs[0]);
    for (uint32_t i = 1; i < n; ++i)
        if (x_format(ctxs[i]) != fmt)
            return ctxs[i]->fail(AD_E_STATE, "ad_exchange_local: every store needs the same id format (global dictionary on all or none)");
    const size_t RW = AD_XROW_WORDS(n);
    const double t0 = now_ms();
    // 1. every store's export sizes; the bounds read back
    std::vector<ExportArgs> ea(n);
    std::vector<std::vector<uint64_t>> cum(n, std::vector<uint64_t>(4 * (size_t)(n + 1)));
    for (uint32_t i = 0; i < n; ++i)
    {
        ad_ctx* c = ctxs[i];
        if (hipSetDevice(c->device) != hipSuccess) return c->fail(AD_E_DEVICE, "hipSetDevice");
        if (int rc = export_sizes(c, res[i], txn_index[i], n, dest_first[i], fmt, c->stream, &ea[i])) return rc;
        // into the store's pinned read-back words: the stores' size passes overlap, read after the sync below
        uint64_t* rb = cum[i].size() <= UP_WORDS ? rb_slot(c) : nullptr;
        if (rb) HIPCHK(c, hipMemcpyAsync(rb, c->x_cnt.p, sizeof(uint64_t) * cum[i].size(), hipMemcpyDeviceToHost, c->stream));
        else HIPCHK(c, d2h(cum[i].data(), c->x_cnt.p, sizeof(uint64_t) * cum[i].size(), c->stream));
    }
    // 2. the exchange table, as the RCCL path gathers it
    std::vector<uint64_t> table(RW * n, 0);
    for (uint32_t s = 0; s < n; ++s)
    {
        ad_ctx* c = ctxs[s];
        if (hipSetDevice(c->device) != hipSuccess) return c->fail(AD_E_DEVICE, "hipSetDevice");
        HIPCHK(c, hipStreamSynchronize(c->stream));
        if (cum[s].size() <= UP_WORDS && c->h_rb) memcpy(cum[s].data(), c->h_rb, sizeof(uint64_t) * cum[s].size());
        uint64_t* row = table.data() + RW * s;
        for (size_t i = 0; i < 4 * (size_t)n; ++i) row[i] = cum[s][i + 4] - cum[s][i];
        const XRowHdr h = x_row_hdr(c, fmt, 0);
        for (uint32_t k = 0; k < AD_XROW_HDR; ++k) row[4 * n + k] = h.w[k];
    }
    std::vector<std::vector<ad_xfer>> xf(n, std::vector<ad_xfer>(4 * (size_t)n));
    std::vector<std::vector<uint64_t>> src_parts(n, std::vector<uint64_t>(n));
    std::vector<std::array<uint64_t, 4>> runits(n);
    // 3. plan, buffers and the parts of every store
    for (uint32_t s = 0; s < n; ++s)
    {
        ad_ctx* c = ctxs[s];
        uint32_t fl = 0;
        int bad = -1;
        if (int rc = x_plan(table.data(), n, s, xf[s].data(), runits[s].data(), src_parts[s].data(), &fl, &bad))
            return c->fail(rc, "ad_exchange_local: exchange table rejected (store %d)", bad);
        uint64_t send_units[XA] = {0, 0, 0, 0};
        for (uint32_t d = 0; d < n; ++d)
            for (int a = 0; a < XA; ++a) send_units[a] += table[RW * s + 4 * d + a];
        if (hipSetDevice(c->device) != hipSuccess) return c->fail(AD_E_DEVICE, "hipSetDevice");
        if (int rc = x_grow(c, send_units, runits[s].data(), fmt)) return rc;
        x_keep_self(c, ea[s], xf[s].data(), n, s, dest_first[s][s], dest_first[s][s + 1], fmt);
        if (int rc = x_emit(c, ea[s], c->stream)) return rc;
    }
    for (uint32_t s = 0; s < n; ++s)
    {
        if (hipSetDevice(ctxs[s]->device) != hipSuccess) return ctxs[s]->fail(AD_E_DEVICE, "hipSetDevice");
        HIPCHK(ctxs[s], hipStreamSynchronize(ctxs[s]->stream));
    }
    const double t1 = now_ms();
    uint64_t moved = 0;
    // 4. each owner gathers what every store exported for it (slice order), device to device
    for (uint32_t d = 0; d < n; ++d)
    {
        ad_ctx* o = ctxs[d];
        if (hipSetDevice(o->device) != hipSuccess) return o->fail(AD_E_DEVICE, "hipSetDevice");
        for (uint32_t s = 0; s < n; ++s)
        {
            ad_ctx* c = ctxs[s];
            for (int a = 0; a < XA; ++a)
            {
                const ad_xfer& from = xf[s][(size_t)a * n + d];
                const ad_xfer& to = xf[d][(size_t)a * n + s];
                if (from.send_bytes != to.recv_bytes) return o->fail(AD_E_STATE, "ad_exchange_local: plans disagree");
                if (!from.send_bytes || s == d) continue;          // own parts: written in place by the export
                char* dst = x_recv(o, a)->as<char>() + to.recv_off;
                const char* src = x_send(c, a)->as<char>() + from.send_off;
                if (c->device == o->device)
                    HIPCHK(o, hipMemcpyAsync(dst, src, from.send_bytes, hipMemcpyDeviceToDevice, o->stream));
                else
                    HIPCHK(o, hipMemcpyPeerAsync(dst, o->device, src, c->device, from.send_bytes, o->stream));
                if (s != d) moved += from.send_bytes;
            }
        }
    }
    const double t2 = now_ms();
    // 5. K3 on every owner. Owners on distinct GPUs: all queued, then each finished (the GPUs merge at once);
    //    owners sharing a GPU merge one after the other (each merge's device time is then its own)
    bool distinct = true;
    for (uint32_t d = 0; d < n && distinct; ++d)
        for (uint32_t e = 0; e < d && distinct; ++e) distinct = ctxs[d]->device != ctxs[e]->device;
    double ms_merge = 0;
    std::vector<MergeTail> tails(n);
    for (uint32_t d = 0; d < n; ++d)
    {
        ad_ctx* o = ctxs[d];
        if (hipSetDevice(o->device) != hipSuccess) return o->fail(AD_E_DEVICE, "hipSetDevice");
        if (int rc = x_merge(o, n, src_parts[d].data(), runits[d].data(), fmt, txn_base[d], n_owned[d], o->stream, &out[d],
                             &tails[d]))
            return rc;
        if (!distinct)
        {
            if (int rc = merge_tail(o, tails[d], &out[d])) return rc;
            ms_merge += out[d].ms_device;
        }
    }
    for (uint32_t d = 0; d < n && distinct; ++d)
    {
        if (int rc = merge_tail(ctxs[d], tails[d], &out[d])) return rc;
        ms_merge += out[d].ms_device;
    }
    if (stats)
    {
        memset(stats, 0, sizeof(*stats));
        stats->bytes_moved = moved;
        stats->ms_export = t1 - t0;
        stats->ms_move = t2 - t1;
        stats->ms_merge = ms_merge;
        stats->ms_total = now_ms() - t0;
    }
    return AD_OK;
}

int ad_comm_unique_id(uint8_t* id)
{
    if (!id) return AD_E_INVAL;
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return AD_E_DEVICE;
    memcpy(id, u.internal, AD_COMM_ID_BYTES);
    return AD_OK;
}

int ad_comm_init(ad_ctx* c, const uint8_t* id, int rank, int world)
{
    if (!c || !id || world <= 0 || rank < 0 || rank >= world) return AD_E_INVAL;
    if (hipSetDevice(c->device) != hipSuccess) return c->fail(AD_E_DEVICE, "hipSetDevice");
    StreamScope scope_(c->stream, c->cstream);
    if (c->comm) { (void)ncclCommDestroy(c->comm); c->comm = nullptr; }
    // the exchange table lives as long as the communicator: a step never allocates before the collective
    const size_t RW = AD_XROW_WORDS(world), words = RW * (size_t)(world + 1) + 2 * (size_t)world + 2;
    if (!c->xc_dev.ensure(sizeof(uint64_t) * words)) return c->fail(AD_E_NOMEM, "exchange table");
    if (c->h_xtab_words < words)
    {
        if (c->h_xtab) (void)hipHostFree(c->h_xtab);
        c->h_xtab = nullptr;
        c->h_xtab_words = 0;
        HIPCHK(c, hipHostMalloc((void**)&c->h_xtab, sizeof(uint64_t) * words, hipHostMallocDefault));
        c->h_xtab_words = words;
    }
    for (hipEvent_t& e : c->x_ev)
        if (!e) HIPCHK(c, timing_event(&e));
    ncclUniqueId u;
    memcpy(u.internal, id, AD_COMM_ID_BYTES);
    NCCLCHK(c, ncclCommInitRank(&c->comm, world, u, rank));
    c->comm_rank = rank;
    c->comm_world = world;
    return AD_OK;
}

int ad_exchange(ad_ctx* c, const ad_deps_result* res, const int64_t* txn_index, const uint64_t* dest_first, uint64_t txn_base,
                uint64_t n_owned, void* stream, ad_merged* out, ad_exchange_stats* stats)
{
    if (!c) return AD_E_INVAL;
    if (!c->comm) return c->fail(AD_E_STATE, "ad_exchange: no communicator (ad_comm_init)");
    if (hipSetDevice(c->device) != hipSuccess) return c->fail(AD_E_DEVICE, "hipSetDevice");
    StreamScope scope_(c->stream, c->cstream);
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    scope_.add(st);
    const uint32_t W = (uint32_t)c->comm_world, R = (uint32_t)c->comm_rank;
    const uint32_t fmt = x_format(c);
    const size_t RW = AD_XROW_WORDS(W);
    uint64_t* tab = c->xc_dev.as<uint64_t>();          // [W][RW] gathered rows
    uint64_t* mine = tab + RW * W;                      // this rank's row
    uint64_t* sw = mine + RW;                           // growth round: own status word, then W gathered
    uint64_t* h = c->h_xtab;
    const double t0 = now_ms();
    HIPCHK(c, hipEventRecord(c->x_ev[0], st));
    // 1. export sizes -> this rank's row of the table, on the device. A failure here is published in
    //    the row (status), so the peers learn of it from the all-gather instead of waiting for parts.
    ExportArgs ea{};
    int own = !res || !out || !dest_first ? c->fail(AD_E_INVAL, "ad_exchange: res, dest_first and out are required")
                                          : export_sizes(c, res, txn_index, W, dest_first, fmt, st, &ea);
    if (own == AD_OK && run_x_row(c->x_cnt.as<uint64_t>(), W, x_row_hdr(c, fmt, 0), mine, st) != hipSuccess)
        own = c->fail(AD_E_DEVICE, "exchange table row");
    if (own != AD_OK)
    {
        const std::string why = c->err;
        const XRowHdr hd = x_row_hdr(c, fmt, own);
        memset(h, 0, sizeof(uint64_t) * RW);
        memcpy(h + 4 * W, hd.w, sizeof(hd.w));
        if (copy_sync(mine, h, sizeof(uint64_t) * RW, hipMemcpyHostToDevice) != hipSuccess)
            return x_abort(c, own);
        c->err = why;
    }
    // 2. the table: one all-gather of the rows, read back -- the step's planning synchronisation
    ncclResult_t nr = ncclAllGather(mine, tab, RW, ncclUint64, c->comm, st);
    if (nr != ncclSuccess) return x_abort(c, own ? own : nccl_fail(c, nr, "ncclAllGather (exchange table)"));
    HIPCHK(c, d2h(h, tab, sizeof(uint64_t) * RW * W, st));
    HIPCHK(c, hipStreamSynchronize(st));
    // 3. the plan, identical on every rank: a failed or inconsistent rank fails every rank here
    std::vector<ad_xfer> xf(4 * (size_t)W);
    std::vector<uint64_t> src_parts(W);
    uint64_t runits[XA];
    uint32_t flags = 0;
    int bad = -1;
    if (int rc = x_plan(h, W, R, xf.data(), runits, src_parts.data(), &flags, &bad))
    {
        if (own) return own;
        if (rc == AD_E_PEER)
            return c->fail(AD_E_PEER, "ad_exchange: rank %d failed before the move (code -%llu)", bad,
                           (unsigned long long)h[RW * bad + 4 * W + 2]);
        if (rc == AD_E_STATE)
            return c->fail(AD_E_STATE, "ad_exchange: ranks use different id formats (rank %d: %s, rank 0: %s; the global "
                                       "dictionary must be installed on all or none)", bad,
                           h[RW * bad + 4 * W + 1] == AD_IDS_RANK ? "ranks" : "triplets",
                           h[4 * W + 1] == AD_IDS_RANK ? "ranks" : "triplets");
        return c->fail(rc, "ad_exchange: malformed exchange table (row of rank %d)", bad);
    }
    uint64_t send_units[XA] = {0, 0, 0, 0};
    for (uint32_t d = 0; d < W; ++d)
        for (int a = 0; a < XA; ++a) send_units[a] += h[RW * R + 4 * d + a];
    // 4. growth round, taken by every rank when any rank's buffers are short: each grows its own, then a
    //    one-word status all-gather tells all of them whether every rank can go on
    if (flags & AD_XPLAN_GROW)
    {
        const int g = x_grow(c, send_units, runits, fmt);
        uint64_t* hs = h + RW * W;
        hs[0] = g ? (uint64_t)(-(int64_t)g) : 0;
        // (hs is pinned: an ordered async copy, read by the all-gather behind it; no host round trip)
        if (h2d(sw, hs, sizeof(uint64_t), st) != hipSuccess) return x_abort(c, AD_E_DEVICE);
        nr = ncclAllGather(sw, sw + 1, 1, ncclUint64, c->comm, st);
        if (nr != ncclSuccess) return x_abort(c, nccl_fail(c, nr, "ncclAllGather (exchange status)"));
        HIPCHK(c, d2h(hs + 1, sw + 1, sizeof(uint64_t) * W, st));
        HIPCHK(c, hipStreamSynchronize(st));
        if (g) return g;
        for (uint32_t s = 0; s < W; ++s)
            if (hs[1 + s]) return c->fail(AD_E_PEER, "ad_exchange: rank %u could not grow its exchange buffers", s);
    }
    // 5. this rank's parts, grouped by owner, into its send buffers (its own: into its receive buffers)
    x_keep_self(c, ea, xf.data(), W, R, dest_first[R], dest_first[R + 1], fmt);
    int erc = x_emit(c, ea, st);
    if (!erc && hipEventRecord(c->x_ev[1], st) != hipSuccess) erc = c->fail(AD_E_DEVICE, "hipEventRecord");
    // 5b. one-word status all-gather: a rank whose emit failed tells every peer before anyone posts a
    //     send or receive, so the verdict stays collective (no rank waits inside the group for parts
    //     that never come); a single rank has no peer to tell
    if (W == 1 && erc) return erc;
    if (W > 1)
    {
        uint64_t* hs = h + RW * W;
        hs[0] = erc ? (uint64_t)(-(int64_t)erc) : 0;
        if (h2d(sw, hs, sizeof(uint64_t), st) != hipSuccess) return x_abort(c, AD_E_DEVICE);
        nr = ncclAllGather(sw, sw + 1, 1, ncclUint64, c->comm, st);
        if (nr != ncclSuccess) return x_abort(c, nccl_fail(c, nr, "ncclAllGather (emit status)"));
        HIPCHK(c, d2h(hs + 1, sw + 1, sizeof(uint64_t) * W, st));
        HIPCHK(c, hipStreamSynchronize(st));
        if (erc) return erc;
        for (uint32_t q = 0; q < W; ++q)
            if (hs[1 + q]) return c->fail(AD_E_PEER, "ad_exchange: rank %u failed to emit its parts", q);
    }
    // 6. grouped send/recv of the four arrays (own parts are in place already). The group is always
    //    closed; a failure inside it aborts the communicator.
    uint64_t moved = 0;
    nr = ncclGroupStart();
    if (nr != ncclSuccess) return x_abort(c, nccl_fail(c, nr, "ncclGroupStart"));
    for (int a = 0; a < XA && nr == ncclSuccess; ++a)
        for (uint32_t p = 0; p < W && nr == ncclSuccess; ++p)
        {
            if (p == R) continue;
            const ad_xfer& x = xf[(size_t)a * W + p];
            // bytes as uint8 (every array is a whole number of bytes; no reduction)
            if (x.send_bytes) nr = ncclSend(x_send(c, a)->as<char>() + x.send_off, x.send_bytes, ncclUint8, (int)p, c->comm, st);
            if (nr == ncclSuccess && x.recv_bytes)
                nr = ncclRecv(x_recv(c, a)->as<char>() + x.recv_off, x.recv_bytes, ncclUint8, (int)p, c->comm, st);
            moved += x.send_bytes;
        }
    const ncclResult_t ne = ncclGroupEnd();
    if (nr != ncclSuccess) return x_abort(c, nccl_fail(c, nr, "ncclSend/ncclRecv"));
    if (ne != ncclSuccess) return x_abort(c, nccl_fail(c, ne, "ncclGroupEnd"));
    if (hipEventRecord(c->x_ev[2], st) != hipSuccess) return x_abort(c, c->fail(AD_E_DEVICE, "hipEventRecord"));
    // 7. K3 over the parts of every source (rank = slice order); its completion is the step's second
    //    (and last) synchronisation
    if (int rc = x_merge(c, W, src_parts.data(), runits, fmt, txn_base, n_owned, st, out)) return rc;
    if (stats)
    {
        memset(stats, 0, sizeof(*stats));
        stats->bytes_moved = moved;
        stats->ms_export = ev_ms(c->x_ev[0], c->x_ev[1]);     // sizes, table, plan, parts
        stats->ms_move = ev_ms(c->x_ev[1], c->x_ev[2]);
        stats->ms_merge = out->ms_device;
        stats->ms_total = now_ms() - t0;
    }
    return AD_OK;
}

// ---- Pruning.maybePrune on the device (cfk_update.hip run_cfk_prune) -----------
int ad_cfk_prune(ad_ctx* c, const int64_t* keys, uint64_t n_keys, int32_t prune_interval, int64_t min_hlc_delta,
                 uint64_t* n_removed, ad_stats* stats)
{
    if (!c) return AD_E_INVAL;
    if (n_keys && !keys) return c->fail(AD_E_INVAL, "ad_cfk_prune: null key list");
    if (!c->cfk.loaded) return c->fail(AD_E_NOT_LOADED, "ad_cfk_load not called");
    if (hipSetDevice(c->device) != hipSuccess) return c->fail(AD_E_DEVICE, "hipSetDevice");
    StreamScope scope_(c->stream, c->cstream);
    if (c->dirty)
        if (int rc = build_snapshot(c)) return rc;
    if (int rc = sync_host(c)) return rc;
    auto& K = c->cfk;
    // loaded missing() lists go to the device, where pruneBefore's subset test (Pruning.java:239-251) reads them
    if (!c->dmiss_on && !K.miss.empty())
    {
        const int rc = dmiss_enable(c, c->stream);
        if (rc < 0) return rc;
        if (rc) return c->fail(AD_E_STATE, "ad_cfk_prune: the missing() lists are stale (load them again)");
    }
    const uint64_t nk = c->ds.n_keys;
    // key ordinals -> key indices of the store (keys without a CommandsForKey are skipped)
    std::vector<uint32_t> kl;
    if (keys)
    {
        kl.reserve(n_keys);
        for (uint64_t i = 0; i < n_keys; ++i)
        {
            const auto it = std::lower_bound(K.keys.begin(), K.keys.end(), keys[i]);
            if (it != K.keys.end() && *it == keys[i]) kl.push_back((uint32_t)(it - K.keys.begin()));
        }
        std::sort(kl.begin(), kl.end());
        kl.erase(std::unique(kl.begin(), kl.end()), kl.end());
        if (kl.empty())
        {
            if (n_removed) *n_removed = 0;
            if (stats) *stats = ad_stats{};
            return AD_OK;
        }
        if (int rc = upload(c, c->d_prune_keys, kl)) return rc;
    }
    if (!c->cu) c->cu = cfk_upd_work_create();
    CfkDevState d{c->d_status.as<uint8_t>(), c->d_xrank.as<uint32_t>(), c->d_ekey.as<uint32_t>(),
                  c->d_dict_lsb_raw.as<uint64_t>(), c->d_ballot.p ? c->d_ballot.as<Bal>() : nullptr,
                  c->dmiss_on ? c->d_mref.as<uint32_t>() : nullptr,
                  c->d_ent.as<uint2>(), c->d_krec.as<KeyRec>(), c->d_kent.as<KeyEntry>()};
    CfkDerivedBufs b{c->d_cand.as<uint32_t>(), c->d_cand.cap / 4, c->d_cwr.as<uint32_t>(), c->d_cwr.cap / 4,
                     c->d_w.as<uint2>(), c->d_w.cap / 8};
    const CfkGrow grow{c, cfk_grow_dict, cfk_grow_entries, cfk_swap_entries, cfk_ballot_init, cfk_dict_spare, cfk_dict_swap,
                       c->d_rtxw.as<uint32_t>(), c->ds.n_rent, c->d_cell_ent.as<uint64_t>(), c->ds.cell_ent ? c->n_cell_ent : 0,
                       c->d_rb_wm.as<uint32_t>(), c->ds.n_rb, c->dmiss_on ? c->d_mids.as<uint32_t>() : nullptr,
                       c->dmiss_on ? c->dmiss_ids : 0, cfk_keys_spare, cfk_keys_swap,
                       c->d_kcell.p ? c->d_kcell.as<uint32_t>() : nullptr};
    CfkPruneOut o;
    std::string e;
    CfkMiss miss;
    miss.on = c->dmiss_on;
    miss.n_lists = c->dmiss_lists;
    miss.off = c->d_moff.as<uint64_t>();
    miss.ids = c->d_mids.as<uint32_t>();
    miss.ctx = c;
    miss.spare = cfk_miss_spare;
    miss.swap = cfk_miss_swap;
    const int rc = run_cfk_prune(c->cu, c->ds, d, keys ? c->d_prune_keys.as<uint32_t>() : nullptr, keys ? kl.size() : nk,
                                 prune_interval, min_hlc_delta, &b, cfk_need_bufs, c, grow, c->stream, &o, &e, &miss);
    if (rc)
    {
        // the derived arrays may be half built: rebuild everything from the entries at the next use
        c->host_stale = true;
        c->dirty = true;
        return c->fail(rc, "ad_cfk_prune: %s", e.c_str());
    }
    if (o.n_removed)
    {
        if (c->kline_slots)
            HIPCHK(c, run_build_klines(c->ds, c->d_kslot.as<uint32_t>(), c->d_kcell.as<uint32_t>(), c->d_kline.as<KeyLine>(),
                                       c->kline_slots, c->stream));
        // host copies follow from the device (entries moved; prunedBefore per key as ranks and indices)
        if (K.pruned.empty()) K.pruned.assign(nk, -1);
        if (c->h_pruned.size() != nk) c->h_pruned.assign(nk, 0);
        c->host_moved = true;
        c->host_ingested = false;     // entries moved after the ingest
        c->host_stale = true;
        ++c->snap_gen;
    }
    if (n_removed) *n_removed = o.n_removed;
    if (stats)
    {
        *stats = ad_stats{};
        stats->ms_device = o.ms_total;
        stats->n_keys[0] = o.n_removed;
        stats->n_keys[1] = o.n_keys_pruned;
    }
    return AD_OK;
}

int ad_cfk_missing(ad_ctx* c, uint64_t* n_entries, const uint64_t** off, const uint64_t** msb, const uint64_t** lsb,
                   const int32_t** node)
{
    if (!c || !n_entries || !off || !msb || !lsb || !node) return AD_E_INVAL;
    if (!c->cfk.loaded) return c->fail(AD_E_NOT_LOADED, "ad_cfk_load not called");
    if (hipSetDevice(c->device) != hipSuccess) return c->fail(AD_E_DEVICE, "hipSetDevice");
    StreamScope scope_(c->stream, c->cstream);
    if (int rc = sync_host(c)) return rc;
    auto& K = c->cfk;
    if (K.miss_stale) return c->fail(AD_E_STATE, "missing() lists are stale (updates without deps moved entries): load them again");
    const uint64_t ne = K.status.size();
    if (K.miss_off.size() != ne + 1)
    {
        c->z_off.assign(ne + 1, 0);
        *off = c->z_off.data();
    }
    else
        *off = K.miss_off.data();
    const uint64_t nm = K.miss.size();
    c->y_msb.resize(nm);
    c->y_lsb.resize(nm);
    c->y_node.resize(nm);
    for (uint64_t j = 0; j < nm; ++j)
    {
        c->y_msb[j] = K.miss[j].msb;
        c->y_lsb[j] = K.miss[j].lsb;
        c->y_node[j] = K.miss[j].node;
    }
    *n_entries = ne;
    *msb = c->y_msb.data();
    *lsb = c->y_lsb.data();
    *node = c->y_node.data();
    return AD_OK;
}

int ad_cfk_byid(ad_ctx* c, uint64_t* n_keys, const int64_t** keys, const uint64_t** seg, uint64_t* n_entries,
                const uint64_t** txn_msb, const uint64_t** txn_lsb, const int32_t** txn_node, const int64_t** pruned_before)
{
    if (!c || !n_keys || !keys || !seg || !n_entries || !txn_msb || !txn_lsb || !txn_node || !pruned_before) return AD_E_INVAL;
    if (!c->cfk.loaded) return c->fail(AD_E_NOT_LOADED, "ad_cfk_load not called");
    if (hipSetDevice(c->device) != hipSuccess) return c->fail(AD_E_DEVICE, "hipSetDevice");
    StreamScope scope_(c->stream, c->cstream);
    if (int rc = sync_host(c)) return rc;
    auto& K = c->cfk;
    const uint64_t ne = K.txn.size(), nk = K.keys.size();
    c->y_msb.resize(ne);
    c->y_lsb.resize(ne);
    c->y_node.resize(ne);
    for (uint64_t i = 0; i < ne; ++i)
    {
        c->y_msb[i] = K.txn[i].msb;
        c->y_lsb[i] = K.txn[i].lsb;
        c->y_node[i] = K.txn[i].node;
    }
    if (K.pruned.size() == nk) c->y_pruned = K.pruned;
    else c->y_pruned.assign(nk, -1);
    *n_keys = nk;
    *keys = K.keys.data();
    *seg = K.seg.data();
    *n_entries = ne;
    *txn_msb = c->y_msb.data();
    *txn_lsb = c->y_lsb.data();
    *txn_node = c->y_node.data();
    *pruned_before = c->y_pruned.data();
    return AD_OK;
}

// ---- debug invariant checks (check.hip) ------------------------------------------
static int check_finish(ad_ctx* c, hipStream_t st, uint64_t* n_violations, uint64_t* first)
{
    uint64_t h[2] = {0, ~0ull};
    HIPCHK(c, d2h(h, c->chk.p, sizeof(h), st));
    HIPCHK(c, hipStreamSynchronize(st));
    *n_violations = h[0];
    if (first) *first = h[1];
    return AD_OK;
}

static int check_begin(ad_ctx* c, hipStream_t st)
{
    static const uint64_t init[2] = {0, ~0ull};
    if (!c->chk.ensure(sizeof(init))) return c->fail(AD_E_NOMEM, "check counters");
    HIPCHK(c, h2d(c->chk.p, init, sizeof(init), st));
    return AD_OK;
}

int ad_check_result_device(ad_ctx* c, const ad_deps_result* res_dev, void* stream, uint64_t* n_violations, uint64_t* first)
{
    if (!c || !res_dev || !n_violations) return AD_E_INVAL;
    if (!c->cfk.loaded) return c->fail(AD_E_NOT_LOADED, "ad_cfk_load not called");
    if (hipSetDevice(c->device) != hipSuccess) return c->fail(AD_E_DEVICE, "hipSetDevice");
    StreamScope scope_(c->stream, c->cstream);
    for (int m = 0; m < AD_NMAPS && res_dev->n_txns; ++m)
        if (!res_dev->keys_off[m] || !res_dev->keys[m] || !res_dev->txn_off[m] || !res_dev->txns[m] || !res_dev->k2t_off[m] ||
            !res_dev->k2t[m])
            return c->fail(AD_E_INVAL, "ad_check_result_device: a packed array of map %d is missing (AD_PARTS_ONLY result?)", m);
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    scope_.add(st);
    int rc;
    if ((rc = check_begin(c, st))) return rc;
    HIPCHK(c, run_check_result(*res_dev, c->ds.n_dict, c->chk.p, st));
    return check_finish(c, st, n_violations, first);
}

int ad_check_snapshot(ad_ctx* c, uint64_t* n_violations, uint64_t* first)
{
    if (!c || !n_violations) return AD_E_INVAL;
    if (!c->cfk.loaded) return c->fail(AD_E_NOT_LOADED, "ad_cfk_load not called");
    if (hipSetDevice(c->device) != hipSuccess) return c->fail(AD_E_DEVICE, "hipSetDevice");
    StreamScope scope_(c->stream, c->cstream);
    int rc;
    if (c->dirty && (rc = build_snapshot(c))) return rc;
    if ((rc = check_begin(c, c->stream))) return rc;
    HIPCHK(c, run_check_snapshot(c->ds, c->chk.p, c->stream));
    return check_finish(c, c->stream, n_violations, first);
}

}  // extern "C"
