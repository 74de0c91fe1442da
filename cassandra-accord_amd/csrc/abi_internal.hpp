// abi_internal.hpp — what the translation units of the C ABI (abi.cpp, abi_into.cpp, abi_recovery.cpp,
// abi_levels.cpp, abi_exchange.cpp, abi_update.cpp) share: the store context (struct ad_ctx: one
// CommandStore's snapshot in HBM, its batch buffers and host copies), host helpers, and the functions one
// unit calls in another.
//
// Ingest (abi.cpp) restates the derived state of CommandsForKey's constructor (CommandsForKey.java:642-681:
// committedByExecuteAt, maxAppliedWriteByExecuteAt, prunedBefore) and of InMemoryCommandStore.rangeCommands
// (:740-763) once per snapshot; the batch pipeline then answers calculatePartialDeps for every request of a
// batch on the GPU.
#pragma once
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
#include <map>
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

namespace adi {

// ---------------------------------------------------------------------------------------
// helpers
// ---------------------------------------------------------------------------------------
struct Tid {
    uint64_t msb, lsb;
    int32_t node;
};

inline NormTid norm(const Tid& t) { return norm_tid(t.msb, t.lsb, t.node); }

inline unsigned n_threads()
{
    unsigned n = std::thread::hardware_concurrency();
    if (const char* e = getenv("OMP_NUM_THREADS")) n = std::max(1, atoi(e));
    return std::max(1u, std::min(n, 16u));
}

template <class T, class Cmp>
inline void parallel_sort(std::vector<T>& v, Cmp cmp)
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
inline void parallel_for(size_t n, F f, size_t grain = 1 << 14)
{
    const unsigned T_ = std::min(n_threads(), host_threads());
    if (n < grain * 2 || T_ == 1)
    {
        f(0, n);
        return;
    }
    host_parallel(T_, [&](size_t i) { f(n * i / T_, n * (i + 1) / T_); });
}

inline double now_ms()
{
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // namespace adi

using namespace adi;

// ---------------------------------------------------------------------------------------
// the store context
// ---------------------------------------------------------------------------------------
struct ad_ctx {
    ad_config cfg{};
    std::vector<int64_t> slice_s, slice_e;
    // slice sets of per-request slices (ad_slice_sets_load; DevSnapshot.sset_*)
    std::vector<uint64_t> ss_off;
    std::vector<int64_t> ss_start, ss_end;
    DevBuf d_ss_off, d_ss_start, d_ss_end;
    DevBuf q_ss, s_ss;                         // a batch's staged slice_set; the deferred sub-batch's
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
    double ms_truncate = 0;         // RedundantBefore truncations since the last stats read (device time)
    uint64_t n_truncated = 0;       // entries they removed
    uint64_t n_trunc_keys = 0;      // CommandsForKeys they changed

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
    DevBuf d_ds_bkt;                               // their bucket index (build_dict_buckets)
    DevBuf d_kline, d_kslot, d_kcell, d_kl_disp;   // KeyLine table; per key its line and stabbing cell; displacements
    uint64_t kline_slots = 0;
    // host state of the KeyLine perfect hash (incremental placement of new keys)
    std::vector<uint32_t> kl_disp_h;
    std::vector<uint8_t> kl_used;
    std::vector<std::vector<int64_t>> kl_members;   // per bucket (built on first use from kl_keys_all)
    std::vector<int64_t> kl_keys_all;
    uint64_t kl_nb_h = 0;
    // new keys of an update batch placed on a host thread while the batch runs on the device
    // (cfk_keys_added); joined right after run_cfk_update, consumed by cfk_after_new_keys
    std::thread kl_thread;
    bool kl_async = false, kl_async_rebuild = false;
    int kl_async_rc = 0;
    DevBuf d_keys2, d_krec2, d_kcell2, d_khash2, d_kent2;   // spare key-indexed arrays (new keys)

    // batch buffers
    DevBuf q_tm, q_tl, q_tn, q_em, q_el, q_en, q_me, q_ko, q_k;
    DevBuf q_ro, q_rs, q_re;                   // Range-domain requests: staged ranges
    bool upd_applied = false;                  // ad_cfk_update_status: the last update batch stands
    int64_t upd_failed = -1;                   //   and the update its failure names
    DevBuf rq_cnt, rq_off, rq_err, rq_bsum, rq_keys, rq_hi, rq_kind, rq_list;   // their expansion into probes
    struct SplitBufs {       // per-request / per-probe arrays of the split kernels
        DevBuf t_S, t_self, t_kinds, t_epoch, p_txn, p_rec, p_off, p_c0, p_c1, p_roff, p_rcnt, p_rb, sz, t_reg;
    } split, sub;
    DevBuf s_tm, s_tl, s_tn, s_em, s_el, s_en, s_me, s_ko, s_k, s_cnt, s_khi, s_kind;   // deferred sub-batch inputs
    DevBuf p_slot;                             // lean passes: per probe its KeyLine (k_prepare)
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
    DevBuf d_adv_m, d_adv_l, d_adv_n, d_adv_rank;     // ad_redundant_advance: the new watermarks, their ranks
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
inline hipError_t copy_sync(void* dst, const void* src, size_t bytes, hipMemcpyKind kind)
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

using namespace adi;

// ---- shared by the abi*.cpp translation units ---------------------------------------------
namespace adi {

template <class T>
bool ens(DevBuf& b, uint64_t n) { return b.ensure(sizeof(T) * std::max<uint64_t>(n, 1)); }

template <class T>
int upload(ad_ctx* c, DevBuf& b, const std::vector<T>& v)
{
    if (!b.ensure(sizeof(T) * std::max<size_t>(v.size(), 1))) return c->fail(AD_E_NOMEM, "hipMalloc %zu", sizeof(T) * v.size());
    if (!v.empty()) HIPCHK(c, h2d(b.p, v.data(), sizeof(T) * v.size(), c->stream));
    return 0;
}

template <class T>
T* stage_q(ad_ctx* c, DevBuf& b, const T* src, uint64_t n, int* rc)
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

// A small upload (at most UP_WORDS words) ordered on a stream without a host wait (up_small); UP_WORDS pinned
// words for read-backs that end in one synchronisation (rb_slot)
constexpr uint64_t UP_WORDS = 512;
hipError_t up_small(ad_ctx* c, int k, void* dst, const void* src, size_t bytes, hipStream_t st);
uint64_t* rb_slot(ad_ctx* c);

// snapshot (abi.cpp): build, host copies of the device state, the node-wide dictionary, the KeyLine hash
int build_snapshot(ad_ctx* c);
int build_dict_buckets(ad_ctx* c, hipStream_t st);   // abi_snapshot.cpp: the sample level's bucket index
// the snapshot truncated to the RedundantBefore it holds (SafeCommandStore.maybeTruncate, every key)
int truncate_to_rb(ad_ctx* c);
// Range commands and RedundantBefore of a snapshot build (abi_snapshot.cpp): the stabbing index's cell ends,
// whether it could be built, the range entries
struct RangePart {
    std::vector<int64_t> cell_E;
    bool cell_ok = false;
    uint64_t n_rent = 0;
};
int build_ranges(ad_ctx* c, const std::vector<uint32_t>& cmd_rank, const std::vector<uint32_t>& wm_rank, RangePart* out);
int set_range_views(ad_ctx* c, const RangePart& rp, uint64_t nrb);
// the key's shardRedundantBefore on the host copy (RedundantBefore.get; null: none or NONE), and whether
// t is below it
const Tid* rb_wm_of(const ad_ctx* c, int64_t key);
bool below_redundant(const ad_ctx* c, int64_t key, const Tid& t);
bool tid_gt_none(const Tid& t);
int sync_host(ad_ctx* c);
int host_dict(ad_ctx* c);
int pull_missing(ad_ctx* c);
void drop_global_dict(ad_ctx* c);
int kl_place_all(ad_ctx* c, const std::vector<int64_t>& keys, uint64_t nb, bool sparse);
int kl_add_keys(ad_ctx* c, const std::vector<int64_t>& nkeys, uint64_t nk_total, bool* need_rebuild);
// batches (abi.cpp): validation, SEQUENTIAL insertion, the pipeline, host results
int check_query_host(ad_ctx* c, const ad_query_soa* q, uint32_t flags = 0);
int sequential_on_device(ad_ctx* c, const ad_query_soa* q);
int apply_preaccepts(ad_ctx* c, const ad_query_soa* q);
int run_pipeline(ad_ctx* c, const ad_query_soa* q, hipStream_t st, ad_deps_result* out, bool parts_only = false,
                 bool n_keys_given = false, int recovery_scan = -1, const RecoveryView* rv = nullptr);
int result_to_host(ad_ctx* c, uint64_t n, const ad_deps_result& dev, ad_deps_result** out);
// CommandsForKey maintenance (abi_update.cpp)
int cfk_need_bufs(void* vc, uint64_t n_cand, uint64_t n_cwr, uint64_t n_w, CfkDerivedBufs* b);
// the CfkGrow / CfkMiss callbacks over the ctx's buffers
int cfk_grow_dict(void* vc, uint64_t n_old, uint64_t n_new, uint64_t** hi, uint64_t** lo, int32_t** node, uint64_t** raw);
int cfk_grow_entries(void* vc, uint64_t ne, uint2** ent, uint8_t** st, uint32_t** xr, uint32_t** ek, Bal** bal, uint32_t** mref);
int cfk_swap_entries(void* vc, uint64_t ne, uint2** ent, uint8_t** st, uint32_t** xr, uint32_t** ek, Bal** bal, uint32_t** mref);
int cfk_ballot_init(void* vc, uint64_t ne, Bal** bal);
int cfk_dict_spare(void* vc, uint64_t n, uint64_t** hi, uint64_t** lo, int32_t** node, uint64_t** raw);
int cfk_dict_swap(void* vc, uint64_t** hi, uint64_t** lo, int32_t** node, uint64_t** raw);
int cfk_keys_spare(void* vc, uint64_t nk, KeyBufs* b);
int cfk_keys_swap(void* vc, KeyBufs* b);
void cfk_keys_added(void* vc, const int64_t* keys, uint64_t n, uint64_t nk, hipStream_t st);
void kl_join(ad_ctx* c);
int cfk_miss_spare(void* vc, uint64_t n, uint64_t n_ids, uint64_t** off, uint32_t** ids);
int cfk_miss_swap(void* vc, uint64_t** off, uint32_t** ids);
int cfk_update_run(ad_ctx* c, const CfkUpdIn& u, hipStream_t st, uint64_t* n_applied, ad_stats* stats);
int cfk_update_follow(ad_ctx* c, const CfkUpdOut& o, int rc, hipStream_t st);
// ids (host) joined to the device dictionary where it does not hold them; ranks[i] their member ranks (host
// copies follow as after an update batch). ms: host-timed.
int dict_ensure_ids(ad_ctx* c, const std::vector<Tid>& ids, std::vector<uint32_t>* ranks, uint64_t* n_new);

}  // namespace adi
