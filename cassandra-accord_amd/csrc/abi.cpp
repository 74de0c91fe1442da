// abi.cpp — C ABI of libaccord_deps.so, core: store context lifecycle, the snapshot loads (ad_cfk_load,
// ad_range_cmds_load / _update, ad_redundant_load, slice sets), SEQUENTIAL insertion, the batch entry points
// (ad_deps_batch, ad_deps_batch_device), dictionary views, invariant checks. The snapshot build is in
// abi_snapshot.cpp, the batch pipeline in abi_resolve.cpp.
#include "abi_internal.hpp"

namespace adi {

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
// RangeCommand.update's union with its earlier ranges is not modelled). The registry is an unordered set:
// a new command is appended (the oracle's TreeMap inserts it in TxnId order); the snapshot build sorts the
// range part by TxnId and recovery facts are parallel arrays appended alongside, so nothing reads position
// as order (tests/test_gpu_ranges.py::test_sequential_range_txn_below_registered).
int register_range_txns(ad_ctx* c, const ad_query_soa* q, const std::vector<uint64_t>& idx)
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
int apply_preaccepts(ad_ctx* c, const ad_query_soa* q)
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
            // CommandsForKey.update ignores a txnId below the key's shardRedundantBefore (CommandsForKey.java:997)
            if (in && !below_redundant(c, key, t)) ins.push_back({key, norm(t), t});
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

// =======================================================================================
// C ABI
// =======================================================================================

// ---- range-command registry upkeep (ad_range_cmds_update) ------------------------------------
using RangeList = std::vector<std::pair<int64_t, int64_t>>;

// Range.compareIntersecting (Range.java:296-305)
static int cmp_intersecting(const std::pair<int64_t, int64_t>& x, const std::pair<int64_t, int64_t>& y)
{
    if (x.first >= y.second) return 1;
    if (x.second <= y.first) return -1;
    return 0;
}

// Ranges.with (Ranges.java:136-139): AbstractRanges.union(MERGE_OVERLAPPING) (:486-574) after
// supersetLinearMerge (:429-474) -- a run that merged an intersection also takes touching ranges
RangeList ranges_with(const RangeList& left, const RangeList& right)
{
    if (right.empty()) return left;
    if (left.empty()) return right;
    const RangeList* A = &left;
    const RangeList* B = &right;
    if ((*A)[0].first > (*B)[0].first || ((*A)[0].first == (*B)[0].first && A->back().second < B->back().second)) std::swap(A, B);
    const RangeList& as = *A;
    const RangeList& bs = *B;
    size_t ai = 0, bi = 0;
    while (ai < as.size() && bi < bs.size())
    {
        auto a = as[ai];
        const auto b = bs[bi];
        const int c = cmp_intersecting(a, b);
        if (c < 0) ++ai;
        else if (c > 0 || b.first < a.first) break;
        else if (b.second <= a.second)
        {
            ++bi;
            if (b.second == a.second) ++ai;
        }
        else
        {
            size_t t = ai;
            bool out = false;
            do
            {
                if (++t == as.size() || a.second != as[t].first) { out = true; break; }
                a = as[t];
            } while (a.second < b.second);
            if (out) break;
            ++bi;
            ai = t;
        }
    }
    if (bi == bs.size()) return as;
    RangeList r(as.begin(), as.begin() + ai);
    while (ai < as.size() && bi < bs.size())
    {
        auto a = as[ai];
        const auto b = bs[bi];
        const int c = cmp_intersecting(a, b);
        if (c < 0) { r.push_back(a); ++ai; }
        else if (c > 0) { r.push_back(b); ++bi; }
        else
        {
            const int64_t start = std::min(a.first, b.first);
            int64_t end = std::max(a.second, b.second);
            ++ai;
            ++bi;
            while (ai < as.size() || bi < bs.size())
            {
                std::pair<int64_t, int64_t> mn;
                bool from_a;
                if (ai == as.size()) { mn = bs[bi]; from_a = false; }
                else if (bi == bs.size() || as[ai].first < bs[bi].first) { mn = a = as[ai]; from_a = true; }
                else { mn = bs[bi]; from_a = false; }
                if (mn.first > end) break;
                if (mn.second > end) end = mn.second;
                if (from_a) ++ai;
                else ++bi;
            }
            r.push_back({start, end});
        }
    }
    r.insert(r.end(), as.begin() + ai, as.end());
    r.insert(r.end(), bs.begin() + bi, bs.end());
    return r;
}

// The range part of a built snapshot rebuilt from the host registry (range entries, range table, stabbing cells,
// per-key cells in the key hash and KeyLines, range trees, RedundantBefore views) -- the CommandsForKeys, their
// derived arrays and the dictionary stay; commands [n_old, n) are new: their txnIds join the dictionary first.
int refresh_range_part(ad_ctx* c, uint64_t n_old, uint64_t* n_new_ids)
{
    const auto& R = c->cmds;
    const uint64_t ncmd = R.txn.size(), nrb = c->rb.wm.size(), nk = c->ds.n_keys;
    hipStream_t st = c->stream;
    *n_new_ids = 0;
    if (c->h_cmd_rank.size() != n_old) return c->fail(AD_E_STATE, "range command ranks out of step (internal)");
    if (ncmd > n_old)
    {
        std::vector<Tid> ids(R.txn.begin() + n_old, R.txn.end());
        std::vector<uint32_t> ranks;
        if (int rc = dict_ensure_ids(c, ids, &ranks, n_new_ids)) return rc;
        c->h_cmd_rank.insert(c->h_cmd_rank.end(), ranks.begin(), ranks.end());
    }
    std::vector<uint32_t> wm_rank(nrb, 0);
    if (nrb)
    {
        HIPCHK(c, d2h(wm_rank.data(), c->d_rb_wm.p, 4 * nrb, st));
        HIPCHK(c, hipStreamSynchronize(st));
    }
    RangePart rp;
    if (int rc = build_ranges(c, c->h_cmd_rank, wm_rank, &rp)) return rc;
    if (int rc = set_range_views(c, rp, nrb)) return rc;
    if (int rc = upload(c, c->d_rt_start, c->rt_start)) return rc;
    if (int rc = upload(c, c->d_rt_end, c->rt_end)) return rc;
    // every key's stabbing cell (KeySlot and the per-key array the KeyLines read) under the new endpoints
    if (nk)
        HIPCHK(c, ingest_keys(c->d_keys.as<int64_t>(), nk, rp.cell_ok ? c->d_cell_E.as<int64_t>() : nullptr,
                              rp.cell_ok ? rp.cell_E.size() : 0, c->cfg.range_start_inclusive, c->d_kcell.as<uint32_t>(),
                              c->d_khash.as<KeySlot>(), c->ds.khash_mask + 1, st));
    HIPCHK(c, build_range_trees(c->ds, st));
    if (c->kline_slots)
        HIPCHK(c, run_build_klines(c->ds, c->d_kslot.as<uint32_t>(), c->d_kcell.as<uint32_t>(), c->d_kline.as<KeyLine>(),
                                   c->kline_slots, st));
    HIPCHK(c, hipStreamSynchronize(st));
    c->rv_rng_gen = ~0ull;
    return 0;
}

}  // namespace adi

extern "C" {

int ad_abi_version(void) { return AD_ABI_VERSION; }

}  // extern "C"

namespace adi {

static thread_local std::string g_create_err;

}  // namespace adi

extern "C" {

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
    kl_join(c);
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

int ad_range_cmds_update(ad_ctx* c, const ad_range_cmds_soa* in, ad_stats* stats)
{
    if (!c || !in) return AD_E_INVAL;
    const uint64_t n = in->n_cmds;
    if (n && (!in->txn_msb || !in->txn_lsb || !in->txn_node || !in->range_off || (in->range_off[n] && (!in->range_start || !in->range_end))))
        return c->fail(AD_E_INVAL, "ad_range_cmds_update: null arrays");
    for (uint64_t i = 0; i < n; ++i)
    {
        if ((in->txn_lsb[i] & 1) == 0) return c->fail(AD_E_INVAL, "range command %llu has a key-domain TxnId", (unsigned long long)i);
        if (in->range_off[i + 1] < in->range_off[i]) return c->fail(AD_E_INVAL, "range_off not monotone");
        for (uint64_t r = in->range_off[i]; r < in->range_off[i + 1]; ++r)
            if (in->range_start[r] >= in->range_end[r] || (r > in->range_off[i] && in->range_start[r] < in->range_end[r - 1]))
                return c->fail(AD_E_INVAL, "range command %llu: ranges not normalised", (unsigned long long)i);
    }
    if (stats) *stats = ad_stats{};
    const double t0 = now_ms();
    auto& R = c->cmds;
    const uint64_t n_old = R.txn.size();
    // the registry as per-command range lists (only the touched ones materialised), live / historical by TxnId
    auto cmp = [](const NormTid& a, const NormTid& b) { return norm_cmp(a, b) < 0; };
    std::map<NormTid, uint64_t, decltype(cmp)> live(cmp), hist(cmp);
    for (uint64_t i = 0; i < n_old; ++i)
        ((!R.historical.empty() && R.historical[i]) ? hist : live)[norm(R.txn[i])] = i;
    std::map<uint64_t, RangeList> touched;
    auto ranges_of = [&](uint64_t i) -> RangeList& {
        auto it = touched.find(i);
        if (it != touched.end()) return it->second;
        RangeList& l = touched[i];
        if (i < n_old)
            for (uint64_t r = R.off[i]; r < R.off[i + 1]; ++r) l.push_back({R.start[r], R.end[r]});
        return l;
    };
    if (R.erased.empty()) R.erased.assign(n_old, 0);
    if (R.historical.empty()) R.historical.assign(n_old, 0);
    auto add_cmd = [&](const Tid& t, uint8_t historical) -> uint64_t {
        const uint64_t i = R.txn.size();
        R.txn.push_back(t);
        R.erased.push_back(0);
        R.historical.push_back(historical);
        touched[i];
        (historical ? hist : live)[norm(t)] = i;
        return i;
    };
    for (uint64_t i = 0; i < n; ++i)
    {
        const Tid t{in->txn_msb[i], in->txn_lsb[i], in->txn_node[i]};
        const NormTid k = norm(t);
        RangeList add;
        for (uint64_t r = in->range_off[i]; r < in->range_off[i + 1]; ++r) add.push_back({in->range_start[r], in->range_end[r]});
        if (in->historical && in->historical[i])
        {
            // registerHistoricalTransactions: nothing when rangeCommands holds it (InMemoryCommandStore.java:814-828)
            if (live.count(k)) continue;
            auto it = hist.find(k);
            const uint64_t j = it != hist.end() ? it->second : add_cmd(t, 1);
            RangeList& l = ranges_of(j);
            l = ranges_with(l, add);
        }
        else if (in->erased && in->erased[i])
        {
            auto it = live.find(k);          // the command's status became Erased: the scan skips it (:892)
            if (it != live.end()) R.erased[it->second] = 1;
        }
        else
        {
            // InMemorySafeStore.update (:740-763): computeIfAbsent(txnId).update(ranges) (RangeCommand.update :547-551)
            auto it = live.find(k);
            const uint64_t j = it != live.end() ? it->second : add_cmd(t, 0);
            RangeList& l = ranges_of(j);
            l = ranges_with(l, add);
        }
    }
    // the registry's CSR again
    const uint64_t ncmd = R.txn.size();
    std::vector<uint64_t> off(ncmd + 1, 0);
    std::vector<int64_t> st, en;
    st.reserve(R.start.size() + 16);
    en.reserve(R.end.size() + 16);
    for (uint64_t i = 0; i < ncmd; ++i)
    {
        auto it = touched.find(i);
        if (it != touched.end())
            for (auto& p : it->second) { st.push_back(p.first); en.push_back(p.second); }
        else
            for (uint64_t r = R.off[i]; r < R.off[i + 1]; ++r) { st.push_back(R.start[r]); en.push_back(R.end[r]); }
        off[i + 1] = st.size();
    }
    R.off.swap(off);
    R.start.swap(st);
    R.end.swap(en);
    R.rec = false;                   // recovery facts belong to the registry as it was (reload them)
    c->rv_rng_gen = ~0ull;
    const double ms_host = now_ms() - t0;
    if (!c->cfk.loaded || c->dirty) return AD_OK;     // the next build reads the registry
    if (hipSetDevice(c->device) != hipSuccess) return c->fail(AD_E_DEVICE, "hipSetDevice");
    StreamScope scope_(c->stream, c->cstream);
    uint64_t n_new = 0;
    const double t1 = now_ms();
    if (int rc = refresh_range_part(c, n_old, &n_new))
    {
        c->dirty = true;
        return rc;
    }
    if (stats)
    {
        stats->ms_stage[0] = ms_host;                 // registry upkeep on the host copy
        stats->ms_stage[1] = now_ms() - t1;           // range part rebuilt (dictionary growth included)
        stats->n_keys[0] = ncmd - n_old;              // commands registered
        stats->n_keys[1] = c->ds.n_rent;              // range entries
        stats->n_keys[2] = n_new;                     // ids added to the dictionary
    }
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

int ad_slice_sets_load(ad_ctx* c, uint32_t n_sets, const uint64_t* set_off, const int64_t* start, const int64_t* end)
{
    if (!c || (n_sets && !set_off)) return AD_E_INVAL;
    const uint64_t nr = n_sets ? set_off[n_sets] : 0;
    if (nr && (!start || !end)) return c->fail(AD_E_INVAL, "slice sets: start / end required");
    for (uint32_t k = 0; k < n_sets; ++k)
    {
        if (set_off[k] > set_off[k + 1]) return c->fail(AD_E_INVAL, "slice sets: set_off not monotone at set %u", k);
        for (uint64_t j = set_off[k]; j < set_off[k + 1]; ++j)
            if (start[j] >= end[j] || (j > set_off[k] && end[j - 1] > start[j]))
                return c->fail(AD_E_INVAL, "slice set %u: ranges not normalised (start < end, ascending, disjoint)", k);
    }
    if (n_sets && set_off[0] != 0) return c->fail(AD_E_INVAL, "slice sets: set_off[0] must be 0");
    if (hipSetDevice(c->device) != hipSuccess) return c->fail(AD_E_DEVICE, "hipSetDevice");
    StreamScope scope_(c->stream, c->cstream);
    c->ss_off.assign(set_off, set_off + (n_sets ? n_sets + 1 : 0));
    c->ss_start.assign(start, start + nr);
    c->ss_end.assign(end, end + nr);
    int rc;
    if ((rc = upload(c, c->d_ss_off, c->ss_off)) || (rc = upload(c, c->d_ss_start, c->ss_start)) ||
        (rc = upload(c, c->d_ss_end, c->ss_end)))
        return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    // the views of a built snapshot (a later build takes them from the ctx too, set_views)
    c->ds.n_ssets = n_sets;
    c->ds.sset_off = c->d_ss_off.as<uint64_t>();
    c->ds.sset_start = c->d_ss_start.as<int64_t>();
    c->ds.sset_end = c->d_ss_end.as<int64_t>();
    return AD_OK;
}

}  // extern "C"

namespace adi {


// SEQUENTIAL PreAccepts as device-side CommandsForKey.update insertions (PREACCEPTED, executeAt =
// txnId) of every request into the CommandsForKey of each of its keys in the slice, as
// apply_preaccepts does on the host (keys without a CommandsForKey and older ids included). Returns
// 0 (applied), 1 (not applicable here: no built snapshot, or a batch the device path refuses) or an
// AD_E_* error.
int sequential_on_device(ad_ctx* c, const ad_query_soa* q)
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
            if (!in || below_redundant(c, key, t)) continue;          // CommandsForKey.java:997
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

}  // namespace adi

extern "C" {

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
    d.slice_set = stage_q(c, c->q_ss, q->slice_set, n, &rc);
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
    host_trace("resolve: enter");
    // AD_REGIONS and AD_PARTS_ONLY: no packed copy (the regions are the result)
    rc = run_pipeline(c, q, st, out, (flags & (AD_PARTS_ONLY | AD_REGIONS)) != 0, (flags & AD_N_KEYS) != 0);
    host_trace("resolve: done");
    return rc;
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

int ad_copy_to_host(ad_ctx* c, void* dst, const void* src, uint64_t bytes)
{
    if (!c || (!dst && bytes) || (!src && bytes)) return AD_E_INVAL;
    if (!bytes) return AD_OK;
    if (hipSetDevice(c->device) != hipSuccess) return c->fail(AD_E_DEVICE, "hipSetDevice");
    StreamScope scope_(c->stream, c->cstream);
    HIPCHK(c, copy_sync(dst, src, bytes, hipMemcpyDeviceToHost));
    return AD_OK;
}

}  // extern "C"

namespace adi {

// ---- debug invariant checks (check.hip) ------------------------------------------
int check_finish(ad_ctx* c, hipStream_t st, uint64_t* n_violations, uint64_t* first)
{
    uint64_t h[2] = {0, ~0ull};
    HIPCHK(c, d2h(h, c->chk.p, sizeof(h), st));
    HIPCHK(c, hipStreamSynchronize(st));
    *n_violations = h[0];
    if (first) *first = h[1];
    return AD_OK;
}

int check_begin(ad_ctx* c, hipStream_t st)
{
    static const uint64_t init[2] = {0, ~0ull};
    if (!c->chk.ensure(sizeof(init))) return c->fail(AD_E_NOMEM, "check counters");
    HIPCHK(c, h2d(c->chk.p, init, sizeof(init), st));
    return AD_OK;
}

}  // namespace adi

extern "C" {

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
