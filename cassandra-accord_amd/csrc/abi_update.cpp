// abi_update.cpp — device-resident CommandsForKey maintenance: ad_cfk_update*, pruning, missing() lists,
// ballots and the store's views (ad_cfk_entries, ad_cfk_byid).
#include "abi_internal.hpp"

namespace adi {

// ---- device-resident CommandsForKey maintenance ----------------------------
int cfk_need_bufs(void* vc, uint64_t n_cand, uint64_t n_cwr, uint64_t n_w, CfkDerivedBufs* b)
{
    ad_ctx* c = (ad_ctx*)vc;
    // (with slack: the store grows every batch -- an exact-size buffer would be reallocated by each one)
    if (!c->d_cand.grow(4 * std::max<uint64_t>(n_cand, 1)) || !c->d_cwr.grow(4 * std::max<uint64_t>(n_cwr, 1)) ||
        !c->d_w.grow(8 * std::max<uint64_t>(n_w, 1)))
        return AD_E_NOMEM;
    b->cand = c->d_cand.as<uint32_t>();
    b->cwr = c->d_cwr.as<uint32_t>();
    b->w = c->d_w.as<uint2>();
    return 0;
}

// DevBuf growth keeping the first `keep` bytes (slack for the next batches)
bool grow_keep(DevBuf& b, size_t keep, size_t need)
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

int cfk_grow_dict(void* vc, uint64_t n_old, uint64_t n_new, uint64_t** hi, uint64_t** lo, int32_t** node, uint64_t** raw)
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

int cfk_grow_entries(void* vc, uint64_t ne, uint2** ent, uint8_t** st, uint32_t** xr, uint32_t** ek, Bal** bal,
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

void swap_buf(DevBuf& a, DevBuf& b)
{
    std::swap(a.p, b.p);
    std::swap(a.cap, b.cap);
}

int size_cfk_trees(ad_ctx* c, uint64_t ne)
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
            if (!c->d_lvl[cl][l].grow(sizeof(uint32_t) * ((s.lvl_n[l] + 63) / 64 * 64))) return AD_E_NOMEM;
            s.lvl[cl][l] = c->d_lvl[cl][l].as<uint32_t>();
        }
    return 0;
}

int cfk_swap_entries(void* vc, uint64_t ne, uint2** ent, uint8_t** st, uint32_t** xr, uint32_t** ek, Bal** bal,
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

int cfk_ballot_init(void* vc, uint64_t ne, Bal** bal)
{
    ad_ctx* c = (ad_ctx*)vc;
    if (!c->d_ballot.ensure(sizeof(Bal) * ne + sizeof(Bal) * (ne / 4))) return AD_E_NOMEM;
    if (dev_zero_sync(c->d_ballot.p, sizeof(Bal) * ne) != hipSuccess) return AD_E_DEVICE;
    *bal = c->d_ballot.as<Bal>();
    return 0;
}

int cfk_keys_spare(void* vc, uint64_t nk, KeyBufs* b)
{
    ad_ctx* c = (ad_ctx*)vc;
    uint64_t hcap = 16;
    while (hcap < 2 * nk) hcap <<= 1;
    if (!c->d_keys2.grow(8 * nk) || !c->d_krec2.grow(sizeof(KeyRec) * nk) || !c->d_kcell2.grow(4 * nk) ||
        !c->d_khash2.ensure(sizeof(KeySlot) * hcap) || !c->d_kent2.grow(sizeof(KeyEntry) * nk))
        return AD_E_NOMEM;
    *b = KeyBufs{c->d_keys2.as<int64_t>(), c->d_krec2.as<KeyRec>(), c->d_kcell2.as<uint32_t>(), c->d_khash2.as<KeySlot>(),
                 c->d_kent2.as<KeyEntry>(), hcap};
    return 0;
}

int cfk_keys_swap(void* vc, KeyBufs* b)
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

// The batch's new keys, as soon as add_keys has them: placed in the KeyLine hash on a host thread while
// the rest of the batch runs on the device (the placement is host work of ~0.1 ms per 1000 keys). Nothing
// else touches the KeyLine host state until kl_join.
void cfk_keys_added(void* vc, const int64_t* keys, uint64_t n, uint64_t nk, hipStream_t st)
{
    ad_ctx* c = (ad_ctx*)vc;
    kl_join(c);
    c->kl_async = false;
    if (!n) return;
    std::vector<int64_t> nkeys(n);
    if (d2h(nkeys.data(), keys, 8 * n, st) != hipSuccess || hipStreamSynchronize(st) != hipSuccess) return;   // later, synchronously
    c->kl_async = true;
    c->kl_async_rc = 0;
    c->kl_async_rebuild = false;
    try
    {
        c->kl_thread = std::thread([c, nkeys = std::move(nkeys), nk]() {
            bool rebuild = false;
            c->kl_async_rc = kl_add_keys(c, nkeys, nk, &rebuild);
            c->kl_async_rebuild = rebuild;
        });
    }
    catch (...)
    {
        c->kl_async = false;
    }
}

void kl_join(ad_ctx* c)
{
    if (c->kl_thread.joinable()) c->kl_thread.join();
}

// After new keys on the device: the KeyLine perfect hash takes them (incrementally on the host -- already
// done by cfk_keys_added's thread when it ran), displacements uploaded, every key's line recomputed on the device.
int cfk_after_new_keys(ad_ctx* c, const CfkUpdOut& o, hipStream_t st)
{
    const uint64_t nk = c->ds.n_keys, U = o.n_new_keys;
    bool rebuild = false;
    kl_join(c);
    if (c->kl_async)
    {
        c->kl_async = false;
        if (c->kl_async_rc) return c->kl_async_rc;
        rebuild = c->kl_async_rebuild;
    }
    else
    {
        std::vector<int64_t> nkeys(U);
        HIPCHK(c, d2h(nkeys.data(), o.new_keys, 8 * U, st));
        HIPCHK(c, hipStreamSynchronize(st));
        if (int rc = kl_add_keys(c, nkeys, nk, &rebuild)) return rc;
    }
    host_trace("new_keys: kl_add_keys (joined)");
    if (rebuild)
    {
        // the whole table again, half full (every key of the store, from the device)
        std::vector<int64_t> all(nk);
        HIPCHK(c, copy_sync(all.data(), c->d_keys.p, 8 * nk, hipMemcpyDeviceToHost));
        if (int rc = kl_place_all(c, all, std::max<uint64_t>(1, nk / 4), true)) return c->fail(rc, "key perfect hash did not converge");
    }
    if (int rc = upload(c, c->d_kl_disp, c->kl_disp_h)) return rc;
    host_trace("new_keys: disp upload");
    if (!c->d_kslot.grow(4 * nk)) return c->fail(AD_E_NOMEM, "key slots");
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

int cfk_dict_spare(void* vc, uint64_t n, uint64_t** hi, uint64_t** lo, int32_t** node, uint64_t** raw)
{
    ad_ctx* c = (ad_ctx*)vc;
    if (!c->d_dict_hi2.grow(8 * n) || !c->d_dict_lo2.grow(8 * n) || !c->d_dict_node2.grow(4 * n) ||
        !c->d_dict_raw2.grow(8 * n))
        return AD_E_NOMEM;
    *hi = c->d_dict_hi2.as<uint64_t>();
    *lo = c->d_dict_lo2.as<uint64_t>();
    *node = c->d_dict_node2.as<int32_t>();
    *raw = c->d_dict_raw2.as<uint64_t>();
    return 0;
}

int cfk_dict_swap(void* vc, uint64_t** hi, uint64_t** lo, int32_t** node, uint64_t** raw)
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
int cfk_after_merge(ad_ctx* c, const uint64_t* pos_dev, uint64_t U, hipStream_t st)
{
    // (a current host dictionary is read back whole below -- a stale one stays stale, read on demand; host rank
    // copies that are stale -- host_moved -- are rebuilt from the device later, their remap here is then moot)
    const uint64_t nd = c->ds.n_dict;
    std::vector<uint64_t> pos(U);
    HIPCHK(c, d2h(pos.data(), pos_dev, 8 * U, st));
    if (!c->host_dict_stale)
    {
        c->dict_msb.resize(nd);
        c->dict_lsb.resize(nd);
        c->dict_node.resize(nd);
        HIPCHK(c, d2h(c->dict_msb.data(), c->d_dict_hi.p, 8 * nd, st));
        HIPCHK(c, d2h(c->dict_lsb.data(), c->d_dict_lsb_raw.p, 8 * nd, st));
        HIPCHK(c, d2h(c->dict_node.data(), c->d_dict_node.p, 4 * nd, st));
    }
    HIPCHK(c, hipStreamSynchronize(st));
    auto remap = [&](uint32_t r) -> uint32_t {
        if (r == 0) return 0;
        const uint64_t i = (r - 1) / 2;
        return (uint32_t)(2 * (i + (uint64_t)(std::upper_bound(pos.begin(), pos.end(), i) - pos.begin())) + 1);
    };
    auto remap_txw = [&](uint32_t y) -> uint32_t { return (y & ~RANK_MASK) | remap(y & RANK_MASK); };
    // the per-entry copies are rebuilt from the device when they are stale anyway (host_moved)
    if (!c->host_moved)
    {
        for (auto& r : c->h_txn_rank) r = remap(r);
        for (auto& r : c->h_exec_rank) r = remap(r);
        for (auto& r : c->h_pruned) r = remap(r);
    }
    for (auto& r : c->h_cmd_rank) r = remap(r);
    for (auto& y : c->h_rtxw) y = remap_txw(y);
    ++c->rank_gen;
    return 0;
}

int cfk_miss_spare(void* vc, uint64_t n, uint64_t n_ids, uint64_t** off, uint32_t** ids)
{
    ad_ctx* c = (ad_ctx*)vc;
    if (!c->d_moff2.grow(8 * (n + 1)) || !c->d_mids2.grow(4 * std::max<uint64_t>(n_ids, 1)))
        return AD_E_NOMEM;
    *off = c->d_moff2.as<uint64_t>();
    *ids = c->d_mids2.as<uint32_t>();
    c->dmiss_lists = n;
    c->dmiss_ids = n_ids;
    return 0;
}

int cfk_miss_swap(void* vc, uint64_t** off, uint32_t** ids)
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
int dmiss_enable(ad_ctx* c, hipStream_t st)
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

int cfk_update_follow(ad_ctx* c, const CfkUpdOut& o, int rc, hipStream_t st);

int cfk_update_run(ad_ctx* c, const CfkUpdIn& u, hipStream_t st, uint64_t* n_applied, ad_stats* stats)
{
    StreamScope scope_(st, c->stream, c->cstream);
    c->upd_applied = false;
    host_trace("upd: enter");
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
                       c->d_kcell.p ? c->d_kcell.as<uint32_t>() : nullptr, cfk_keys_added};
    if (int rc = host_dict(c)) return rc;
    CfkMiss miss;
    host_trace("upd: host_dict");
    miss.on = c->dmiss_on && u.dep_off;
    miss.n_lists = c->dmiss_lists;
    miss.off = c->d_moff.as<uint64_t>();
    miss.ids = c->d_mids.as<uint32_t>();
    miss.ctx = c;
    miss.spare = cfk_miss_spare;
    miss.swap = cfk_miss_swap;
    c->lp_upd.clear(); c->lp_keys.clear(); c->lp_msb.clear(); c->lp_lsb.clear(); c->lp_node.clear();
    const int rc = run_cfk_update(c->cu, c->ds, d, u, &b, cfk_need_bufs, c, grow, st, &o, &e, &miss);
    kl_join(c);
    if (!o.n_new_keys) c->kl_async = false;
    host_trace("upd: run_cfk_update");
    // what the batch left is known here, before any follow-up copy can fail: a caller reading the status after
    // an error must never take a batch that stands for one that did not (and apply it twice)
    c->upd_applied = rc == AD_OK || o.batch_stood;
    c->upd_failed = o.failed_update;
    const int frc = cfk_update_follow(c, o, rc, st);
    c->kl_async = false;        // consumed by the follow-up, or dropped with it (a failed one leaves the store dirty)
    if (frc)
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
int cfk_update_follow(ad_ctx* c, const CfkUpdOut& o, int rc, hipStream_t st)
{
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
    host_trace("follow: after_new_keys");
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
    if (o.n_new_ids)
    {
        // ids appended to the device dictionary (kept even when the batch then failed): a current host copy takes
        // them (a stale one is read whole on demand)
        const uint64_t nd1 = c->dict_msb.size();
        if (!c->host_dict_stale && c->ds.n_dict > nd1)
        {
            const uint64_t add = c->ds.n_dict - nd1;
            c->dict_msb.resize(nd1 + add);
            c->dict_lsb.resize(nd1 + add);
            c->dict_node.resize(nd1 + add);
            HIPCHK(c, copy_sync(c->dict_msb.data() + nd1, c->d_dict_hi.as<uint64_t>() + nd1, 8 * add, hipMemcpyDeviceToHost));
            HIPCHK(c, copy_sync(c->dict_lsb.data() + nd1, c->d_dict_lsb_raw.as<uint64_t>() + nd1, 8 * add, hipMemcpyDeviceToHost));
            HIPCHK(c, copy_sync(c->dict_node.data() + nd1, c->d_dict_node.as<int32_t>() + nd1, 4 * add, hipMemcpyDeviceToHost));
    host_trace("follow: dict append copy");
        }
        drop_global_dict(c);         // global ranks of the multi-store exchange no longer cover the dictionary
        // the sampled index over the grown dictionary (a stale one is still correct, only slower)
        // (a buffer that could not grow may have been released: then no sample, the searches span the
        // whole dictionary)
        const uint64_t ns = dict_samples(c->ds.n_dict), ne = dict_sample_entries(c->ds.n_dict);
        const bool ok = c->d_ds_hi.grow(8 * ne) && c->d_ds_lo.grow(8 * ne) && c->d_ds_node.grow(4 * ne);
        c->ds.ds_hi = c->d_ds_hi.as<uint64_t>();
        c->ds.ds_lo = c->d_ds_lo.as<uint64_t>();
        c->ds.ds_node = c->d_ds_node.as<int32_t>();
        c->ds.n_samp = ok ? ns : 0;
        c->ds.n_samp2 = ok ? dict_samples2(c->ds.n_dict) : 0;
        if (ok) HIPCHK(c, run_dict_sample(c->ds, c->d_ds_hi.as<uint64_t>(), c->d_ds_lo.as<uint64_t>(), c->d_ds_node.as<int32_t>(), st));
        if (int rb = build_dict_buckets(c, st)) return rb;
    host_trace("follow: dict sample");
    }
    if (o.n_inserted) { c->host_moved = true; c->host_ingested = false; }
    if ((rc == 0 || o.rolled_back || o.rederived || o.batch_stood) && c->kline_slots)
        HIPCHK(c, run_build_klines(c->ds, c->d_kslot.as<uint32_t>(), c->d_kcell.as<uint32_t>(), c->d_kline.as<KeyLine>(),
                                   c->kline_slots, st));
    host_trace("follow: klines");
    return 0;
}

int dict_ensure_ids(ad_ctx* c, const std::vector<Tid>& ids, std::vector<uint32_t>* ranks, uint64_t* n_new)
{
    const uint64_t nx = ids.size();
    ranks->assign(nx, 0);
    *n_new = 0;
    if (!nx) return 0;
    std::vector<uint64_t> xm(nx), xl(nx);
    std::vector<int32_t> xn(nx);
    for (uint64_t j = 0; j < nx; ++j)
    {
        xm[j] = ids[j].msb;
        xl[j] = ids[j].lsb;
        xn[j] = ids[j].node;
    }
    if (int rc = upload(c, c->d_adv_m, xm)) return rc;
    if (int rc = upload(c, c->d_adv_l, xl)) return rc;
    if (int rc = upload(c, c->d_adv_n, xn)) return rc;
    if (!c->d_adv_rank.ensure(4 * nx)) return c->fail(AD_E_NOMEM, "id ranks");
    if (!c->cu) c->cu = cfk_upd_work_create();
    CfkDevState d{c->d_status.as<uint8_t>(), c->d_xrank.as<uint32_t>(), c->d_ekey.as<uint32_t>(),
                  c->d_dict_lsb_raw.as<uint64_t>(), c->d_ballot.p ? c->d_ballot.as<Bal>() : nullptr,
                  c->dmiss_on ? c->d_mref.as<uint32_t>() : nullptr,
                  c->d_ent.as<uint2>(), c->d_krec.as<KeyRec>(), c->d_kent.as<KeyEntry>()};
    const CfkGrow grow{c, cfk_grow_dict, cfk_grow_entries, cfk_swap_entries, cfk_ballot_init, cfk_dict_spare, cfk_dict_swap,
                       c->d_rtxw.as<uint32_t>(), c->ds.n_rent, c->d_cell_ent.as<uint64_t>(), c->ds.cell_ent ? c->n_cell_ent : 0,
                       c->d_rb_wm.as<uint32_t>(), c->ds.n_rb, c->dmiss_on ? c->d_mids.as<uint32_t>() : nullptr,
                       c->dmiss_on ? c->dmiss_ids : 0, cfk_keys_spare, cfk_keys_swap,
                       c->d_kcell.p ? c->d_kcell.as<uint32_t>() : nullptr};
    // the host's per-entry copies are rebuilt from the device on demand after a merge (it remaps every rank): no
    // host remap of them here
    if (!c->host_moved)
    {
        c->host_moved = true;
        c->host_ingested = true;      // ranks change, entries do not: host missing() lists stay aligned
    }
    c->host_stale = true;
    CfkUpdOut o;
    std::string e;
    CfkDerivedBufs b{c->d_cand.as<uint32_t>(), c->d_cand.cap / 4, c->d_cwr.as<uint32_t>(), c->d_cwr.cap / 4,
                     c->d_w.as<uint2>(), c->d_w.cap / 8};
    const int rc = run_cfk_dict_ensure(c->cu, c->ds, d, c->d_adv_m.as<uint64_t>(), c->d_adv_l.as<uint64_t>(),
                                       c->d_adv_n.as<int32_t>(), nx, grow, &b, cfk_need_bufs, c, c->stream, &o,
                                       c->d_adv_rank.as<uint32_t>(), &e);
    if (const int frc = cfk_update_follow(c, o, rc, c->stream))
    {
        c->dirty = true;
        return frc;
    }
    if (rc)
    {
        c->dirty = true;        // rebuilt from the host copies at the next use
        return c->fail(rc, "id dictionary growth: %s", e.c_str());
    }
    HIPCHK(c, d2h(ranks->data(), c->d_adv_rank.p, 4 * nx, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    *n_new = o.n_new_ids;
    return 0;
}

int check_update_soa(ad_ctx* c, const ad_cfk_update_soa* u)
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

}  // namespace adi

extern "C" {

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

// ---- RedundantBefore advanced in place (SafeCommandStore.maybeTruncate on the next reads) ----
int ad_redundant_advance(ad_ctx* c, const ad_redundant_soa* in, ad_stats* stats)
{
    if (!c || !in) return AD_E_INVAL;
    auto& B = c->rb;
    const uint64_t n = in->n;
    if (n != B.start.size())
        return c->fail(AD_E_INVAL, "ad_redundant_advance: %llu entries, %llu loaded (a change of ranges is ad_redundant_load)",
                       (unsigned long long)n, (unsigned long long)B.start.size());
    if (n && (!in->range_start || !in->range_end || !in->start_epoch || !in->end_epoch || !in->wm_msb || !in->wm_lsb ||
              !in->wm_node))
        return c->fail(AD_E_INVAL, "ad_redundant_advance: null arrays");
    std::vector<uint64_t> moved;
    for (uint64_t i = 0; i < n; ++i)
    {
        if (in->range_start[i] != B.start[i] || in->range_end[i] != B.end[i])
            return c->fail(AD_E_INVAL, "ad_redundant_advance: entry %llu's range differs from the loaded one (a change of ranges "
                           "is ad_redundant_load)", (unsigned long long)i);
        const Tid t{in->wm_msb[i], in->wm_lsb[i], in->wm_node[i]};
        const int cmp = norm_cmp(norm(t), norm(B.wm[i]));
        if (cmp < 0)
            return c->fail(AD_E_INVAL, "ad_redundant_advance: entry %llu: expect the new shardAppliedOrInvalidatedBefore to be "
                           "ahead of the existing one (CommandsForKey.java:1319)", (unsigned long long)i);
        if (tid_gt_none(t) && (t.lsb & 1) == 0) return c->fail(AD_E_INVAL, "redundantBefore watermark must be range-domain");
        if (cmp > 0) moved.push_back(i);
    }
    if (stats) *stats = ad_stats{};
    for (uint64_t i = 0; i < n; ++i)
    {
        B.e0[i] = in->start_epoch[i];
        B.e1[i] = in->end_epoch[i];
        B.wm[i] = Tid{in->wm_msb[i], in->wm_lsb[i], in->wm_node[i]};
    }
    // before the first build the snapshot reads them (and truncates) when it is built
    if (!c->cfk.loaded || c->dirty) return AD_OK;
    if (hipSetDevice(c->device) != hipSuccess) return c->fail(AD_E_DEVICE, "hipSetDevice");
    StreamScope scope_(c->stream, c->cstream);
    const double t0 = now_ms();
    if (int rc = upload(c, c->d_rb_e0, B.e0)) return rc;
    if (int rc = upload(c, c->d_rb_e1, B.e1)) return rc;
    c->ds.rb_e0 = c->d_rb_e0.as<int64_t>();
    c->ds.rb_e1 = c->d_rb_e1.as<int64_t>();
    if (moved.empty())
    {
        HIPCHK(c, hipStreamSynchronize(c->stream));
        return AD_OK;
    }
    // the new watermarks join the id dictionary (appended or merged with the rank remap of an update
    // batch), their member ranks replace the moved entries' in rb_wm
    const uint64_t nx = moved.size();
    std::vector<Tid> ids(nx);
    for (uint64_t j = 0; j < nx; ++j) ids[j] = B.wm[moved[j]];
    std::vector<uint32_t> nr;
    uint64_t n_new = 0;
    if (int rc = dict_ensure_ids(c, ids, &nr, &n_new)) return rc;
    std::vector<uint32_t> wr(n);
    HIPCHK(c, d2h(wr.data(), c->d_rb_wm.p, 4 * n, c->stream));      // remapped by a merge
    HIPCHK(c, hipStreamSynchronize(c->stream));
    for (uint64_t j = 0; j < nx; ++j) wr[moved[j]] = nr[j];
    if (int rc2 = upload(c, c->d_rb_wm, wr)) return rc2;
    c->ds.rb_wm = c->d_rb_wm.as<uint32_t>();
    const double ms_dict = now_ms() - t0;
    c->ms_truncate = 0;
    c->n_truncated = 0;
    c->n_trunc_keys = 0;
    if (int rc2 = truncate_to_rb(c)) return rc2;
    if (stats)
    {
        stats->ms_device = c->ms_truncate;
        stats->ms_stage[0] = ms_dict;               // host-timed: watermark upload + dictionary growth
        stats->n_keys[0] = c->n_truncated;
        stats->n_keys[1] = c->n_trunc_keys;
        stats->n_keys[2] = n_new;
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

}  // extern "C"
