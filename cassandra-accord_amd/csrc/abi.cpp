// abi.cpp — C ABI of libaccord_deps.so, core: store context lifecycle, snapshot loads and ingest (id
// dictionary, ranks, per-key index arrays, range-entry table), SEQUENTIAL insertion and the batch pipeline
// driving the resolve kernels (ad_deps_batch, ad_deps_batch_device), dictionary views, invariant checks.
#include "abi_internal.hpp"

namespace adi {

// ---------------------------------------------------------------------------------------
// ingest
// ---------------------------------------------------------------------------------------
struct DictRec {
    uint64_t hi, lo;
    int32_t node;
    uint32_t pad;
    uint64_t src;
};

inline bool rec_less(const DictRec& a, const DictRec& b)
{
    if (a.hi != b.hi) return a.hi < b.hi;
    if (a.lo != b.lo) return a.lo < b.lo;
    return a.node < b.node;
}

inline bool rec_eq(const DictRec& a, const DictRec& b) { return a.hi == b.hi && a.lo == b.lo && a.node == b.node; }

bool tid_gt_none(const Tid& t)
{
    // compareTo(Timestamp.NONE) > 0, NONE = (0, 0, 0)
    const NormTid z = {0, 0, 0};
    return norm_cmp(norm(t), z) > 0;
}


int sync_host(ad_ctx* c);

// uninstall the node-wide dictionary (a new snapshot, or ids it does not hold)
void drop_global_dict(ad_ctx* c)
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
int kl_place_all(ad_ctx* c, const std::vector<int64_t>& keys, uint64_t nb, bool sparse)
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
void kl_members_ensure(ad_ctx* c)
{
    if (!c->kl_members.empty() || c->kl_keys_all.empty()) return;
    c->kl_members.assign(c->kl_nb_h, {});
    for (int64_t key : c->kl_keys_all) c->kl_members[kl_bucket(key_hash(key), c->kl_nb_h)].push_back(key);
    std::vector<int64_t>().swap(c->kl_keys_all);
}

// New keys into the perfect hash: a bucket keeps its displacement when its new keys land on free
// lines, else it is placed again (its old lines freed first); a bucket that does not fit, or a table
// above 70 % load, rebuilds the whole hash. Returns whether the table was rebuilt (size may change).
int kl_add_keys(ad_ctx* c, const std::vector<int64_t>& nkeys, uint64_t nk_total, bool* need_rebuild)
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

int build_ranges(ad_ctx* c, const std::vector<uint32_t>& cmd_rank, const std::vector<uint32_t>& wm_rank, RangePart* out)
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

// The range part's views (range entries, stabbing cells, range trees' levels, RedundantBefore)
int set_range_views(ad_ctx* c, const RangePart& rp, uint64_t nrb)
{
    DevSnapshot& s = c->ds;
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
    int L = 1;
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
    s.rng32 = getenv("AD_RNG64") == nullptr && c->rt_start.size() < (1ull << 26) && 2 * s.n_dict + 2 < (1ull << 26);
    return 0;
}

// The DevSnapshot views over the ctx's device buffers of a built snapshot (both build routes)
int set_views(ad_ctx* c, uint64_t n_dict, uint64_t n_samp, const NormTid& last, uint64_t nk, uint64_t ne, uint64_t hcap,
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
    if (int rc = set_range_views(c, rp, nrb)) return rc;
    s.n_slices = c->slice_s.size();
    s.slice_start = c->d_slices_s.as<int64_t>();
    s.slice_end = c->d_slices_e.as<int64_t>();
    s.n_ssets = c->ss_off.empty() ? 0 : c->ss_off.size() - 1;
    s.sset_off = c->d_ss_off.as<uint64_t>();
    s.sset_start = c->d_ss_start.as<int64_t>();
    s.sset_end = c->d_ss_end.as<int64_t>();
    s.start_inclusive = c->cfg.range_start_inclusive;
    s.elide = c->cfg.elide;
    s.rng32 = getenv("AD_RNG64") == nullptr && c->rt_start.size() < (1ull << 26) && 2 * n_dict + 2 < (1ull << 26);
    return 0;
}

// ---- the snapshot built on the device (ingest.hip + the update path's derivation) ----------------
int host_inputs(ad_ctx* c);

int build_snapshot_device(ad_ctx* c)
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

int build_snapshot_host(ad_ctx* c);

int build_snapshot(ad_ctx* c)
{
    // the device route takes a snapshot whose columns the load put in HBM, unless a node-wide
    // dictionary is installed (its ranks are the installed dictionary's: the host route)
    int rc;
    if (c->raw_dev && !c->gd_set)
        rc = build_snapshot_device(c);
    else if (!(rc = host_inputs(c)))
    {
        c->raw_dev = false;
        rc = build_snapshot_host(c);
    }
    // every read of a CommandsForKey truncates it to the store's RedundantBefore first: the snapshot
    // is read only as truncated
    return rc ? rc : truncate_to_rb(c);
}

const Tid* rb_wm_of(const ad_ctx* c, int64_t key)
{
    const auto& B = c->rb;
    const int incl = c->cfg.range_start_inclusive;
    size_t lo = 0, hi = B.start.size();
    while (lo < hi)
    {
        const size_t m = (lo + hi) >> 1;
        if (incl ? B.start[m] <= key : B.start[m] < key) lo = m + 1;
        else hi = m;
    }
    if (!lo || !range_contains(incl, B.start[lo - 1], B.end[lo - 1], key)) return nullptr;
    return tid_gt_none(B.wm[lo - 1]) ? &B.wm[lo - 1] : nullptr;
}

bool below_redundant(const ad_ctx* c, int64_t key, const Tid& t)
{
    const Tid* w = rb_wm_of(c, key);
    return w && norm_cmp(norm(t), norm(*w)) < 0;
}

int truncate_to_rb(ad_ctx* c)
{
    bool any = false;
    for (const Tid& t : c->rb.wm) any = any || tid_gt_none(t);
    if (!any || !c->ds.n_keys) return 0;
    auto& K = c->cfk;
    const uint64_t nk = c->ds.n_keys;
    // host-held missing() lists follow on the host (their ids need not be in the dictionary); the
    // device-held ones (dmiss_on) on the device
    const bool host_lists = !c->dmiss_on && !K.miss_off.empty() && !K.miss_stale;
    if (host_lists)
        if (int rc = sync_host(c)) return rc;          // K.seg and the lists index the device's entries
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
    CfkMiss miss;
    miss.on = c->dmiss_on;
    miss.n_lists = c->dmiss_lists;
    miss.off = c->d_moff.as<uint64_t>();
    miss.ids = c->d_mids.as<uint32_t>();
    miss.ctx = c;
    miss.spare = cfk_miss_spare;
    miss.swap = cfk_miss_swap;
    std::vector<uint32_t> pos(host_lists ? nk : 0);
    CfkTruncOut o;
    std::string e;
    const int rc = run_cfk_truncate(c->cu, c->ds, d, &b, cfk_need_bufs, c, grow, c->stream, &o, &e, &miss,
                                    host_lists ? pos.data() : nullptr);
    if (rc)
    {
        c->host_stale = true;
        c->dirty = true;
        return c->fail(rc, "RedundantBefore truncation: %s", e.c_str());
    }
    c->ms_truncate += o.ms_total;
    c->n_truncated += o.n_removed;
    c->n_trunc_keys += o.n_keys;
    if (!o.n_keys) return 0;
    if (c->kline_slots)
        HIPCHK(c, run_build_klines(c->ds, c->d_kslot.as<uint32_t>(), c->d_kcell.as<uint32_t>(), c->d_kline.as<KeyLine>(),
                                   c->kline_slots, c->stream));
    if (host_lists && o.n_removed)
    {
        // removeRedundantMissing on the kept entries of the keys that lost some (Utils.java:265-275)
        std::vector<uint64_t> off{0};
        std::vector<Tid> ids;
        ids.reserve(K.miss.size());
        for (uint64_t k = 0; k < nk; ++k)
        {
            const Tid* wm = pos[k] ? rb_wm_of(c, K.keys[k]) : nullptr;
            for (uint64_t x = K.seg[k] + pos[k]; x < K.seg[k + 1]; ++x)
            {
                for (uint64_t j = K.miss_off[x]; j < K.miss_off[x + 1]; ++j)
                    if (!wm || norm_cmp(norm(K.miss[j]), norm(*wm)) >= 0) ids.push_back(K.miss[j]);
                off.push_back(ids.size());
            }
        }
        K.miss_off.swap(off);
        K.miss.swap(ids);
    }
    // host copies follow from the device (entries moved, prunedBefore cleared); host lists were trimmed above
    c->host_moved = true;
    c->host_ingested = host_lists;
    c->host_stale = true;
    ++c->snap_gen;
    return 0;
}

int build_snapshot_host(ad_ctx* c)
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
int sync_host_entries(ad_ctx* c);

// TxnInfo.missing() lists maintained on the device -> the host copy (ids from their ranks)
int pull_missing(ad_ctx* c)
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
int host_dict(ad_ctx* c)
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
int host_inputs(ad_ctx* c)
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

int sync_host(ad_ctx* c)
{
    if (int rc = host_dict(c)) return rc;
    if (int rc = host_inputs(c)) return rc;
    if (!c->host_stale) return 0;
    if (int rc = sync_host_entries(c)) return rc;
    return c->dmiss_on ? pull_missing(c) : 0;
}

int sync_host_entries(ad_ctx* c)
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

// ---------------------------------------------------------------------------------------
// batch pipeline
// ---------------------------------------------------------------------------------------

// A small upload (at most UP_WORDS words) ordered on st without a host wait: copied into the context's
// pinned slot `k`, whose previous copy has completed first (its event; normally long done). A pageable
// h2d would return only after the copy -- after everything queued before it on st.

hipError_t up_small(ad_ctx* c, int k, void* dst, const void* src, size_t bytes, hipStream_t st)
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
uint64_t* rb_slot(ad_ctx* c)
{
    if (!c->h_rb && hipHostMalloc((void**)&c->h_rb, sizeof(uint64_t) * UP_WORDS, hipHostMallocDefault) != hipSuccess)
        c->h_rb = nullptr;
    return c->h_rb;
}

// bind the split kernels' per-batch arrays for a batch of n requests / np probes
bool bind_split(ad_ctx::SplitBufs& S, BatchBufs& b, uint64_t n, uint64_t np, bool own_sizes)
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

int run_split(ad_ctx* c, const BatchBufs& b, hipStream_t st)
{
    HIPCHK(c, run_encode(c->ds, b, st));
    HIPCHK(c, run_scan(c->ds, b, st));
    HIPCHK(c, run_range(c->ds, b, st));
    HIPCHK(c, run_build(c->ds, b, st));
    return 0;
}

// requests per wave of lean pass 1 by the batch's keys per request (lean_rpw1): four up to 4.5 keys on
// average, else two; AD_LEAN_RPW overrides (tests: every width on any batch; 8 measured no faster on a
// store's share of requests spanning many stores).

uint32_t lean_rpw1(uint64_t n, uint64_t np)
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

bool lean_wide1(const ad_ctx* c)
{
    if (const char* e = getenv("AD_LEAN_WIDE1")) return atoi(e) != 0;
    return c->lean_wide;
}

void lean_wide1_update(ad_ctx* c, uint64_t n, const BatchCtl& h)
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
hipError_t batch_wait(ad_ctx* c, hipStream_t st)
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

int run_pipeline(ad_ctx* c, const ad_query_soa* q, hipStream_t st, ad_deps_result* out, bool parts_only,
                        bool n_keys_given, int recovery_scan, const RecoveryView* rv)
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
        HIPCHK(c, run_range_count(c->ds, n, q->key_off, q->range_off, q->range_start, q->range_end, q->slice_set,
                                  c->rq_cnt.as<uint32_t>(), c->rq_err.as<uint32_t>(), c->rq_list.as<uint32_t>(), nr,
                                  recovery_scan < 0, st));
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
        HIPCHK(c, run_range_fill(c->ds, n, q->key_off, q->keys, q->range_off, q->range_start, q->range_end, q->slice_set,
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
    b.q_slice_set = q->slice_set;
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
    }
    if (const char* e = getenv("AD_K2_BIG")) b.k2_big = (uint32_t)strtoul(e, nullptr, 10);   // tests: force k_build_big
    b.kb_sort = 16384;                                                                           // KB_LDS_CAP
    if (const char* e = getenv("AD_KB_SORT")) b.kb_sort = (uint32_t)strtoul(e, nullptr, 10);   // tests: 0 = global scratch
    b.kb_merge = 1;
    if (const char* e = getenv("AD_KB_MERGE")) b.kb_merge = (uint32_t)strtoul(e, nullptr, 10);
    // the pack copy spread over the whole output when the batch has too few requests to fill the chip with
    // k_pack_tiles's wave per 64 requests (tests: AD_PACK_EVEN=0/1 forces either)
    b.pack_even = n <= 131072;
    if (const char* e = getenv("AD_PACK_EVEN")) b.pack_even = strtoul(e, nullptr, 10) != 0;
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
                // the general fused kernel on what both lean passes deferred (routing them to the split kernels
                // instead measured 1.94 ms for the request mix against 0.98)
                BatchBufs b2 = b;
                b2.req_list = b.deferred2;
                b2.req_count = &b.ctl->n_deferred2;
                HIPCHK(c, run_resolve(c->ds, b2, st));
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
                    (b.q_slice_set && !ens<uint32_t>(c->s_ss, nd)) ||
                    (b.p_kind && (!ens<int64_t>(c->s_khi, snp) || !ens<uint8_t>(c->s_kind, snp))))
                    return c->fail(AD_E_NOMEM, "deferred buffers");
                uint64_t* sko = c->s_ko.as<uint64_t>();     // the scanned counts are the sub-batch key_off
                HIPCHK(c, run_defer_gather(b, b.deferred, nd, c->s_ko.as<uint64_t>(), sb, c->s_tm.as<uint64_t>(),
                                           c->s_tl.as<uint64_t>(), c->s_tn.as<int32_t>(), c->s_em.as<uint64_t>(),
                                           c->s_el.as<uint64_t>(), c->s_en.as<int32_t>(), c->s_me.as<int64_t>(), sko,
                                           c->s_k.as<int64_t>(), b.p_kind ? c->s_khi.as<int64_t>() : nullptr,
                                           b.p_kind ? c->s_kind.as<uint8_t>() : nullptr,
                                           b.q_slice_set ? c->s_ss.as<uint32_t>() : nullptr, st));
                sb.q_txn_msb = c->s_tm.as<uint64_t>(); sb.q_txn_lsb = c->s_tl.as<uint64_t>(); sb.q_txn_node = c->s_tn.as<int32_t>();
                sb.q_exec_msb = c->s_em.as<uint64_t>(); sb.q_exec_lsb = c->s_el.as<uint64_t>(); sb.q_exec_node = c->s_en.as<int32_t>();
                sb.q_min_epoch = b.q_min_epoch ? c->s_me.as<int64_t>() : nullptr;
                sb.q_slice_set = b.q_slice_set ? c->s_ss.as<uint32_t>() : nullptr;
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
            if (h.error == ERR_SLICE)
                return c->fail(AD_E_INVAL, "a request's slice_set is beyond the store's slice sets (ad_slice_sets_load)");
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


// A library-owned host result array (released by free() in ad_result_free). Large ones are 2 MB aligned
// and advised as transparent huge pages: the copy-out then first-touches a few hundred pages instead of
// ~90k 4 KB ones per config-2 batch (the page faults were most of ad_deps_batch's host time).
void* host_result_alloc(size_t bytes)
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
int d2h_result(ad_ctx* c, T** out, const T* src, uint64_t n, uint64_t bound, const char* what, int m)
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
int result_to_host(ad_ctx* c, uint64_t n, const ad_deps_result& dev, ad_deps_result** out)
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
                if (int rc = d2h_result(c, offs[a], src_off[a], n + 1, n + 1, names[a], m)) return rc;
                const uint64_t* o = *offs[a];
                if (o[0] != 0 || o[n] != tot[a])
                    return c->fail(AD_E_DEVICE, "result offsets of %s, map %d: [0] = %llu, [n] = %llu, batch total %llu", names[a],
                                   m, (unsigned long long)o[0], (unsigned long long)o[n], (unsigned long long)tot[a]);
            }
            if (int rc = d2h_result(c, &r->keys[m], dev.keys[m], tot[0], tot[0], names[0], m)) return rc;
            if (int rc = d2h_result(c, &r->txns[m], dev.txns[m], tot[1], tot[1], names[1], m)) return rc;
            if (int rc = d2h_result(c, &r->k2t[m], dev.k2t[m], tot[2], tot[2], names[2], m)) return rc;
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

int check_query_host(ad_ctx* c, const ad_query_soa* q, uint32_t flags)
{
    if (q->slice_set)
    {
        const uint64_t ns = c->ss_off.empty() ? 0 : c->ss_off.size() - 1;
        for (uint64_t i = 0; i < q->n_txns; ++i)
            if (q->slice_set[i] != AD_SLICE_STORE && q->slice_set[i] >= ns)
                return c->fail(AD_E_INVAL, "request %llu: slice_set %u beyond the store's %llu slice sets",
                               (unsigned long long)i, q->slice_set[i], (unsigned long long)ns);
    }
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
