// abi_snapshot.cpp — the store snapshot of libaccord_deps: the KeyLine perfect hash, the range-entry table and
// stabbing index, the snapshot build (device ingest and host route), RedundantBefore truncation at build time, and
// the host copies of the device state (pulled on demand).
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

// The first sample level's bucket index (common.hpp dict_bucket_of), rebuilt whenever the samples are: about one
// sample per bucket (2^lg >= n_samp, at most 2^22). Without its buffer the searches run over all the samples.
int build_dict_buckets(ad_ctx* c, hipStream_t st)
{
    DevSnapshot& s = c->ds;
    s.ds_bkt = nullptr;
    if (!s.n_samp || !s.ds_hi) return 0;
    uint32_t lg = 0;
    while ((1ull << lg) < s.n_samp && lg < 22) ++lg;
    if (!c->d_ds_bkt.ensure(4 * (DB_HDR + (1ull << lg) + 1))) return 0;
    HIPCHK(c, run_dict_buckets(s, c->d_ds_bkt.as<uint32_t>(), lg, st));
    s.ds_bkt = c->d_ds_bkt.as<uint32_t>();
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
    if ((rc = build_dict_buckets(c, st))) return rc;
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
        if (int rc2 = build_dict_buckets(c, c->stream)) return rc2;
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

}  // namespace adi
