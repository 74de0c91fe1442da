// abi_recovery.cpp — recovery scans: the RecoveryView of a live store and ad_recovery_batch*.
#include "abi_internal.hpp"

namespace adi {

// device view of the snapshot for mapReduceFull: entries in load order with executeAt ranks,
// status, kind and their TxnInfo.missing() lists as ranks (built once per snapshot / missing load)
// The live range commands of the view: per range entry of the snapshot its command, the commands'
// recovery facts normalised. Host-built from the loaded commands; rebuilt when ranks change.
int build_rv_ranges(ad_ctx* c, bool live_cmds)
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
int build_recovery_view_device(ad_ctx* c)
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

int build_recovery_view(ad_ctx* c, RecoveryView* v)
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

}  // namespace adi

extern "C" {

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
    d.slice_set = stage_q(c, c->q_ss, q->slice_set, n, &rc);
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

}  // extern "C"
