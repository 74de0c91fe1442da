// abi_levels.cpp — PreAccept timestamp proposal (ad_preaccept_*) and execution levels (§8 a12, ad_levels*).
#include "abi_internal.hpp"

namespace adi {

int load_range_map(ad_ctx* c, const ad_range_map_soa* m, ad_ctx::RangeMapBufs& B, const char* what)
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

DevRangeMap dev_range_map(ad_ctx::RangeMapBufs& B)
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

}  // namespace adi

extern "C" {

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

}  // extern "C"

namespace adi {

int levels_run(ad_ctx* c, const LevelsIn& in, uint32_t* out_dev, hipStream_t st, ad_stats* stats)
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

}  // namespace adi

extern "C" {

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

}  // extern "C"
