// abi_exchange.cpp — multi-GPU exchange (SURVEY §8 e, a10; f2): node dictionary, parts export, K3 merge / union, the
// exchange plan and its two transports (ad_exchange_local, ad_exchange over RCCL).
#include "abi_internal.hpp"

extern "C" {

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

namespace adi {

// Export, phase 1 (ad_parts_export, ad_exchange, ad_exchange_local): validate, bind the export
// arguments and enqueue the size pass; c->x_cnt then holds the cumulative [n_dest + 1][4] bounds
// {parts, key words, ids, k2t} of the destinations. Nothing is read back.
int export_sizes(ad_ctx* c, const ad_deps_result* res, const int64_t* txn_index, uint32_t n_dest,
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
int export_emit(ad_ctx* c, ExportArgs& a, int64_t* hdr, int64_t* keys, int64_t* ids, int32_t* k2t, hipStream_t st)
{
    a.hdr = hdr; a.okeys = keys; a.oids = ids; a.ok2t = k2t;
    HIPCHK(c, run_export_emit(a, st));
    return AD_OK;
}

}  // namespace adi

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

}  // extern "C"

namespace adi {

// The end of a merge once its kernels and read-backs are queued: one synchronisation, then the result's
// views (parts_merge with a MergeTail returns before it, so that ad_exchange_local's owners merge at once)
struct MergeTail {
    hipStream_t st;
    MergeArgs a;
    bool by_request, rank_ids;
    uint64_t n_owned, txn_base;
};

int merge_malformed(ad_ctx* c, uint32_t e)
{
    return c->fail(AD_E_INVAL, "ad_parts_merge: malformed parts (%s)",
                   e & 1  ? "request outside the owned range or bad map" :
                   e & 2  ? "two parts of one request and map from one source" :
                   e & 4  ? "keys of different stores overlap or are out of slice order" :
                   e & 16 ? "id rank outside the global dictionary" :
                            "ids of a part not sorted and unique");
}

int merge_tail(ad_ctx* c, const MergeTail& t, ad_merged* out)
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

int parts_merge(ad_ctx* c, const ad_parts* in, uint32_t n_src, const uint64_t* src_parts, uint64_t txn_base,
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

}  // namespace adi

extern "C" {

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

// =======================================================================================
// Node exchange (SURVEY §8 e): the per-store PartialDeps of a node batch combined
// on the store that owns each request -- CommandStores.mapReduce's reduce (CommandStores.java:576-593)
// with PartialDeps.with (PreAccept.reduce, PreAccept.java:140-156) -- as export -> move -> K3 merge.
// Two transports of one protocol: device copies between the contexts of one process
// (ad_exchange_local: the Java host's one process per node, hipMemcpyPeerAsync over xGMI between
// GPUs) and RCCL grouped send/recv between processes (ad_exchange).
// =======================================================================================

}  // extern "C"

namespace adi {

constexpr int XA = 4;                                  // hdr, keys, ids, k2t

size_t x_unit_bytes(int a, uint32_t fmt)       // bytes per counted unit of array a
{
    switch (a)
    {
        case 0: return 32;                             // 4 int64 per part
        case 1: return 8;                              // key words
        case 2: return fmt == AD_IDS_RANK ? 4 : 24;    // ids
        default: return 4;                             // k2t
    }
}

DevBuf* x_send(ad_ctx* c, int a) { DevBuf* b[XA] = {&c->xs_hdr, &c->xs_keys, &c->xs_ids, &c->xs_k2t}; return b[a]; }

DevBuf* x_recv(ad_ctx* c, int a) { DevBuf* b[XA] = {&c->xr_hdr, &c->xr_keys, &c->xr_ids, &c->xr_k2t}; return b[a]; }

uint32_t x_format(const ad_ctx* c) { return c->global_ok ? AD_IDS_RANK : AD_IDS_TRIPLET; }

// The plan of `R` from an agreed exchange table (layout: accord_deps.h, ad_exchange_plan). Every rank
// runs it on the same table, so every verdict -- failure, id formats, growth round -- is collective.
// bad: the rank whose row failed a check (-1: none).
int x_plan(const uint64_t* table, uint32_t W, uint32_t R, ad_xfer* xf, uint64_t* recv_units, uint64_t* src_parts,
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
XRowHdr x_row_hdr(ad_ctx* c, uint32_t fmt, int status)
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
int x_grow(ad_ctx* c, const uint64_t* send_units, const uint64_t* recv_units, uint32_t fmt)
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
void x_keep_self(ad_ctx* c, ExportArgs& a, const ad_xfer* xf, uint32_t W, uint32_t self, uint64_t lo, uint64_t hi,
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

int x_emit(ad_ctx* c, ExportArgs& a, hipStream_t st)
{
    return export_emit(c, a, c->xs_hdr.as<int64_t>(), c->xs_keys.as<int64_t>(), c->xs_ids.as<int64_t>(),
                       c->xs_k2t.as<int32_t>(), st);
}

// K3 on c over its receive buffers: sources in slice (= rank / context) order
int x_merge(ad_ctx* c, uint32_t n_src, const uint64_t* src_parts, const uint64_t* recv_units, uint32_t fmt,
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
int x_abort(ad_ctx* c, int code)
{
    if (c->comm) (void)ncclCommAbort(c->comm);
    c->comm = nullptr;
    return code;
}

int nccl_fail(ad_ctx* c, ncclResult_t r, const char* what)
{
    return c->fail(AD_E_DEVICE, "%s: %s", what, ncclGetErrorString(r));
}

#define NCCLCHK(ctx, expr)                                                                         \
    do {                                                                                           \
        ncclResult_t _r = (expr);                                                                  \
        if (_r != ncclSuccess) return nccl_fail((ctx), _r, #expr);                                 \
    } while (0)

float ev_ms(hipEvent_t a, hipEvent_t b)
{
    float ms = 0;
    return hipEventElapsedTime(&ms, a, b) == hipSuccess ? ms : 0.f;
}

}  // namespace adi

extern "C" {

int ad_exchange_plan(const uint64_t* table, uint32_t world, uint32_t rank, ad_xfer* xfers, uint64_t* recv_units,
                     uint64_t* src_parts, uint32_t* flags)
{
    if (!table || world == 0 || rank >= world || !xfers || !recv_units || !src_parts || !flags) return AD_E_INVAL;
    int bad = -1;
    return x_plan(table, world, rank, xfers, recv_units, src_parts, flags, &bad);
}

}  // extern "C"

namespace adi {

int exchange_local_run(ad_ctx* const* ctxs, uint32_t n, const ad_deps_result* const* res, const int64_t* const* txn_index,
                              const uint64_t* const* dest_first, const uint64_t* txn_base, const uint64_t* n_owned,
                              ad_merged* out, ad_exchange_stats* stats);

}  // namespace adi

extern "C" {

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

}  // extern "C"

namespace adi {

int exchange_local_run(ad_ctx* const* ctxs, uint32_t n, const ad_deps_result* const* res, const int64_t* const* txn_index,
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
    // on a failure, every owner whose merge was queued is drained before returning (no kernel or pinned
    // read-back left in flight behind the caller); its out[] entry is then unset
    auto drain = [&](int rc) {
        for (uint32_t e = 0; e < n; ++e)
            if (hipSetDevice(ctxs[e]->device) == hipSuccess) (void)hipStreamSynchronize(ctxs[e]->stream);
        return rc;
    };
    for (uint32_t d = 0; d < n; ++d)
    {
        ad_ctx* o = ctxs[d];
        if (hipSetDevice(o->device) != hipSuccess) return drain(o->fail(AD_E_DEVICE, "hipSetDevice"));
        if (int rc = x_merge(o, n, src_parts[d].data(), runits[d].data(), fmt, txn_base[d], n_owned[d], o->stream, &out[d],
                             &tails[d]))
            return drain(rc);
        if (!distinct)
        {
            if (int rc = merge_tail(o, tails[d], &out[d])) return drain(rc);
            ms_merge += out[d].ms_device;
        }
    }
    for (uint32_t d = 0; d < n && distinct; ++d)
    {
        if (int rc = merge_tail(ctxs[d], tails[d], &out[d])) return drain(rc);
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

}  // namespace adi

extern "C" {

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

}  // extern "C"
