// abi_into.cpp — ad_deps_batch_into: the PCIe-facing batch path into caller-owned (pinned) host arrays.
#include "abi_internal.hpp"

namespace adi {

// ---- ad_deps_batch_into, key-only SNAPSHOT batches: inputs packed by the host worker pool into pinned
// staging (one H2D per slice, the next slice packed while this one resolves; the key-order check is the
// same pass), results copied by a kernel straight into the caller's pinned arrays (CU stores over PCIe run
// beside the SDMA H2D: both directions at once), offsets of maps empty in a slice filled by the pool at
// the end. Pageable output arrays fall back to staged copies.

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

int deps_into_fast(ad_ctx* c, const ad_query_soa* q, ad_deps_result* out, const uint64_t* cap, uint64_t* need,
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

}  // namespace adi

extern "C" {

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
    // (batches naming slice sets take the staged path: its per-array copies carry slice_set)
    const bool fast = !(flags & AD_SEQUENTIAL) && !(n && q->range_off && q->range_off[n] > q->range_off[0]) && !q->slice_set;
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
        d.slice_set = q->slice_set ? stage_q(c, c->q_ss, q->slice_set + lo, nc, &rc) : nullptr;
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

}  // extern "C"
