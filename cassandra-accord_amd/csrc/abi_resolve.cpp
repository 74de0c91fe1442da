// abi_resolve.cpp — the batch pipeline of libaccord_deps: request staging, the lean / general / split resolve
// kernels chosen per batch, the pack or regions output, and the host copies of a result.
#include "abi_internal.hpp"

namespace adi {

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
    if (lean)
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


}  // namespace adi
