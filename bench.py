#!/usr/bin/env python3
"""Benchmark of the MI355X dependency-resolution hot path (BASELINE.json metric:
"deps resolved: txn-key pairs/sec + HBM GB/s %peak at 1/2/4/8 MI355X").

One step = one batch of PreAccept.calculatePartialDeps requests resolved on the GPU(s), with
the requests already resident in HBM when the timed region starts and the PartialDeps CSR
(keyDeps / rangeDeps / directKeyDeps) left in HBM:
  K0 encode -> K1 CommandsForKey conflict scan -> K4 range probe -> K2 build (size pass,
  offsets, emit pass)  [+ for N > 1: all-to-all of per-store partials over RCCL and K3 merge]

Workload: config 2 of BASELINE.json (1M txns x 8 Zipf(0.99) keys over 1M keys, 16M-entry
CommandsForKey history, SNAPSHOT). For N > 1 the same per-GPU shape is scaled weakly (see
DESIGN.md §6). Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "cassandra-accord_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402  (loads the HIP runtime first; see accord_deps.native.lib)

from accord_deps import _abi as A  # noqa: E402
import torch.distributed as dist  # noqa: E402

from accord_deps import exchange, native, synth  # noqa: E402

METRIC = "deps resolved: txn-key pairs/sec + HBM GB/s %peak at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E peak, /opt/skills/guides/MI355X_MICROARCH.md
STAGES = ["lean resolve pass 1", "deferred requests (split K0..K2)", "prepare (request records: S / self ranks; probe KeyLines for the lean passes)",
          "lean resolve pass 2 (2 requests/wave, 2 emissions/lane)", "offsets scan", "offsets + pack (tile sums, tile scan, scan+pack)",
          "general fused resolve (lean deferrals)"]
# K1 + K2 of every request run in these stages / kernels: the roofline's "dominant kernel"
# (k_prepare included since it also resolves every probe's KeyLine for the lean passes)
RESOLVE_STAGES = [0, 2, 3, 6]
# the committed profiles the roofline's counter traffic may come from: this round's only (a profile of an older
# tree may name kernels that no longer run the same way)
PROFILE_ROUND = "r6"


def resolve_kernels(stats, split_ms, min_ms=0.02):
    """Names (as rocprofv3 reports them, namespace and arguments stripped) of the kernels that ran the resolve
    stages of this batch, from what the library reports it launched (ad_stats.lean_rpw1 / lean_flags; abi.cpp
    run_pipeline -> lean.hip run_resolve_lean, resolve.hip run_prepare): never re-derived from the workload's
    shape. Stages that took under min_ms (e.g. an empty pass 2) are left out."""
    rpw1 = int(stats.get("lean_rpw1", 0))
    fl = int(stats.get("lean_flags", 0))
    rng = bool(fl & A.AD_LEAN_RANGES)
    names = []
    if split_ms[2] > min_ms:
        names.append("k_prepare<true>" if rpw1 else "k_prepare<false>")     # the lean passes read its probe KeyLines
    if rpw1:
        wide = bool(fl & A.AD_LEAN_WIDE1)
        names.append("k_resolve_lean<%du, %s, %s, 1>" % (rpw1, "true" if rng else "false", "true" if wide else "false"))
        if fl & A.AD_LEAN_PASS2 and split_ms[3] > min_ms:
            if rng:
                names.append("k_resolve_lean<2u, true, false, 2>" if rpw1 == 4 else "k_resolve_lean<1u, true, false, 2>")
            else:
                names.append("k_resolve_lean<2u, false, true, 2>")
        if split_ms[6] > min_ms:
            names.append("k_resolve")
    elif split_ms[0] > min_ms:
        names.append("k_resolve")
    return names


# device of the small timing / count reductions: the GPU under RCCL, the host under gloo
RED_DEV = None


def _red_dev(dev):
    return RED_DEV if RED_DEV is not None else dev


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def measured_traffic(kernels, tag=None):
    """HBM bytes per launch summed over `kernels` from the newest committed PMC summary of this round
    (profiles/<PROFILE_ROUND>*_pmc.json, by name) that holds every one of them (FETCH_SIZE doubled for gfx950 as
    MI355X_MICROARCH.md prescribes, + WRITE_SIZE; scripts/summarize_prof.py). With `tag`, only summaries whose name
    holds it (the profile of the same workload: "config2", "config4", "mix"). Without such a profile: (None, a
    note naming what is missing) and a warning on stderr -- never an older round's profile of other kernels."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", PROFILE_ROUND + "*_pmc.json")))
    if tag is not None:
        files = [f for f in files if tag in os.path.basename(f)]
    for f in reversed(files):
        with open(f) as fh:
            d = json.load(fh)
        if all(k in d and d[k].get("fetch_bytes_per_launch") is not None for k in kernels):
            tot = sum(2 * d[k]["fetch_bytes_per_launch"] + (d[k].get("write_bytes_per_launch") or 0) for k in kernels)
            return tot, os.path.relpath(f, ROOT)
    note = "missing: no %s profile%s holds %s" % (PROFILE_ROUND, " of " + tag if tag else "", " + ".join(kernels))
    log("WARNING: roofline traffic unmeasured (%s)" % note)
    return None, note


def measured_traffic_per_step(kernels, tag, unit_kernel):
    """HBM bytes per step of a stage made of several kernels launched different numbers of times per
    step (K5's build: radix passes, chain walks, scans): each kernel's per-launch bytes from the newest
    committed PMC summary whose name holds `tag`, weighted by its launches per `unit_kernel` launch in
    the same profile's kernel-stats CSV. Kernels absent from the profile count 0. (None, None) without
    such a profile."""
    import csv
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "%s*%s*_pmc.json" % (PROFILE_ROUND, tag))))
    for f in reversed(files):
        stats = f[:-len("_pmc.json")] + "_kernel_stats.csv"
        if not os.path.exists(stats):
            continue
        calls = {}
        with open(stats) as fh:
            for row in csv.DictReader(fh):
                name = row.get("Name") or row.get("KernelName") or ""
                short = name.split("(")[0].replace("void ", "").replace("adx::", "").replace("(anonymous namespace)::", "")
                calls[short] = calls.get(short, 0) + int(float(row.get("Calls") or 0))
        if not calls.get(unit_kernel):
            continue
        with open(f) as fh:
            d = json.load(fh)
        tot = 0.0
        for k in kernels:
            if k in d and d[k].get("fetch_bytes_per_launch") is not None and calls.get(k):
                per = 2 * d[k]["fetch_bytes_per_launch"] + (d[k].get("write_bytes_per_launch") or 0)
                tot += per * calls[k] / calls[unit_kernel]
        return tot, os.path.relpath(f, ROOT)
    note = "missing: no %s profile of %s" % (PROFILE_ROUND, tag)
    log("WARNING: roofline traffic unmeasured (%s)" % note)
    return None, note


def stage_bytes(w, stats):
    """Algorithmic bytes per pipeline stage and launch.
    Fused resolve: request inputs (txnId + executeAt 40 B, key_off 8 B, 8 B per key) + the
    SURVEY.md §8(d) config-2 compulsory CommandsForKey read (every touched key's segment once,
    17 B per entry + 16 B header) + the range-command table once (16 B per entry) + the CSR
    output written to its region (8 B per key/range head, 4 B per keysToTxnIds int, 4 B per
    txnId index) + 9 x 4 B sizes and 3 x 8 B region offsets per request.
    Pack: reads and writes the CSR output once more."""
    q = w.queries
    keys_touched = np.unique(q.keys)
    pos = np.searchsorted(w.cfk.keys, keys_touched)
    ok = pos < len(w.cfk.keys)
    pos = pos[ok]
    pos = pos[w.cfk.keys[pos] == keys_touched[ok]]
    seg = w.cfk.seg.astype(np.int64)
    lk = seg[pos + 1] - seg[pos]
    pairs = sum(stats["n_pairs"])
    heads = sum(stats["n_keys"])
    uniq = sum(stats["n_unique"])
    out_bytes = 8 * heads + 4 * (heads + pairs) + 4 * uniq
    b = [0] * 7
    b[0] = len(q) * (40 + 8) + 8 * q.n_probes + int((17 * lk + 16).sum()) + 16 * int(w.cmds.range_off[-1]) + \
        out_bytes + len(q) * (9 * 4 + 3 * 8)
    b[2] = len(q) * (56 + 16) + q.n_probes * (8 + 16 + 4)   # request ids + key_off, record; keys, KeySlot, slot
    b[4] = 9 * (4 + 8) * len(q)
    b[5] = 2 * out_bytes + len(q) * (9 * (4 + 8) + 3 * 8)
    return b


def cpu_info():
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return os.cpu_count(), model


def cpu_threads():
    """Host threads the CPU baseline may use: the box's CPU share (OMP_NUM_THREADS is set to it on
    the GPU box), at most os.cpu_count()."""
    n = os.cpu_count() or 1
    try:
        n = min(n, int(os.environ.get("OMP_NUM_THREADS", n)))
    except ValueError:
        pass
    return max(1, n)


def cpu_baseline_stores(w, budget_s=15.0, threads=None, gpu_take=None):
    """The reference's own concurrency model on the host cores: the store's key space split into
    `threads` EvenSplit token slices (ShardDistributor.EvenSplit, ShardDistributor.java:106-156), one
    CommandStore each on its own thread (InMemoryCommandStore's single-thread executors,
    :1144-1202), every store resolving its share of a prefix of the same batch with the CPU
    restatement (oracle/refcpu.c), then the per-store PartialDeps reduced request-wise with
    PartialDeps.with (CommandStores.mapReduce :576-593, rc_result_merge). Timed: the parallel
    resolve + the reduce; median of 5 runs of a prefix sized to ~budget/5 s each. The merged result
    of the prefix is compared bit-exactly with the GPU's (`gpu_take(idx)` -> PartialDepsBatch)."""
    import ctypes as C
    import threading
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    threads = threads or cpu_threads()
    L = pyoracle.lib()
    base = w
    if w.slices is not None and len(w.slices) == 1 and int(w.slices[0][0]) == -(1 << 63) and \
            int(w.slices[0][1]) == (1 << 63) - 1:
        from accord_deps.model import Workload
        base = Workload(w.name, w.cfk, w.cmds, w.redundant, w.queries, w.flags, w.params, w.range_start_inclusive, None)
    lo, hi = synth.shard_bounds(threads)
    subs = [synth.slice_workload(base, lo[g], hi[g]) for g in range(threads)] if threads > 1 else [base]
    stores = [pyoracle.OracleStore(s.range_start_inclusive, 1, s.slices).load(s) for s in subs]
    soas = [s.queries.soa() for s in subs]

    def run(count):
        outs = [C.POINTER(pyoracle.RcResult)() for _ in stores]
        rcs = [0] * len(stores)

        def one(g):
            rcs[g] = L.rc_deps_batch(stores[g].h, C.byref(soas[g]), base.flags, 0, count, C.byref(outs[g]))
        t0 = time.perf_counter()
        ts = [threading.Thread(target=one, args=(g,)) for g in range(len(stores))]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        merged = C.POINTER(pyoracle.RcResult)()
        arr = (C.POINTER(pyoracle.RcResult) * len(outs))(*outs)
        rc = L.rc_result_merge(arr, len(outs), C.byref(merged)) if len(outs) > 1 else 0
        dt = time.perf_counter() - t0
        if any(rcs) or rc:
            raise RuntimeError("refcpu failed: %r %r" % (rcs, rc))
        res = merged if len(outs) > 1 else outs[0]
        batch = pyoracle.result_to_batch(res.contents)
        for o in outs:
            L.rc_result_free(o)
        if len(outs) > 1:
            L.rc_result_free(merged)
        return dt, batch

    n = len(base.queries)
    p = min(n, 256)
    dt, _ = run(p)
    p = int(min(n, max(p, p * (budget_s / 5.0) / max(dt, 1e-6))))
    times, batch = [], None
    for _ in range(5):
        dt, batch = run(p)
        times.append(dt)
    for s in stores:
        s.close()
    t = float(np.median(times))
    pairs = int(base.queries.key_off[p])
    ncpu, model = cpu_info()
    out = dict(value=pairs / t, unit="txn-key pairs/s", cores=threads, kind="port",
               sample="first %d of %d requests of the same batch (%d txn-key pairs), median of 5 runs (%s s); "
                      "refcpu = C restatement of the reference Java, %d CommandStores (EvenSplit token slices) on %d "
                      "threads + PartialDeps.with reduce; host %d CPUs, %s" %
                      (p, n, pairs, "/".join("%.2f" % x for x in times), threads, threads, ncpu, model))
    if gpu_take is not None:
        got = gpu_take(np.arange(p))
        ok, why = got.equals(batch, detail=True)
        out["parity_sample"] = "%d requests bit-exact vs GPU" % p if ok else "MISMATCH: %s" % why
    return out


def cpu_baseline(w, budget_s=15.0):
    """The CPU restatement (oracle/refcpu.c, the reference algorithm, one thread = one
    CommandStore) on a bounded prefix of the same batch, same snapshot."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    st = pyoracle.OracleStore(w.range_start_inclusive, 1, w.slices)
    st.load(w)
    n = 16
    t = 0.0
    done_pairs = 0
    first = 0
    total = len(w.queries)
    while first < total:
        cnt = min(n, total - first)
        t0 = time.perf_counter()
        st.deps_batch(w.queries, w.flags, first, cnt)
        dt = time.perf_counter() - t0
        t += dt
        done_pairs += int(w.queries.key_off[first + cnt] - w.queries.key_off[first])
        first += cnt
        if t >= budget_s:
            break
        n = max(1, min(int(n * 2), int(cnt * max(0.1, (budget_s - t) / max(dt, 1e-6)))))
    st.close()
    return dict(value=done_pairs / t, unit="txn-key pairs/s", cores=1, kind="port",
                sample="first %d of %d requests of the same batch (%d txn-key pairs, %.1f s), refcpu = C "
                       "restatement of the reference Java, 1 thread = 1 CommandStore" % (first, total, done_pairs, t))


def cpu_baseline_levels(g, budget_s=15.0):
    """The CPU restatement of the levels computation (oracle rc_levels: executeAt order, per-key
    predecessor walk, 1 thread) on the whole graph, repeated while within budget."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    t = 0.0
    reps = 0
    while reps == 0 or t < budget_s / 4:
        t0 = time.perf_counter()
        pyoracle.levels(g)
        t += time.perf_counter() - t0
        reps += 1
    pairs = int(g.key_off[-1]) * reps
    return dict(value=pairs / t, unit="txn-key pairs/s", cores=1, kind="port",
                sample="whole config-5 graph x%d (%d txns, %d txn-key pairs each, %.1f s), refcpu rc_levels = C "
                       "restatement, 1 thread" % (reps, len(g.kind), int(g.key_off[-1]), t))


def bench_levels(args, rank, world, local, dev):
    """Config 5: execution ordering of a 1M-txn waitingOn graph -> apply levels (K5). Not sharded
    (a txn's keys span stores and levels chain across them): with N GPUs every rank levels its own
    replica of the graph ("replicas only")."""
    s = args.scale
    g, params = synth.config5(n_txns=int(1_000_000 * s), n_keys=max(1, int(100_000 * s)), seed=0xACC0D005 + rank)
    gdev, keep = native.device_graph(g, dev)
    out = torch.zeros(len(g.kind), dtype=torch.int32, device=dev)
    st = native.DeviceCommandStore(device=local)
    stream = torch.cuda.current_stream(dev).cuda_stream
    stats = None
    for _ in range(args.warmup):
        stats = st.levels_device(gdev, out.data_ptr(), stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ms = np.zeros(2)
    launches = 0
    t_start = time.perf_counter()
    for _ in range(args.steps):
        stats = st.levels_device(gdev, out.data_ptr(), stream)
        ms += np.array(stats["ms_stage"][:2])
        launches += stats["n_launches"]
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    ms /= max(args.steps, 1)
    pairs = int(g.key_off[-1])
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=_red_dev(dev))
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        p = torch.tensor([pairs], dtype=torch.int64, device=_red_dev(dev))
        dist.all_reduce(p, op=dist.ReduceOp.SUM)
        pairs = int(p.item())
    ms_per_step = 1000.0 * elapsed / max(args.steps, 1)
    dom = int(np.argmax(ms))
    pull = launches == args.steps          # one leveling launch per step: the rank-ordered dataflow (default)
    packed = bool(stats.get("packed"))
    if packed:
        names = ["k5 build (packed exec sort + key-chain sort + predecessor records)",
                 "k5 rank-ordered dataflow (k_level_rec)"]
    elif pull:
        names = ["k5 build (exec radix sort + key chains + predecessor CSR)", "k5 rank-ordered dataflow (k_level_pull)"]
    else:
        names = ["k5 build (exec radix sort + key chains + successor CSR)", "k5 frontier loop (k_level_step)"]
    achieved = stats["bytes_stage"][dom] / (ms[dom] / 1000.0) / 1e9 if ms[dom] > 0 else 0.0
    lk = "k_level_rec" if packed else ("k_level_pull" if pull else "k_level_step")
    if dom == 1:
        traffic, traffic_src = measured_traffic([lk], tag="config5")
    else:
        if packed:
            build = ["k_exec_words", "k_exec_pack", "k_exec_rank_p", "k_direct_check", "k_occ_pack", "k_walk",
                     "k_scan_reduce", "k_scan_sums", "k_scan_tile", "__amd_rocclr_copyBuffer",
                     "__amd_rocclr_fillBufferAligned"] + ["k_rk_count<%d>" % d for d in range(8, 12)] + \
                    ["k_rk_scatter<%d>" % d for d in range(8, 12)]
        else:
            build = ["k_exec_words", "k_exec_gather", "k_radix_count", "k_radix_scatter", "k_scan_reduce", "k_scan_sums",
                     "k_scan_tile", "k_exec_rank", "k_occ_fill", "k_chain<0>", "k_chain<1>", "k_chain<2>", "k_direct<0>",
                     "k_direct<1>", "k_direct<2>", "__amd_rocclr_copyBuffer", "__amd_rocclr_fillBufferAligned"]
        traffic, traffic_src = measured_traffic_per_step(build, "config5", lk)
    res = {
        "metric": METRIC, "value": pairs / (ms_per_step / 1000.0), "unit": "txn-key pairs/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms_per_step, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u32", "data": "synthetic",
        "config": {"workload": "config5: %d-txn waitingOn graph x %d keys over %d keys -> topological apply levels"
                               "%s" % (len(g.kind), params["keys_per_txn"], params["n_keys"],
                                       ", one replica per GPU" if world > 1 else ""),
                   "txns_per_step": len(g.kind) * world, "txn_key_pairs_per_step": pairs,
                   "parallelism": "replicas x%d" % world},
        "roofline": {"bound": "hbm", "kernel": names[dom], "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                     "algorithmic_bytes_per_launch": stats["bytes_stage"][dom], "launch_ms": ms[dom]},
        "stages_ms": {names[0]: round(float(ms[0]), 4), names[1]: round(float(ms[1]), 4)},
        "levels": stats["n_levels"], "edges": stats["n_edges"], "leveling_launches_per_step": launches / max(args.steps, 1),
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline_levels(g, args.cpu_budget)
    if rank == 0:
        print(json.dumps(res), flush=True)
    st.close()
    if world > 1:
        dist.destroy_process_group()


def _timed_steps(args, world, dev, step):
    stats = None
    for _ in range(args.warmup):
        stats = step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    all_stats = []
    t_start = time.perf_counter()
    for _ in range(args.steps):
        all_stats.append(step())
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=_red_dev(dev))
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed, all_stats


def _sum_over_ranks(world, dev, x):
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.int64, device=_red_dev(dev))
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return int(t.item())


def bench_ranges(args, rank, world, local, dev):
    """Config 4: 1M key txns x 4 keys against 100k Range-domain commands plus a 1M-txn
    CommandsForKey history (SNAPSHOT): keyDeps from the CFK and rangeDeps from the interval probe
    (SearchableRangeList / mapReduceRangesInternal), merged per request. Requests newer than every
    id of the store take the lean kernels, which read rangeDeps from the stabbing-index cells; the
    rest run the general fused kernel (k_resolve: K1 + K4 + K2). With N GPUs, N independent replicas."""
    s = args.scale
    w = synth.config4(n_txns=int(1_000_000 * s), n_keys=int(1_000_000 * s), n_ranges=max(1, int(100_000 * s)),
                      n_hist_txns=int(1_000_000 * s), seed=0xACC0D004 + rank)
    if args.range_frac > 0:
        # Range-domain requests beside the key txns: with range commands in the store they take the split kernels
        w = synth.with_range_requests(w, args.range_frac)
    store = native.DeviceCommandStore(device=local, slices=w.slices)
    store.load(w)
    qdev, keep = native.device_queries(w.queries, dev)
    sp = torch.cuda.current_stream(dev).cuda_stream
    regions = args.output == "regions"     # the headline's output contract (AD_REGIONS) unless --output packed
    elapsed, all_stats = _timed_steps(args, world, dev, lambda: store.deps_batch_device(qdev, sp, regions=regions)[1])
    stats = all_stats[-1]
    ms = np.mean([st["ms_stage"] for st in all_stats], axis=0)
    pairs = _sum_over_ranks(world, dev, w.queries.n_probes)
    other = "packed" if regions else "regions"
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(5):
        store.deps_batch_device(qdev, sp, regions=not regions)
    torch.cuda.synchronize(dev)
    other_ms = 1000.0 * (time.perf_counter() - t0) / 5
    # the per-kernel split from three steps with the library's extra stage events (see bench_deps)
    split_ms = np.zeros(7)
    os.environ["AD_STAGE_EVENTS"] = "1"
    try:
        for _ in range(3):
            split_ms += np.array(store.deps_batch_device(qdev, sp, regions=regions)[1]["ms_stage"][:7]) / 3
    finally:
        del os.environ["AD_STAGE_EVENTS"]
    ms_per_step = 1000.0 * elapsed / max(args.steps, 1)
    heads = sum(stats["n_keys"])
    out_bytes = 8 * heads + 4 * (heads + sum(stats["n_pairs"])) + 4 * sum(stats["n_unique"])
    n_rent = int(w.cmds.range_off[-1])
    # interval table once (16 B each) + 40 B per query + output, over the
    # resolve stages (lean passes with the stabbing-index range round + the general kernel on what
    # they deferred)
    alg = 16 * n_rent + 40 * len(w.queries) + out_bytes
    res_ms = float(sum(ms[i] for i in RESOLVE_STAGES))
    achieved = alg / (res_ms / 1000.0) / 1e9 if res_ms > 0 else 0.0
    res_kernels = resolve_kernels(stats, split_ms)
    traffic, src = measured_traffic(res_kernels, "config4")
    res = {
        "metric": METRIC, "value": pairs / (ms_per_step / 1000.0), "unit": "txn-key pairs/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms_per_step, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u32", "data": "synthetic",
        "config": {"workload": "config4: %d txns x 4 keys vs %d range commands + %d-entry CommandsForKey history, "
                               "SNAPSHOT%s" % (len(w.queries), len(w.cmds.txn), w.cfk.n_entries,
                                               ", one replica per GPU" if world > 1 else ""),
                   "txns_per_step": len(w.queries) * world, "txn_key_pairs_per_step": pairs,
                   "parallelism": "replicas x%d" % world,
                   "output": "regions (AD_REGIONS)" if regions else "packed arrays (request order)"},
        "%s_ms_per_step" % other: other_ms,
        "roofline": {"bound": "hbm", "kernel": " + ".join(res_kernels), "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": src,
                     "algorithmic_bytes_per_launch": alg, "launch_ms": res_ms},
        "stages_ms": {STAGES[i]: round(float(split_ms[i]), 4) for i in range(7)},
        "stages_note": "per-kernel split from 3 steps after the timed region (AD_STAGE_EVENTS=1); resolve %.4f ms "
                       "per timed step" % res_ms,
        "pairs_out": {A.MAP_NAMES[m]: int(stats["n_pairs"][m]) for m in range(3)},
    }
    if w.queries.range_off is not None:
        res["config"]["range_requests"] = int(np.count_nonzero(np.diff(w.queries.range_off.astype(np.int64))))
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline(w, args.cpu_budget)
    if rank == 0:
        print(json.dumps(res), flush=True)
    store.close()
    if world > 1:
        dist.destroy_process_group()


def bench_preaccept(args, rank, world, local, dev):
    """SURVEY §8 f3 on config 2's batch: the PreAccept timestamp proposal (CommandStore.preaccept
    minus the clock) of 1M requests x 8 keys against the maxConflicts of the 16M-entry history
    (one point interval per key). With N GPUs, N independent replicas."""
    s = args.scale
    w = synth.config2(n_txns=int(1_000_000 * s), n_keys=int(1_000_000 * s), n_hist_entries=int(16_000_000 * s),
                      seed=0xACC0D002 + rank)
    mc = synth.max_conflicts_from_cfk(w.cfk)
    st = native.DeviceCommandStore(device=local)
    st.load(w)                 # the store's snapshot: its keys carry per-key interval indexes
    st.load_preaccept_maps(mc, None)
    qdev, keep = native.device_queries(w.queries, dev)
    n = len(w.queries)
    out = dict(msb=torch.zeros(n, dtype=torch.int64, device=dev), lsb=torch.zeros(n, dtype=torch.int64, device=dev),
               node=torch.zeros(n, dtype=torch.int32, device=dev), flags=torch.zeros(n, dtype=torch.uint8, device=dev))
    sp = torch.cuda.current_stream(dev).cuda_stream
    elapsed, all_stats = _timed_steps(args, world, dev, lambda: st.preaccept_device(qdev, out, 1, 0, sp))
    pairs = _sum_over_ranks(world, dev, w.queries.n_probes)
    ms_per_step = 1000.0 * elapsed / max(args.steps, 1)
    kernel_ms = float(np.mean([x["ms_device"] for x in all_stats]))
    # algorithmic bytes: request inputs (txnId 20 B + key_off 8 B + 8 B per key), the map once
    # (8 B start + 20 B value + 1 B present per interval), outputs 21 B per request
    alg = 28 * n + 8 * w.queries.n_probes + 29 * len(mc) + 21 * n
    achieved = alg / (kernel_ms / 1000.0) / 1e9 if kernel_ms > 0 else 0.0
    res = {
        "metric": "PreAccept witnessedAt proposals: txn-key pairs/sec", "value": pairs / (ms_per_step / 1000.0),
        "unit": "txn-key pairs/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u64",
        "data": "synthetic",
        "config": {"workload": "config2 batch (%d txns x 8 keys) vs maxConflicts of %d intervals (SURVEY 8 f3)"
                               % (n, len(mc)), "txn_key_pairs_per_step": pairs, "parallelism": "replicas x%d" % world},
        "roofline": {"bound": "hbm", "kernel": "k_preaccept", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": None, "algorithmic_bytes_per_launch": alg,
                     "launch_ms": kernel_ms},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import pyoracle
        m = min(n, 200_000)
        qs = w.queries.window(0, m)
        t0 = time.perf_counter()
        pyoracle.preaccept(mc, None, qs, 1, 0)
        t = time.perf_counter() - t0
        res["cpu_baseline"] = dict(value=qs.n_probes / t, unit="txn-key pairs/s", cores=1, kind="port",
                                   sample="first %d requests (%.2f s), rc_preaccept, 1 thread" % (m, t))
    if rank == 0:
        print(json.dumps(res), flush=True)
    st.close()
    if world > 1:
        dist.destroy_process_group()


def bench_union(args, rank, world, local, dev):
    """SURVEY §8 f2 on config 2's batch: the coordinator's Deps.merge of R replica replies
    (ad_parts_union). R stores hold the config-2 snapshot (replicas that agree: every pair arrives R
    times, the full-deduplication case), each resolves the batch and exports its PartialDeps as
    rank-format parts; the timed step is the union of all R replies for every request. With N GPUs,
    N replicas of the job."""
    s = args.scale
    R = args.union
    w = synth.config2(n_txns=int(1_000_000 * s), n_keys=int(1_000_000 * s), n_hist_entries=int(16_000_000 * s),
                      seed=0xACC0D002 + rank)
    n = len(w.queries)
    sp = torch.cuda.current_stream(dev).cuda_stream
    engines, keep = [], []
    for r in range(R):
        st = native.DeviceCommandStore(device=local)
        st.load(w)
        qdev, k = native.device_queries(w.queries, dev)
        keep.append(k)
        engines.append(exchange.GpuEngine(st, qdev, np.arange(n), dev, stream=sp))
    g = exchange.build_global_dict([e.dictionary() for e in engines])
    for e in engines:
        e.set_global_dict(g)
    sends = []
    for e in engines:
        e.resolve()
        sends.append(e.export(np.array([0, n], np.uint64)))
    torch.cuda.synchronize(dev)
    recv, totals = {}, np.zeros(4, np.int64)
    for a, (name, mult) in enumerate((("hdr", 4), ("keys", 1), ("ids", 1), ("k2t", 1))):
        recv[name] = torch.cat([sd[0][name][:int(sd[1][0, a]) * mult] for sd in sends])
    for sd in sends:
        totals += sd[1][0]
    p = A.AdParts()
    p.hdr, p.keys, p.ids, p.k2t = (recv[k].data_ptr() for k in ("hdr", "keys", "ids", "k2t"))
    p.n_parts, p.n_key_words, p.n_ids, p.n_k2t = (int(x) for x in totals)
    p.id_format = A.AD_IDS_RANK
    owner = engines[0].store
    src = [int(sd[1][0, 0]) for sd in sends]
    last = {}

    def step():
        last["mg"] = owner.union_parts(p, src, 0, n, sp)
        return {"ms_device": last["mg"].ms_device}
    elapsed, all_stats = _timed_steps(args, world, dev, step)
    in_pairs = int(totals[3] - totals[1])
    pairs = _sum_over_ranks(world, dev, in_pairs)
    ms_per_step = 1000.0 * elapsed / max(args.steps, 1)
    kernel_ms = float(np.mean([x["ms_device"] for x in all_stats]))
    mg = last["mg"]
    out_bytes = sum(8 * int(mg.n_keys[m]) + 4 * int(mg.n_ids[m]) + 4 * int(mg.n_k2t[m]) for m in range(3))
    alg = int(32 * totals[0] + 8 * totals[1] + 4 * totals[2] + 4 * totals[3]) + out_bytes
    achieved = alg / (kernel_ms / 1000.0) / 1e9 if kernel_ms > 0 else 0.0
    res = {
        "metric": "Deps.merge of replica replies: input txn-key pairs/sec", "value": pairs / (ms_per_step / 1000.0),
        "unit": "txn-key pairs/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
        "data": "synthetic",
        "config": {"workload": "config2 batch (%d txns x 8 keys), %d replica replies per request (SURVEY 8 f2)" % (n, R),
                   "input_pairs_per_step": pairs, "parallelism": "replicas x%d" % world},
        "roofline": {"bound": "hbm", "kernel": "k_union_rank + k_union_emit", "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                     "algorithmic_bytes_per_launch": alg, "launch_ms": kernel_ms},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import pyoracle
        m = min(n, 1_000)
        reps = [pyoracle.resolve(w, first=0, count=m) for r in range(R)]
        t0 = time.perf_counter()
        merged = pyoracle.merge_batches(reps)
        t = time.perf_counter() - t0
        sp_pairs = sum(int(b.pair_count(mm)) for b in reps for mm in range(3))
        res["cpu_baseline"] = dict(value=sp_pairs / t, unit="txn-key pairs/s", cores=1, kind="port",
                                   sample="first %d requests' %d replies (%.2f s), rc_result_merge, 1 thread" % (m, R, t))
        del merged
    if rank == 0:
        print(json.dumps(res), flush=True)
    for e in engines:
        e.store.close()
    if world > 1:
        dist.destroy_process_group()


def bench_recovery(args, rank, world, local, dev):
    """SURVEY §8 f4 on config 2's snapshot: the BeginRecovery scan --recovery-scan (AD_RECOVER_*) for
    a batch of recovering txns (half of them txnIds of the history, i.e. known to the
    CommandsForKey, half new ones from the config-2 batch), entries carrying TxnInfo.missing()
    lists. mapReduceFull scans every probed key's byId range (CommandsForKey.java:854), as the
    reference does. With N GPUs, N independent replicas."""
    s = args.scale
    w = synth.config2(n_txns=int(1_000_000 * s), n_keys=int(1_000_000 * s), n_hist_entries=int(16_000_000 * s),
                      seed=0xACC0D002 + rank)
    w.cfk = synth.with_missing_fast(w.cfk, 0xACC0D00F)
    n = max(2, int(args.recovery * s))
    rng = np.random.default_rng(0xACC0D00F)
    key_of = np.repeat(np.arange(len(w.cfk.keys)), np.diff(w.cfk.seg.astype(np.int64)))
    e = rng.choice(w.cfk.n_entries, n // 2, replace=False)
    from accord_deps.model import Queries, Tids
    q = w.queries
    nb = n - n // 2
    txn = Tids.concat([w.cfk.txn.take(e), q.txn.take(np.arange(nb))])
    keys = [w.cfk.keys[key_of[e]].reshape(-1, 1), q.keys[:int(q.key_off[nb])]]
    off = np.concatenate([np.arange(n // 2 + 1, dtype=np.uint64), (n // 2 + q.key_off[1:nb + 1]).astype(np.uint64)])
    rq = Queries(txn, txn, off, np.concatenate([k.reshape(-1) for k in keys]))
    st = native.DeviceCommandStore(device=local)
    st.load(w)
    qdev, keep = native.device_queries(rq, dev)
    sp = torch.cuda.current_stream(dev).cuda_stream
    scan = args.recovery_scan
    elapsed, all_stats = _timed_steps(args, world, dev, lambda: st.recovery_scan_device(qdev, scan, sp)[1])
    stats = all_stats[-1]
    probes = _sum_over_ranks(world, dev, rq.n_probes)
    ms_per_step = 1000.0 * elapsed / max(args.steps, 1)
    ms_scan = float(np.mean([x["ms_stage"][0] for x in all_stats]))   # k_encode_recover .. k_build
    # algorithmic bytes: compulsory read of every probed key's entries once (16 B each: ranks, status,
    # missing offset) + their missing ids (4 B) + requests (24 B + 8 B per key) + the CSR output
    touched = np.searchsorted(w.cfk.keys, np.unique(rq.keys))
    ok = touched < len(w.cfk.keys)
    touched = touched[ok][w.cfk.keys[touched[ok]] == np.unique(rq.keys)[ok]]
    seg = w.cfk.seg.astype(np.int64)
    ent = int((seg[touched + 1] - seg[touched]).sum())
    mo = w.cfk.miss_off.astype(np.int64)
    nmiss = int((mo[seg[touched + 1]] - mo[seg[touched]]).sum())
    pk = np.searchsorted(w.cfk.keys, rq.keys)
    hit = pk < len(w.cfk.keys)
    hit[hit] &= w.cfk.keys[pk[hit]] == rq.keys[hit]
    pk = pk[hit]
    probe_seg = int((seg[pk + 1] - seg[pk]).sum())      # entries a whole-segment scan of every probe reads
    heads = sum(stats["n_keys"])
    out_bytes = 8 * heads + 4 * (heads + sum(stats["n_pairs"])) + 4 * sum(stats["n_unique"])
    alg = 16 * ent + 4 * nmiss + 24 * n + 8 * rq.n_probes + out_bytes
    achieved = alg / (ms_scan / 1000.0) / 1e9 if ms_scan > 0 else 0.0
    names = ["AD_RECOVER_STARTED_BEFORE_ACCEPTED_NO_WITNESS", "AD_RECOVER_STARTED_BEFORE_STABLE_WITNESS",
             "AD_RECOVER_STARTED_AFTER_ACCEPTED_NO_WITNESS", "AD_RECOVER_EXECUTES_AFTER_STABLE_NO_WITNESS"]
    res = {
        "metric": "BeginRecovery mapReduceFull scans: txn-key probes/sec", "value": probes / (ms_per_step / 1000.0),
        "unit": "txn-key probes/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
        "data": "synthetic",
        "config": {"workload": "config2 snapshot (%d entries, missing() lists), %d recovering txns (half known), scan %s "
                               "(SURVEY 8 f4)" % (w.cfk.n_entries, n, names[scan]),
                   "txn_key_probes_per_step": probes, "parallelism": "replicas x%d" % world},
        "roofline": {"bound": "hbm", "kernel": "k_scan_full (+ encode, probe, k_build)", "achieved": achieved,
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                     "algorithmic_bytes_per_launch": alg, "launch_ms": ms_scan,
                     "scan_bytes_per_launch": 16 * probe_seg},
        "stages_ms": {"encode+probe+k_scan_full+k_build": round(ms_scan, 4),
                      "offsets": round(float(np.mean([x["ms_stage"][4] for x in all_stats])), 4),
                      "pack": round(float(np.mean([x["ms_stage"][5] for x in all_stats])), 4)},
        "pairs_out": {A.MAP_NAMES[m]: int(stats["n_pairs"][m]) for m in range(3)},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import pyoracle
        ost = pyoracle.OracleStore()
        ost.load(w)
        m, t, done = 16, 0.0, 0
        while done < n and t < args.cpu_budget:
            c = min(m, n - done)
            t0 = time.perf_counter()
            ost.recovery_batch(rq, scan, done, c)
            t += time.perf_counter() - t0
            done += c
            m *= 2
        ost.close()
        pr = int(rq.key_off[done])
        res["cpu_baseline"] = dict(value=pr / t, unit="txn-key probes/s", cores=1, kind="port",
                                   sample="first %d of %d recovering txns (%d probes, %.1f s), rc_recovery_batch "
                                          "(mapReduceFull restatement), 1 thread" % (done, n, pr, t))
    if rank == 0:
        print(json.dumps(res), flush=True)
    st.close()
    if world > 1:
        dist.destroy_process_group()


def bench_cfk_update(args, rank, world, local, dev):
    """SURVEY §8 f1 on config 2's snapshot: a step is one batch of N CommandsForKey.update status
    transitions applied to the device-resident snapshot (ad_cfk_update_device: locate + apply +
    re-derivation of every derived array). Batch b raises a random N-subset of the entries that are
    not APPLIED by one status (PREACCEPTED -> ACCEPTED -> COMMITTED -> STABLE -> APPLIED, executeAt
    kept), so every step changes the store. It replaces a host re-ingest + re-upload of the snapshot
    (ingest_ms). With N GPUs, N independent replicas."""
    s = args.scale
    w = synth.config2(n_txns=int(1_000_000 * s), n_keys=int(1_000_000 * s), n_hist_entries=int(16_000_000 * s),
                      seed=0xACC0D002 + rank)
    cfk = w.cfk
    from accord_deps.model import CfkUpdates
    n = max(1, int(args.cfk_update * s))
    rng = np.random.default_rng(0xACC0D01F)
    key_of = np.repeat(cfk.keys, np.diff(cfk.seg.astype(np.int64)))
    status = cfk.status.copy()
    batches = []
    n_ins = int(n * args.cfk_insert_frac) // 8 * 8       # fresh PreAccepts: 8 keys each
    n_tr = n - n_ins
    from accord_deps.model import Tids, make_txn_ids
    for b in range(args.warmup + args.steps):
        live = np.nonzero(status < A.ST_APPLIED)[0]
        e = np.sort(rng.choice(live, min(n_tr, len(live)), replace=False)) if len(live) else np.zeros(0, np.int64)
        st = np.maximum(status[e] + 1, A.ST_ACCEPTED).astype(np.uint8)
        status[e] = st
        u = CfkUpdates(key_of[e], cfk.txn.take(e), cfk.exec.take(e), st)
        if args.cfk_deps:
            # each transition (a deps status) carries deps: the up-to-D entries before it in its key's
            # byId that its kind witnesses (key-domain ids) -> the device maintains every missing()
            # list and inserts absent deps (Updating.insertOrUpdate)
            D = args.cfk_deps
            lo_of = np.repeat(cfk.seg[:-1].astype(np.int64), np.diff(cfk.seg.astype(np.int64)))[e]
            cand = e[:, None] - np.arange(1, D + 1)[None, :]
            ok = cand >= lo_of[:, None]
            cc = np.where(ok, cand, 0)
            wk = np.array([0b10, 0b11, 0b10, 0b11, 0b11011, 0, 0, 0], np.uint64)[cfk.txn.kind()[e].astype(np.int64)]
            ok &= ((wk[:, None] >> cfk.txn.kind()[cc].astype(np.uint64)) & np.uint64(1)) == 1
            ok &= (cfk.txn.lsb[cc] & np.uint64(1)) == 0
            ok = ok[:, ::-1]                          # ascending ids: earliest first
            cc = cc[:, ::-1]
            cnt = ok.sum(axis=1)
            off = np.zeros(len(e) + 1, np.uint64)
            off[1:] = np.cumsum(cnt)
            sel = cc[ok]
            u = CfkUpdates(u.keys, u.txn, u.exec, u.status, None, off, cfk.txn.take(sel))
        if n_ins:
            # PreAccepts of txnIds newer than the store (epoch above the history's), inserted as
            # PREACCEPTED into 8 existing keys each (CommandsForKey.update's insert branch)
            m = n_ins // 8
            t = make_txn_ids(16 + b, np.arange(m, dtype=np.uint64) * 2 + 1, rng.integers(0, 2, m), rng.integers(1, 17, m))
            rows = np.repeat(np.arange(m), 8)
            ks = cfk.keys[rng.integers(0, len(cfk.keys), n_ins)]
            ti = t.take(rows)
            dep_off, deps = u.dep_off, u.deps
            u = CfkUpdates(np.concatenate([u.keys, ks]), Tids.concat([u.txn, ti]), Tids.concat([u.exec, ti]),
                           np.concatenate([u.status, np.full(n_ins, A.ST_PREACCEPTED, np.uint8)]))
            if dep_off is not None:       # PreAccepts carry no deps (PREACCEPTED has none)
                u.dep_off = np.concatenate([dep_off, np.full(n_ins, dep_off[-1], np.uint64)])
                u.deps = deps
        batches.append((u,) + native.device_updates(u, dev))
    store = native.DeviceCommandStore(device=local)
    t0 = time.time()
    store.load(w)
    ingest_ms = 1000 * (time.time() - t0)
    sp = torch.cuda.current_stream(dev).cuda_stream
    it = iter(batches)

    def step():
        b = next(it)
        applied, stt = store.cfk_update_device(b[1], sp)
        stt["applied"] = applied
        stt["inserted"] = stt["n_keys"][0]
        return stt
    elapsed, all_stats = _timed_steps(args, world, dev, step)
    ms_per_step = 1000.0 * elapsed / max(args.steps, 1)
    upd = _sum_over_ranks(world, dev, sum(len(batches[args.warmup + i][0]) for i in range(args.steps)))
    # algorithmic bytes of one launch sequence: the update batch (49 B each) + per entry the state
    # read (status 1 + executeAt rank 4 + ent 8 + key index 4) and tau written (4) + the derived
    # lists written (cand 4 B per never-elided class entry, cwr 4 B, w 8 B per committed Write) and
    # the committed entries' (key, executeAt) sort (12 B written and read once) + per key krec 32 +
    # KeyEntry 64
    ne, nk = cfk.n_entries, len(cfk.keys)
    kinds = cfk.txn.kind()
    comm = (status >= A.ST_COMMITTED) & (status <= A.ST_APPLIED)
    rw = (kinds <= A.KIND_WRITE)
    never = (status != A.ST_TRANSITIVELY_KNOWN) & (status != A.ST_INVALID) & ~(comm & rw)
    n_cand = int(never.sum()) * 3
    alg = 49 * n + 21 * ne + 4 * n_cand + 4 * int((comm & rw).sum()) + 8 * int((comm & (kinds == A.KIND_WRITE)).sum()) \
        + 24 * int(comm.sum()) + 96 * nk
    ms_dev = float(np.mean([x["ms_device"] for x in all_stats]))
    achieved = alg / (ms_dev / 1000.0) / 1e9 if ms_dev > 0 else 0.0
    res = {
        "metric": "CommandsForKey.update on the device-resident snapshot: updates/sec", "value": upd / elapsed,
        "unit": "updates/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms_per_step,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32", "data": "synthetic",
        "config": {"workload": "config2 snapshot (%d entries, %d keys), batches of %d status transitions + %d insertions "
                               "(PreAccepts of new txnIds, 8 keys each) (SURVEY 8 f1)" % (ne, nk, n_tr, n_ins),
                   "parallelism": "replicas x%d" % world},
        "roofline": {"bound": "hbm", "kernel": "k_upd_* + k_drv_* + radix sort + trees", "achieved": achieved,
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                     "algorithmic_bytes_per_launch": alg, "launch_ms": ms_dev},
        "stages_ms": {"locate+apply": round(float(np.mean([x["ms_stage"][0] for x in all_stats])), 4),
                      "re-derivation": round(float(np.mean([x["ms_stage"][1] for x in all_stats])), 4)},
        "applied": [x["applied"] for x in all_stats],
        "inserted": [x["inserted"] for x in all_stats],
        "ingest_ms": ingest_ms,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import cfk_update as U
        u0 = batches[0][0]
        done = min(n_tr, 100_000)
        sub = CfkUpdates(u0.keys[:done], u0.txn.take(np.arange(done)), u0.exec.take(np.arange(done)), u0.status[:done])
        t0 = time.perf_counter()
        U.cfk_update(cfk, sub)
        t = time.perf_counter() - t0
        res["cpu_baseline"] = dict(value=done / t, unit="updates/s", cores=1, kind="port",
                                   sample="first %d of %d updates of the first batch (status transitions; %.1f s), "
                                          "oracle/cfk_update.py (CommandsForKey.update restatement: binarySearch + raise), "
                                          "1 thread" % (done, len(u0), t))
    if rank == 0:
        print(json.dumps(res), flush=True)
    store.close()
    if world > 1:
        dist.destroy_process_group()


def bench_steady(args, rank, world, local, dev):
    """Steady state of a config-2 store: a step resolves one batch of R fresh
    PreAccepts (8 Zipf keys each; ad_deps_batch_device, SNAPSHOT), then one ad_cfk_update_device
    batch registers them -- CommandsForKey.update inserting each txn PREACCEPTED into its keys -- and
    moves the previous step's txns on to APPLIED (executeAt = txnId), plus T status transitions of
    the history's live entries. Each step's requests are newer than the last step's, so a resolve
    sees the previous batch in flight and everything before it applied. The store grows by R x 8
    entries per step. With N GPUs, N independent replicas."""
    s = args.scale
    w = synth.config2(n_txns=int(1_000_000 * s), n_keys=int(1_000_000 * s), n_hist_entries=int(16_000_000 * s),
                      seed=0xACC0D002 + rank)
    R = max(1, int(args.steady * s))
    T = int(args.steady_transitions * s) if args.steady_transitions >= 0 else R
    n_b = args.warmup + args.steps
    # Zipf over the whole key space: keys the store has never seen get their CommandsForKey from the
    # update that registers their first txn
    stream = synth.config2_stream(w, n_b, R, seed=0xACC0D5EE + rank)
    cfk = w.cfk
    from accord_deps.model import CfkUpdates, Tids
    rng = np.random.default_rng(0xACC0D01E)
    key_of = np.repeat(cfk.keys, np.diff(cfk.seg.astype(np.int64)))
    status = cfk.status.copy()
    batches = []
    prev = None
    for b in range(n_b):
        q = stream[b]
        qdev, keep = native.device_queries(q, dev)
        live = np.nonzero(status < A.ST_APPLIED)[0]
        e = np.sort(rng.choice(live, min(T, len(live)), replace=False)) if len(live) else np.zeros(0, np.int64)
        st = np.maximum(status[e] + 1, A.ST_ACCEPTED).astype(np.uint8)
        status[e] = st
        rows = np.repeat(np.arange(len(q)), np.diff(q.key_off.astype(np.int64)))
        ti = q.txn.take(rows)
        parts = [(q.keys, ti, ti, np.full(len(rows), A.ST_PREACCEPTED, np.uint8)),
                 (key_of[e], cfk.txn.take(e), cfk.exec.take(e), st)]
        if prev is not None:
            parts.append((prev[0], prev[1], prev[1], np.full(len(prev[0]), A.ST_APPLIED, np.uint8)))
        prev = (q.keys, ti)
        u = CfkUpdates(np.concatenate([p_[0] for p_ in parts]), Tids.concat([p_[1] for p_ in parts]),
                       Tids.concat([p_[2] for p_ in parts]), np.concatenate([p_[3] for p_ in parts]))
        ud, ukeep = native.device_updates(u, dev)
        rdev = rkeep = None
        if args.steady_recovery:
            # recovery of the txns this step registers (BeginRecovery on a live store: the view is
            # built from the device state the update just left)
            k = min(args.steady_recovery, len(q))
            rq = q.window(0, k)
            rdev, rkeep = native.device_queries(rq, dev)
        batches.append((qdev, keep, ud, ukeep, len(u), q.n_probes, rdev, rkeep))
    store = native.DeviceCommandStore(device=local)
    store.load(w)
    sp = torch.cuda.current_stream(dev).cuda_stream
    it = iter(batches)

    def step():
        b = next(it)
        _, rs = store.deps_batch_device(b[0], sp)
        _, us = store.cfk_update_device(b[2], sp)
        rec_ms = 0.0
        if b[6] is not None:
            _, rc = store.recovery_scan_device(b[6], args.recovery_scan, sp)
            rec_ms = rc["ms_device"]
        return dict(resolve_ms=rs["ms_device"], update_ms=us["ms_device"], locate_ms=us["ms_stage"][0],
                    derive_ms=us["ms_stage"][1], inserted=us["n_keys"][0], pairs=sum(rs["n_pairs"]), recovery_ms=rec_ms)
    elapsed, all_stats = _timed_steps(args, world, dev, step)
    ms_per_step = 1000.0 * elapsed / max(args.steps, 1)
    reqs = _sum_over_ranks(world, dev, R * args.steps)
    mean = lambda k: round(float(np.mean([x[k] for x in all_stats])), 4)   # noqa: E731
    res = {
        "metric": "steady-state PreAccept on a config-2 store: requests/sec (deps resolved + registered by "
                  "CommandsForKey.update + status transitions)", "value": reqs / elapsed,
        "unit": "requests/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms_per_step,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32", "data": "synthetic",
        "config": {"workload": "config2 store (%d entries initially), per step %d fresh PreAccepts x 8 keys resolved "
                               "then inserted, the previous step's applied, + %d history transitions" % (cfk.n_entries, R, T),
                   "parallelism": "replicas x%d" % world},
        "stages_ms": {"resolve": mean("resolve_ms"), "update": mean("update_ms"), "update.locate+apply+insert":
                      mean("locate_ms"), "update.re-derivation": mean("derive_ms"),
                      "recovery (live store, view rebuilt from the device state)": mean("recovery_ms")},
        "entries_after": int(cfk.n_entries + sum(x["inserted"] for x in all_stats)),
        "updates_per_step": int(np.mean([b_[4] for b_ in batches])),
        "pairs_per_step": mean("pairs"),
    }
    if rank == 0:
        print(json.dumps(res), flush=True)
    store.close()
    if world > 1:
        dist.destroy_process_group()


def bench_sequential(args, rank, world, local, dev):
    """Config 1: 10k txns x 4 keys over 1k keys, one CommandStore, SEQUENTIAL PreAccept (each txn
    inserted as PREACCEPTED before its deps). SEQUENTIAL runs through the host API: a step is one
    snapshot upload + ad_deps_batch call on one store -- host arrays in and out, snapshot ingest (the
    batch's own PreAccepts) and PCIe included, so this line is latency, not the device-resident
    throughput of configs 2/4. The result stays in the C ABI's host CSR arrays (what a Java caller
    wraps with KeyDeps.SerializerSupport.create); Python objects are not built in the timed step."""
    w = synth.config1(seed=0xACC0D001 + rank)
    st = native.DeviceCommandStore(device=local)
    if args.resident:
        # steady state of one store: the snapshot stays in HBM; batch b is config 1's
        # batch moved to epoch +b+1 (fresh txnIds, same keys), PreAccepted by device-side insertion
        from accord_deps.model import Queries, Tids
        st.load(w, prepare=False)
        st.deps_batch_stats(w.queries, w.flags)            # creates the 1k CommandsForKeys (host path)
        qs = []
        for b in range(args.warmup + args.steps):
            q = w.queries
            t = Tids(q.txn.msb + np.uint64((b + 1) << 15), q.txn.lsb, q.txn.node)
            qs.append(Queries(t, t, q.key_off, q.keys))
        it = iter(qs)

        def step():
            return st.deps_batch_stats(next(it), w.flags)
    else:
        def step():
            # SEQUENTIAL inserts the batch into the store: every step re-uploads the initial snapshot
            st.load(w, prepare=False)
            return st.deps_batch_stats(w.queries, w.flags)
    elapsed, all_stats = _timed_steps(args, world, dev, step)
    st.close()
    pairs = _sum_over_ranks(world, dev, w.queries.n_probes)
    ms_per_step = 1000.0 * elapsed / max(args.steps, 1)
    stats = all_stats[-1]
    res = {
        "metric": METRIC, "value": pairs / (ms_per_step / 1000.0), "unit": "txn-key pairs/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms_per_step, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u32", "data": "synthetic",
        "config": {"workload": "config1: 10000 txns x 4 keys over 1000 keys, SEQUENTIAL PreAccept, host API " +
                               ("(resident store: each step a fresh batch inserted on the device + PCIe + device)"
                                if args.resident else "(ingest + PCIe + device per step)"),
                   "txns_per_step": len(w.queries) * world,
                   "txn_key_pairs_per_step": pairs, "parallelism": "replicas x%d" % world},
        "device_ms": stats["ms_device"], "ingest_ms": stats["ms_ingest"],
        "pairs_out": {A.MAP_NAMES[m]: int(stats["n_pairs"][m]) for m in range(3)},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import pyoracle
        t0 = time.perf_counter()
        reps = 0
        while reps == 0 or time.perf_counter() - t0 < args.cpu_budget / 3:
            pyoracle.resolve(w)
            reps += 1
        t = time.perf_counter() - t0
        res["cpu_baseline"] = dict(value=w.queries.n_probes * reps / t, unit="txn-key pairs/s", cores=1, kind="port",
                                   sample="whole config-1 batch x%d (%.1f s), refcpu SEQUENTIAL, 1 thread" % (reps, t))
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--scale", type=float, default=1.0, help="shrink the workload (tests / dry runs)")
    ap.add_argument("--cpu-budget", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--output", choices=("regions", "packed"), default="regions",
                    help="config 2 on one GPU: read the result through its regions (AD_REGIONS, default) or the packed arrays")
    ap.add_argument("--config", type=int, default=None, choices=(1, 2, 3, 4, 5),
                    help="default: 2 on one GPU (BASELINE config 2, the headline), 3 on N > 1 GPUs (N/8 of BASELINE "
                         "config 3, exactly config 3 at N = 8, through the library's RCCL node exchange); "
                         "1: SEQUENTIAL PreAccept batch (host API); 4: range transactions; 5: execution levels (K5)")
    ap.add_argument("--union", type=int, default=0, metavar="R",
                    help="with config 2: the coordinator's Deps.merge of R replica replies (SURVEY 8 f2)")
    ap.add_argument("--preaccept", action="store_true",
                    help="with config 2: the PreAccept timestamp proposal (SURVEY 8 f3) instead of deps")
    ap.add_argument("--recovery", type=int, default=0, metavar="N",
                    help="with config 2: BeginRecovery scans for N recovering txns on the config-2 snapshot (SURVEY 8 f4)")
    ap.add_argument("--cfk-update", type=int, default=0, metavar="N",
                    help="with config 2: batches of N CommandsForKey.update status transitions on the device (SURVEY 8 f1)")
    ap.add_argument("--steady", type=int, default=0, metavar="R",
                    help="config-2 steady state: per step resolve R fresh PreAccepts, then register them "
                         "(CommandsForKey.update inserts) with --steady-transitions status transitions")
    ap.add_argument("--steady-transitions", type=int, default=-1, metavar="T", help="default 8R")
    ap.add_argument("--steady-recovery", type=int, default=0, metavar="K",
                    help="--steady: each step also runs a recovery scan (--recovery-scan) for K of the txns it registered")
    ap.add_argument("--resident", action="store_true",
                    help="--config 1: keep the store resident, each step a fresh SEQUENTIAL batch (device-side insertion)")
    ap.add_argument("--cfk-deps", type=int, default=0, metavar="D",
                    help="--cfk-update: transitions carry D deps each (device missing() maintenance + additions)")
    ap.add_argument("--cfk-insert-frac", type=float, default=0.5,
                    help="--cfk-update: share of each batch that inserts new txnIds (fresh PreAccepts)")
    ap.add_argument("--accept-frac", type=float, default=0.0,
                    help="config 2: share of Accept requests (in-flight txns, S = proposed executeAt, self excluded)")
    ap.add_argument("--unordered-frac", type=float, default=0.0,
                    help="config 2: share of out-of-order PreAccepts (txnId inside the history's last ticks)")
    ap.add_argument("--unordered-window", type=int, default=2000, help="hlc ticks of --unordered-frac's lateness")
    ap.add_argument("--range-frac", type=float, default=0.0,
                    help="config 2 / 4: this share of the requests Range-domain txns over one range of 1-8 keys each "
                         "(synth.with_range_requests): on config 2's store (no range commands) they run the lean "
                         "passes as the keys inside their ranges; on config 4's the split kernels, beside the lean passes")
    ap.add_argument("--recovery-scan", type=int, default=3, choices=(0, 1, 2, 3), help="AD_RECOVER_* scan of --recovery")
    ap.add_argument("--exchange", action="store_true",
                    help="run the node exchange (ad_exchange over the library's RCCL communicator) even on one GPU")
    ap.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                    help="nccl (RCCL, one GPU per rank: the measured configuration); gloo: rehearsal of the "
                         "N>1 path on fewer GPUs (ranks share GPUs, the exchange is staged through host memory)")
    args = ap.parse_args()

    global RED_DEV
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log("note: --gpus %d but WORLD_SIZE %d; using WORLD_SIZE" % (args.gpus, world))
    if args.dist_backend == "gloo":
        local = local % max(1, torch.cuda.device_count())
        RED_DEV = torch.device("cpu")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    if args.config is None:
        args.config = 3 if world > 1 else 2
    if args.config == 5:
        return bench_levels(args, rank, world, local, dev)
    if args.config == 4:
        return bench_ranges(args, rank, world, local, dev)
    if args.config == 1:
        return bench_sequential(args, rank, world, local, dev)
    if args.preaccept:
        return bench_preaccept(args, rank, world, local, dev)
    if args.union:
        return bench_union(args, rank, world, local, dev)
    if args.recovery:
        return bench_recovery(args, rank, world, local, dev)
    if args.cfk_update:
        return bench_cfk_update(args, rank, world, local, dev)
    if args.steady:
        return bench_steady(args, rank, world, local, dev)

    return bench_deps(args, rank, world, local, dev)


def bench_deps(args, rank, world, local, dev):
    """The BASELINE metric: config 2 on one GPU (the headline); config 3 (N/8 of it on N GPUs, exactly
    config 3 at N = 8) for the node path: every store resolves the requests touching its slice, then
    the library's node exchange (ad_exchange: RCCL over xGMI + K3 merge on the owning GPU) combines them.
    `--config 2` at N > 1: config 2 weak-scaled per GPU through the same exchange."""
    s = args.scale
    cfg = args.config
    t0 = time.time()
    exec_ids = None
    if cfg == 3:
        w, txn_index, n_total, exec_ids = synth.config3_shard(rank, world, txns_per_gpu=int(8_000_000 * s),
                                                             keys_per_gpu=int(1_250_000 * s))
    else:
        w, txn_index, n_total = synth.config2_sharded(rank, world, n_txns_per_gpu=int(1_000_000 * s),
                                                      n_keys_per_gpu=int(1_000_000 * s),
                                                      n_hist_entries_per_gpu=int(16_000_000 * s))
    mix = args.accept_frac > 0 or args.unordered_frac > 0
    if mix:
        if world > 1 or cfg != 2:
            raise SystemExit("--accept-frac / --unordered-frac: config 2 on a single store only")
        w = synth.with_request_mix(w, args.accept_frac, args.unordered_frac, args.unordered_window)
    if args.range_frac > 0:
        if world > 1 or cfg != 2:
            raise SystemExit("--range-frac: config 2 on a single store, or config 4")
        w = synth.with_range_requests(w, args.range_frac)
    log("rank %d: config %d generated in %.1f s: %d keys, %d entries, %d of %d requests routed here, %d probes" %
        (rank, cfg, time.time() - t0, len(w.cfk.keys), w.cfk.n_entries, len(w.queries), n_total, w.queries.n_probes))

    store = native.DeviceCommandStore(device=local, slices=w.slices)
    use_x = (world > 1 and args.dist_backend == "nccl") or args.exchange
    t_ing = time.time()
    # config 3 knows its node-wide dictionary up front: the snapshot is built once, over it
    store.load(w, prepare=not (use_x and cfg == 3))
    ingest_ms = 1000.0 * (time.time() - t_ing)
    qdev, keep = native.device_queries(w.queries, dev)
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream
    last = {}
    node_x = None
    if use_x:
        # ingest-time: the node's global dictionary (ids travel as uint32 global ranks), the RCCL communicator
        t_g = time.time()
        if cfg == 3:
            got = [None] * world
            if world > 1:
                dist.all_gather_object(got, (exec_ids.msb, exec_ids.lsb, exec_ids.node))
            else:
                got = [(exec_ids.msb, exec_ids.lsb, exec_ids.node)]
            from accord_deps.model import Tids
            g = synth.config3_global_dict(w.params, [Tids(*x) for x in got])
        else:
            mine = store.dictionary()
            got = [None] * world
            if world > 1:
                dist.all_gather_object(got, (mine.msb, mine.lsb, mine.node))
            else:
                got = [(mine.msb, mine.lsb, mine.node)]
            from accord_deps.model import Tids
            g = exchange.build_global_dict([Tids(*x) for x in got])
        store.set_global_dict(g)
        node_x = exchange.NodeExchange(store, qdev, txn_index, n_total, rank, world, dev, stream=sp)
        log("rank %d: global dictionary of %d ids + RCCL communicator in %.1f s" % (rank, len(g.msb), time.time() - t_g))

        def step():
            mg = node_x.step()
            return node_x.last_stats, mg.ms_device, node_x.last_exchange
    elif world > 1:
        # gloo rehearsal on fewer GPUs than ranks: the same protocol with a Python transport staged
        # through host memory (RCCL cannot put two ranks on one GPU)
        engine = exchange.GpuEngine(store, qdev, txn_index, dev, stream=sp)
        ex = exchange.ShardExchange(engine, txn_index, n_total, rank, world, count_device=None, stage_cpu=True)
        ex.install_global_dict()

        def step():
            mg = ex.step()
            return engine.last_stats, mg.ms_device, None
    else:
        regions = args.output == "regions"

        def step():
            last["res"], st = store.deps_batch_device(qdev, sp, regions=regions)
            return st, 0.0, None

    stats = None
    for _ in range(args.warmup):
        stats, _, _ = step()
    torch.cuda.synchronize(dev)

    stage_ms = np.zeros(7)
    merge_ms = 0.0
    xs = dict(bytes_moved=0, ms_export=0.0, ms_move=0.0, ms_merge=0.0, ms_total=0.0)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t_start = time.perf_counter()
    for _ in range(args.steps):
        stats, mms, xst = step()
        stage_ms += np.array(stats["ms_stage"][:7])
        merge_ms += mms
        if xst:
            for k in xs:
                xs[k] += xst[k]
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    stage_ms /= max(args.steps, 1)
    merge_ms /= max(args.steps, 1)
    for k in xs:
        xs[k] /= max(args.steps, 1)
    probes = w.queries.n_probes
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=_red_dev(dev))
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        p = torch.tensor([probes, xs["bytes_moved"]], dtype=torch.int64, device=_red_dev(dev))
        dist.all_reduce(p, op=dist.ReduceOp.SUM)
        probes = int(p[0].item())
        xs["bytes_moved_all_ranks"] = int(p[1].item())
    ms_per_step = 1000.0 * elapsed / max(args.steps, 1)
    value = probes / (ms_per_step / 1000.0)
    # the per-kernel split of the resolve (prepare, lean passes, general kernel) from three more steps
    # after the timed region with the library's extra stage events on (AD_STAGE_EVENTS: each record
    # idles the GPU ~4 us, so the timed steps carry only the resolve's start and end events)
    split_ms = np.zeros(7)
    os.environ["AD_STAGE_EVENTS"] = "1"
    try:
        for _ in range(3):
            st_d, _, _ = step()
            split_ms += np.array(st_d["ms_stage"][:7]) / 3
    finally:
        del os.environ["AD_STAGE_EVENTS"]
    torch.cuda.synchronize(dev)

    # roofline of the dominant kernel: the K1+K2 resolve of every request, which runs as lean pass 1,
    # lean pass 2 and the general fused kernel on what they deferred (SURVEY §8(d) compulsory bytes
    # of config 2 over the sum of their HIP-event times)
    sbytes = stage_bytes(w, stats)
    res_ms = float(sum(stage_ms[i] for i in RESOLVE_STAGES))
    achieved = sbytes[0] / (res_ms / 1000.0) / 1e9 if res_ms > 0 else 0.0
    res_kernels = resolve_kernels(stats, split_ms)
    traffic, traffic_src = measured_traffic(res_kernels, "mix" if mix else "config%d" % cfg)   # the same workload's profile
    xdesc = ""
    if world > 1:
        xdesc = (", per-store partials exchanged over RCCL inside libaccord_deps (ad_exchange) + K3 merge on the owning GPU"
                 if use_x else ", per-store partials exchanged over gloo staged through host memory (rehearsal: ranks "
                 "share GPUs) + K3 merge on the owning GPU")
    if cfg == 3:
        workload = ("config3 (%d/8 of it on %d GPU%s): %d txns over %d uniform keys, %d-txn history x 4 keys, %d-request "
                    "probe batch, token-range sharded (EvenSplit), SNAPSHOT, 1 CommandStore per GPU%s" %
                    (world, world, "s" if world > 1 else "", int(w.params["n_txns"]), int(w.params["n_keys"]),
                     int(w.params["n_hist_txns"]), n_total,
                     xdesc))
    else:
        workload = ("config2 (weak-scaled per GPU): per GPU %d txns x 8 Zipf(0.99) keys over %d keys and a %d-entry "
                    "CommandsForKey history (node-wide %d txns), SNAPSHOT, 1 CommandStore per GPU%s" %
                    (int(1_000_000 * s), int(1_000_000 * s), w.cfk.n_entries, n_total,
                     xdesc) +
                    ("; request mix: %d Accepts of in-flight txns (S = executeAt, self excluded), %d PreAccepts up to %d hlc "
                     "ticks late, the rest fresh PreAccepts" % (w.params["n_accept"], w.params["n_unordered"],
                                                                args.unordered_window) if mix else ""))
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "txn-key pairs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic",
        "config": {"workload": workload, "txns_per_step": n_total, "txn_key_pairs_per_step": probes,
                   "parallelism": "store-per-gpu x%d" % world},
        "roofline": {"bound": "hbm", "kernel": " + ".join(res_kernels), "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                     "algorithmic_bytes_per_launch": sbytes[0], "launch_ms": res_ms},
        "stages_ms": {STAGES[i]: round(float(split_ms[i]), 4) for i in range(7)},
        "stages_note": "per-kernel split from 3 steps after the timed region (AD_STAGE_EVENTS=1); the timed steps "
                       "record only the resolve's start and end (resolve %.4f ms per step)" % res_ms,
        "pairs_out": {A.MAP_NAMES[m]: int(stats["n_pairs"][m]) for m in range(3)},
        "deferred": {"lean_pass1_to_pass2": int(stats.get("n_lean_pass2", 0)),
                     "lean_to_general": int(stats.get("n_deferred_lean", 0)), "to_split": int(stats["n_deferred"])},
        "ingest_ms": ingest_ms,
    }
    if node_x is None and world == 1:
        # the output contract of the timed steps, and the packed layout's cost beside it
        r = last["res"]
        out["config"]["output"] = ("regions (AD_REGIONS): each request's keyDeps / rangeDeps / directKeyDeps written once "
                                   "where the kernels build them, plus per-request sizes and packed offsets"
                                   if args.output == "regions" else "packed arrays (request order)")
        out["regions_bytes"] = {"in_use": int(r.regions_bytes), "payload": int(r.region_bytes)}
        other = "packed" if args.output == "regions" else "regions"
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(5):
            store.deps_batch_device(qdev, sp, regions=(other == "regions"))
        torch.cuda.synchronize(dev)
        out["%s_ms_per_step" % other] = 1000.0 * (time.perf_counter() - t0) / 5
    if node_x is not None or world > 1:
        out["stages_ms"]["merge (K3, owner)"] = round(merge_ms, 4)
        out["exchange"] = {"ms_export": round(xs["ms_export"], 4), "ms_move": round(xs["ms_move"], 4),
                           "ms_merge": round(xs["ms_merge"], 4), "ms_total": round(xs["ms_total"], 4),
                           "xgmi_bytes_per_step_rank0": int(xs["bytes_moved"]),
                           "xgmi_bytes_per_step_all_ranks": int(xs.get("bytes_moved_all_ranks", 0))}
    if rank == 0 and world == 1 and not args.no_cpu_baseline and node_x is None:
        # the PCIe-inclusive rate a host caller sees through ad_deps_batch (host arrays in, packed
        # host CSR arrays out; outside the timed region, never `value`)
        # ad_deps_batch_into: caller-owned pinned host arrays, sliced so that copy-out overlaps the resolve
        # of the next slice (the path INTEGRATION.md's Panama binding uses); outputs registered once
        _, _, hout = store.deps_batch_into(w.queries, materialise=False)
        reps = []
        for _ in range(3):
            t0 = time.perf_counter()
            _, _, hout = store.deps_batch_into(w.queries, out=hout, materialise=False)
            reps.append(1000.0 * (time.perf_counter() - t0))
        into_ms = float(np.median(reps))
        hout.release()
        t0 = time.perf_counter()
        store.deps_batch_stats(w.queries)
        host_ms = 1000.0 * (time.perf_counter() - t0)
        out["host_api"] = {"ms_per_batch": into_ms, "pairs_per_s": w.queries.n_probes / (into_ms / 1000.0),
                           "path": "ad_deps_batch_into (pinned caller-owned outputs; slices of 128k+ requests packed "
                                   "into pinned staging by the host pool and sent by SDMA while a kernel writes the "
                                   "previous slice's results over PCIe; keyDeps keys / k2t cross as u8 indices / u16 "
                                   "and are rebuilt by host threads), median of 3; link peaks on the box: "
                                   "scripts/mb_pcie.hip, scripts/mb_pcie2.hip (DESIGN.md section 7)",
                           "ad_deps_batch_ms": host_ms}
        # the device result of the same batch (the host-API call above reused the ctx buffers),
        # read back for the baseline's parity check
        res, _ = store.deps_batch_device(qdev, sp)
        torch.cuda.synchronize(dev)
        out["cpu_baseline"] = cpu_baseline_stores(w, args.cpu_budget, gpu_take=lambda idx: store.device_result_to_host(res, idx))
    if w.queries.range_off is not None:
        out["config"]["range_requests"] = int(np.count_nonzero(np.diff(w.queries.range_off.astype(np.int64))))
    if rank == 0:
        print(json.dumps(out), flush=True)
    store.close()
    if world > 1:
        dist.destroy_process_group()

if __name__ == "__main__":
    main()
