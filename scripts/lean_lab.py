#!/usr/bin/env python3
"""Kernel lab for the config-2 headline batch: one process generates config 2 once, then times the
in-tree libaccord_deps.so and every variants/<name>.so given (built by scripts/build_variant.sh with
different -D flags) on the same store and batch, one after the other. Per library: per-stage HIP-event
times (ad_stats.ms_stage), ms per step, and whether a sample of its device result equals the in-tree
library's (variants that skip work for a measurement report "differs", as they should).

    python scripts/lean_lab.py [--steps 20] [--scale 1.0] variants/a.so variants/b.so ...
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cassandra-accord_amd"))

os.environ.setdefault("AD_STAGE_EVENTS", "1")     # per-kernel stage times (abi.cpp split_stages)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from accord_deps import native, synth  # noqa: E402


def run(lib, w, steps, warmup, sample, dev, regions=False):
    native._lib = None
    native.LIB_PATH = lib
    native.lib()
    st = native.DeviceCommandStore(device=0, slices=w.slices)
    try:
        st.load(w)
        qdev, keep = native.device_queries(w.queries, dev)
        sp = torch.cuda.current_stream(dev).cuda_stream
        for _ in range(warmup):
            res, stats = st.deps_batch_device(qdev, sp, regions=regions)
        torch.cuda.synchronize(dev)
        acc = np.zeros(7)
        t0 = time.perf_counter()
        for _ in range(steps):
            res, stats = st.deps_batch_device(qdev, sp, regions=regions)
            acc += np.array(stats["ms_stage"][:7])
        torch.cuda.synchronize(dev)
        ms = 1000.0 * (time.perf_counter() - t0) / steps
        got = st.device_result_to_host(res, sample)
        return dict(ms_per_step=round(ms, 4), regions=regions, regions_bytes=[int(res.regions_bytes), int(res.region_bytes)],
                    stages=[round(x / steps, 4) for x in acc],
                    pairs=[int(x) for x in stats["n_pairs"]], n_pass2=int(stats.get("n_lean_pass2", 0)),
                    n_general=int(stats.get("n_deferred_lean", 0))), got
    finally:
        st.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--config", type=int, default=2, choices=(2, 3, 4), help="2: the headline batch; 3: bench.py's N = 1 config-3 store; 4: bench.py's config 4")
    ap.add_argument("--regions", action="store_true", help="every library also timed with AD_REGIONS output")
    ap.add_argument("--only", help="time this library alone (no in-tree base run; for counter passes)")
    ap.add_argument("libs", nargs="*")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    t = time.time()
    s = a.scale
    # bench.py's batches (bench_deps for rank 0 of 1): config2_sharded, or config3_shard without the exchange
    if a.config == 4:
        w = synth.config4(n_txns=int(1_000_000 * s), n_keys=int(1_000_000 * s), n_ranges=max(1, int(100_000 * s)),
                          n_hist_txns=int(1_000_000 * s), seed=0xACC0D004)
    elif a.config == 3:
        w = synth.config3_shard(0, 1, txns_per_gpu=int(8_000_000 * s), keys_per_gpu=int(1_250_000 * s))[0]
    else:
        w, _, _ = synth.config2_sharded(0, 1, n_txns_per_gpu=int(1_000_000 * s), n_keys_per_gpu=int(1_000_000 * s),
                                        n_hist_entries_per_gpu=int(16_000_000 * s))
    print("config%d generated in %.1f s" % (a.config, time.time() - t), file=sys.stderr, flush=True)
    rng = np.random.default_rng(5)
    sample = np.unique(np.concatenate([np.arange(2000), rng.choice(len(w.queries), 4000, replace=False)]))
    base_lib = os.path.join(ROOT, "cassandra-accord_amd", "accord_deps", "libaccord_deps.so")
    ref = None
    if a.only:
        base_lib, a.libs = a.only, []
    runs = [(lib, False) for lib in [base_lib] + a.libs]
    if a.regions:
        runs += [(lib, True) for lib in [base_lib] + a.libs]
    for lib, regions in runs:
        r, got = run(lib, w, a.steps, a.warmup, sample, dev, regions)
        if ref is None:
            ref = got
            r["same_as_base"] = True
        else:
            r["same_as_base"] = bool(got.equals(ref))
        r["lib"] = os.path.basename(lib)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
