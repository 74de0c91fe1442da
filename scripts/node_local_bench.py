"""Rehearsal of an N-GPU node on one MI355X: the N CommandStores of config3_shard(r, N) (each 1/8 of
BASELINE config 3 at --scale 1) on cuda:0, every step = each store resolves its requests (parts only)
+ the library's node exchange (ad_exchange_local: export, device copies, K3 merge on each owner).
Prints one JSON line of per-stage times. Not the bench contract (bench.py): a tool to measure the
merge with N sources on one GPU.

Usage: python scripts/node_local_bench.py --stores 8 --scale 0.25 --steps 5
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cassandra-accord_amd"))

from accord_deps import exchange, native, synth  # noqa: E402
from accord_deps.model import Tids  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stores", type=int, default=8)
    ap.add_argument("--scale", type=float, default=0.25)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    args = ap.parse_args()
    n = args.stores
    dev = torch.device("cuda", 0)
    t0 = time.time()
    parts = [synth.config3_shard(r, n, txns_per_gpu=int(8_000_000 * args.scale // n),
                                 keys_per_gpu=int(1_250_000 * args.scale // n)) for r in range(n)]
    g = synth.config3_global_dict(parts[0][0].params, [p[3] for p in parts])
    Q = parts[0][2]
    bases = exchange.owner_bases(Q, n)
    stores, keep, tis, dfs = [], [], [], []
    for w, idx, _, _ in parts:
        st = native.DeviceCommandStore(0, 0, 1, w.slices)
        st.load(w, prepare=False)
        st.set_global_dict(g)
        qdev, k = native.device_queries(w.queries, dev)
        ti = torch.from_numpy(np.ascontiguousarray(idx, np.int64)).to(dev)
        keep += [qdev, k, ti]
        stores.append((st, qdev))
        tis.append(ti.data_ptr())
        dfs.append(np.searchsorted(idx, np.asarray(bases[:n], np.int64)).astype(np.uint64).tolist() + [len(idx)])
    print("setup %.1f s: %d requests, %d stores" % (time.time() - t0, Q, n), file=sys.stderr)

    def step():
        results = []
        for st, qdev in stores:
            res, _ = st.deps_batch_device(qdev, None, parts_only=True)
            results.append(res)
        return native.exchange_local([s for s, _ in stores], results, tis, dfs, bases[:n],
                                     [bases[d + 1] - bases[d] for d in range(n)])

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    acc = {}
    merge_dev = 0.0
    t1 = time.perf_counter()
    for _ in range(args.steps):
        merged, stats = step()
        for k, v in stats.items():
            acc[k] = acc.get(k, 0.0) + v
        merge_dev += sum(m.ms_device for m in merged)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t1) / args.steps
    out = {k: v / args.steps for k, v in acc.items()}
    out.update(stores=n, requests=Q, ms_per_step=1000 * el, ms_merge_device_sum=merge_dev / args.steps,
               merge_ms_per_store=merge_dev / args.steps / n)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
