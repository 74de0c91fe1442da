#!/usr/bin/env python3
"""One-GPU emulation of bench.py's N-GPU step (config 3, N/8 of BASELINE config 3, one CommandStore per
token slice): all N stores of the node live on cuda:0, each resolves its local batch (parts only) and the
library's node exchange (ad_exchange_local: the same plan, export and K3 merge as ad_exchange, device
copies instead of RCCL) combines them on the owners. Prints per-store averages of the device phases, the
request shape each store sees, and the N-GPU value this implies when the stores run in parallel (the
slowest store's resolve + its exchange share), to be read beside the driver's SCALE runs.

    python scripts/emulate_config3.py --world 8 --scale 0.25 --steps 5
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--scale", type=float, default=0.25)
    ap.add_argument("--steps", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    W = a.world
    t0 = time.time()
    parts = [synth.config3_shard(r, W, txns_per_gpu=int(8_000_000 * a.scale), keys_per_gpu=int(1_250_000 * a.scale))
             for r in range(W)]
    print("generated in %.1f s" % (time.time() - t0), file=sys.stderr, flush=True)
    g = synth.config3_global_dict(parts[0][0].params, [p[3] for p in parts])
    Q = parts[0][2]
    bases = exchange.owner_bases(Q, W)
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
        dfs.append(np.searchsorted(idx, np.asarray(bases[:W], np.int64)).astype(np.uint64).tolist() + [len(idx)])
    res_ms = np.zeros(W)
    x = dict(bytes_moved=0.0, ms_export=0.0, ms_move=0.0, ms_merge=0.0, ms_total=0.0)
    for s in range(a.steps + 1):
        results = []
        for i, (st, qdev) in enumerate(stores):
            r, stats = st.deps_batch_device(qdev, None, parts_only=True)
            results.append(r)
            if s:
                res_ms[i] += stats["ms_device"]
        torch.cuda.synchronize()
        merged, xs = native.exchange_local([st for st, _ in stores], results, tis, dfs, bases[:W],
                                           [bases[d + 1] - bases[d] for d in range(W)])
        if s:
            for k in x:
                x[k] += xs[k]
    res_ms /= a.steps
    for k in x:
        x[k] /= a.steps
    probes = sum(p[0].queries.n_probes for p in parts)
    shape = [dict(requests=len(p[0].queries), probes=int(p[0].queries.n_probes), entries=int(p[0].cfk.n_entries))
             for p in parts]
    # per store in a real N-GPU run: its resolve, then its share of export + merge (the move is xGMI)
    per_gpu_ms = float(res_ms.max()) + (x["ms_export"] + x["ms_merge"]) / W
    print(json.dumps(dict(world=W, scale=a.scale, resolve_ms=[round(v, 4) for v in res_ms], exchange=x,
                          per_gpu_ms_est=round(per_gpu_ms, 4), value_est=probes / (per_gpu_ms / 1000.0),
                          per_gpu_value_est=probes / W / (per_gpu_ms / 1000.0), shape=shape[:2])), flush=True)
    for st, _ in stores:
        st.close()


if __name__ == "__main__":
    main()
