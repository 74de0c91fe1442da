"""Single-GPU emulation of the N-GPU config-2 step (bench.py at --gpus N) to time its device phases
per GPU without RCCL: N CommandStores (one per token slice, synth.config2_sharded) live on one
GPU; each step resolves every store's local batch, exports its parts per owner, assembles each
owner's receive buffers by device copies in source order (what the all-to-all delivers) and
merges them (K3). Prints one JSON line per N with per-store averages of each phase and the
payload an all-to-all would move.

Usage: python scripts/emulate_shards.py [--n 1 2 4 8] [--scale 0.25] [--steps 3]
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


def run(n_gpu, scale, steps, dev, rank_ids=True):
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream
    engines, idx, dest = [], [], []
    n_total = None
    t0 = time.time()
    for g in range(n_gpu):
        w, ti, n_total = synth.config2_sharded(g, n_gpu, n_txns_per_gpu=int(1_000_000 * scale),
                                               n_keys_per_gpu=int(1_000_000 * scale),
                                               n_hist_entries_per_gpu=int(16_000_000 * scale))
        st = native.DeviceCommandStore(device=dev.index, slices=w.slices)
        st.load(w)
        qdev, keep = native.device_queries(w.queries, dev)
        e = exchange.GpuEngine(st, qdev, ti, dev, stream=sp)
        e._keep = (keep, w)
        engines.append(e)
        idx.append(np.asarray(ti, np.int64))
        bases = exchange.owner_bases(n_total, n_gpu)
        df = np.searchsorted(idx[-1], np.asarray(bases[:n_gpu] + [n_total], np.int64)).astype(np.uint64)
        df[-1] = len(idx[-1])
        dest.append(df)
    if rank_ids:
        g = exchange.build_global_dict([e.dictionary() for e in engines])
        for e in engines:
            e.set_global_dict(g)
    print("N=%d: %d stores built in %.1f s" % (n_gpu, n_gpu, time.time() - t0), file=sys.stderr, flush=True)
    bases = exchange.owner_bases(n_total, n_gpu)
    acc = dict(resolve=0.0, export=0.0, assemble=0.0, merge=0.0, merge_dev=0.0)
    payload = 0
    n_req = sum(len(i) for i in idx)

    def ms(a, b):
        return a.elapsed_time(b)

    for s in range(steps + 1):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(5)]
        ev[0].record(stream)
        for e in engines:
            e.resolve()
        ev[1].record(stream)
        sends, counts = [], []
        for g, e in enumerate(engines):
            snd, c = e.export(dest[g])
            sends.append({k: v for k, v in snd.items()})
            counts.append(c)
        ev[2].record(stream)
        mult = dict(hdr=4, keys=1, ids=engines[0].id_mult, k2t=1)
        names = ("hdr", "keys", "ids", "k2t")
        recvs = []
        step_payload = 0
        for d, e in enumerate(engines):
            rc = np.stack([counts[g][d] for g in range(n_gpu)])
            totals = rc.sum(axis=0)
            rb = e.recv_buffers(totals)
            for a, nm in enumerate(names):
                at = 0
                for g in range(n_gpu):
                    start = int(counts[g][:d, a].sum()) * mult[nm]
                    cnt = int(counts[g][d, a]) * mult[nm]
                    if cnt:
                        rb[nm][at:at + cnt].copy_(sends[g][nm][start:start + cnt])
                        if g != d:
                            step_payload += cnt * rb[nm].element_size()
                    at += cnt
            recvs.append((totals, rc[:, 0]))
        ev[3].record(stream)
        mdev = 0.0
        for d, e in enumerate(engines):
            totals, src_parts = recvs[d]
            mg = e.merge(totals, src_parts, bases[d], bases[d + 1] - bases[d])
            mdev += mg.ms_device
        ev[4].record(stream)
        torch.cuda.synchronize(dev)
        if s == 0:
            continue            # warmup
        acc["resolve"] += ms(ev[0], ev[1])
        acc["export"] += ms(ev[1], ev[2])
        acc["assemble"] += ms(ev[2], ev[3])
        acc["merge"] += ms(ev[3], ev[4])
        acc["merge_dev"] += mdev
        payload += step_payload
    per = {k: round(v / steps / n_gpu, 4) for k, v in acc.items()}
    st0 = engines[0].last_stats
    out = dict(n_gpus=n_gpu, scale=scale, rank_ids=rank_ids, requests_per_store=n_req / n_gpu, probes_per_store=st0.get("n_probes"),
               ms_per_store=per, a2a_bytes_per_store=payload / steps / n_gpu,
               stages_store0=[round(x, 4) for x in st0["ms_stage"][:7]], deferred=st0.get("n_deferred_lean"))
    print(json.dumps(out), flush=True)
    for e in engines:
        e.store.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--scale", type=float, default=0.25)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--triplets", action="store_true", help="ids as {msb, lsb, node} triplets (no global dictionary)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    for n in a.n:
        run(n, a.scale, a.steps, dev, rank_ids=not a.triplets)


if __name__ == "__main__":
    main()
