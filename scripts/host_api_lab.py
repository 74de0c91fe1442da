"""ad_deps_batch_into on config 2 with the per-slice timeline (AD_INTO_TRACE=1): where the host-API
batch time goes. Usage: python scripts/host_api_lab.py [--slices N] [--pinned-in] [--reps R]"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cassandra-accord_amd"))
os.environ.setdefault("AD_INTO_TRACE", "1")
from accord_deps import native, synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--slices", type=int, nargs="*", default=[0])
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--scale", type=float, default=1.0)
    a = ap.parse_args()
    s = a.scale
    w, _, _ = synth.config2_sharded(0, 1, n_txns_per_gpu=int(1_000_000 * s), n_keys_per_gpu=int(1_000_000 * s),
                                    n_hist_entries_per_gpu=int(16_000_000 * s))
    store = native.DeviceCommandStore(device=0, slices=w.slices)
    store.load(w)
    for sl in a.slices:
        _, _, hout = store.deps_batch_into(w.queries, slices=sl, materialise=False)
        for r in range(a.reps):
            t0 = time.perf_counter()
            _, _, hout = store.deps_batch_into(w.queries, slices=sl, out=hout, materialise=False)
            print("slices=%d rep %d: %.3f ms" % (sl, r, 1000 * (time.perf_counter() - t0)), flush=True)
        hout.release()
    store.close()


if __name__ == "__main__":
    main()
