#!/usr/bin/env python3
"""Per-request output sizes of one steady-state batch (bench.py --steady R's first step): how the pairs are spread
over requests -- the heavy tail k_build_big takes one workgroup per request for.
  python scripts/steady_sizes.py [--steady 16384]"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cassandra-accord_amd"))
from accord_deps import native, synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steady", type=int, default=16384)
    ap.add_argument("--steps", type=int, default=3, help="report the last step's batch")
    a = ap.parse_args()
    from accord_deps import _abi as A
    from accord_deps.model import CfkUpdates, Tids
    w = synth.config2(n_txns=1_000_000, n_keys=1_000_000, n_hist_entries=16_000_000, seed=0xACC0D002)
    n_b = a.steps
    stream = synth.config2_stream(w, n_b, a.steady, seed=0xACC0D5EE)
    cfk = w.cfk
    rng = np.random.default_rng(0xACC0D01E)
    key_of = np.repeat(cfk.keys, np.diff(cfk.seg.astype(np.int64)))
    status = cfk.status.copy()
    st = native.DeviceCommandStore(0)
    prev = None
    try:
        st.load(w)
        # bench.py bench_steady's steps: resolve, then register (PREACCEPTED), the previous step's APPLIED, transitions
        for b in range(n_b):
            q = stream[b]
            r = st.calculate_partial_deps(q)
            live = np.nonzero(status < A.ST_APPLIED)[0]
            e = np.sort(rng.choice(live, min(a.steady, len(live)), replace=False))
            sts = np.maximum(status[e] + 1, A.ST_ACCEPTED).astype(np.uint8)
            status[e] = sts
            rows = np.repeat(np.arange(len(q)), np.diff(q.key_off.astype(np.int64)))
            ti = q.txn.take(rows)
            parts = [(q.keys, ti, ti, np.full(len(rows), A.ST_PREACCEPTED, np.uint8)),
                     (key_of[e], cfk.txn.take(e), cfk.exec.take(e), sts)]
            if prev is not None:
                parts.append((prev[0], prev[1], prev[1], np.full(len(prev[0]), A.ST_APPLIED, np.uint8)))
            prev = (q.keys, ti)
            st.cfk_update(CfkUpdates(np.concatenate([p_[0] for p_ in parts]), Tids.concat([p_[1] for p_ in parts]),
                                     Tids.concat([p_[2] for p_ in parts]), np.concatenate([p_[3] for p_ in parts])))
    finally:
        st.close()
    # the rank span of each request's keyDeps txnIds (positions in the store's sorted ids, approximately the
    # dictionary): the room a per-request bitmap over ranks would need
    dt = np.dtype([("m", np.uint64), ("l", np.uint64), ("n", np.int32)])
    ids = np.zeros(len(cfk.txn.msb) + sum(len(x.txn.msb) for x in stream), dt)
    o = 0
    for t in [cfk.txn] + [x.txn for x in stream]:
        k = len(t.msb)
        ids["m"][o:o + k], ids["l"][o:o + k], ids["n"][o:o + k] = t.msb, t.lsb, t.node
        o += k
    ids = np.unique(ids)
    m0 = r.maps[0]
    toff = m0.txn_off.astype(np.int64)
    has = np.diff(toff) > 0
    lo_i, hi_i = toff[:-1][has], toff[1:][has] - 1
    def pos(ix):
        x = np.zeros(len(ix), dt)
        x["m"], x["l"], x["n"] = m0.txn.msb[ix], m0.txn.lsb[ix], m0.txn.node[ix]
        return np.searchsorted(ids, x)
    span = pos(hi_i) - pos(lo_i) + 1
    sz = np.diff(toff)[has]
    heavy = sz > 512
    print("dictionary ~%d ids; keyDeps rank span per request: median %d, p90 %d, p99 %d, max %d; heavy (>512 txns): "
          "median %d, p90 %d, max %d, <= 2^19: %.3f" % (len(ids), np.median(span), np.percentile(span, 90),
                                                         np.percentile(span, 99), span.max(), np.median(span[heavy]),
                                                         np.percentile(span[heavy], 90), span[heavy].max(),
                                                         (span[heavy] <= 1 << 19).mean()))
    for m, name in enumerate(["keyDeps", "rangeDeps", "directKeyDeps"]):
        k2t = np.diff(r.maps[m].k2t_off.astype(np.int64)) - np.diff(r.maps[m].keys_off.astype(np.int64))
        s = np.sort(k2t)[::-1]
        tot = int(s.sum())
        print("%s: pairs %d, max %d, >16384: %d (%d pairs), >4096: %d, >512: %d; top 1/10/100/1000 share %.3f %.3f %.3f %.3f"
              % (name, tot, s[0] if len(s) else 0, (s > 16384).sum(), s[s > 16384].sum(), (s > 4096).sum(), (s > 512).sum(),
                 s[:1].sum() / max(tot, 1), s[:10].sum() / max(tot, 1), s[:100].sum() / max(tot, 1), s[:1000].sum() / max(tot, 1)))
        print("  top 20:", s[:20].tolist())


if __name__ == "__main__":
    main()
