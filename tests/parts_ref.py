"""Test-side restatement of the multi-GPU transport format (include/accord_deps.h, ad_parts) on
CPU arrays, and a CPU engine that drives accord_deps.exchange.ShardExchange with the oracle in
place of the GPU (world_size > 1 over gloo). TEST INFRASTRUCTURE ONLY."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "cassandra-accord_amd"))

import pyoracle  # noqa: E402
from accord_deps import _abi as A  # noqa: E402
from accord_deps.model import DepsMap, PartialDepsBatch, Tids  # noqa: E402


def encode(batch, txn_index, dest_first):
    """A PartialDepsBatch (materialised) of local requests -> (hdr, keys, ids, k2t, counts[n_dest, 4])."""
    hdr, keys, ids, k2t = [], [], [], []
    n_dest = len(dest_first) - 1
    counts = np.zeros((n_dest, 4), np.int64)
    d = 0
    for r in range(batch.n_txns):
        while r >= dest_first[d + 1]:
            d += 1
        for m in range(3):
            ks, ke, t, o = batch.maps[m].request(r)
            if len(ks) == 0:
                continue
            hdr += [(int(txn_index[r]) << 2) | m, len(ks), len(t), len(o)]
            if m == A.AD_MAP_RANGE:
                kw = np.empty(2 * len(ks), np.int64)
                kw[0::2], kw[1::2] = ks, ke
            else:
                kw = np.asarray(ks, np.int64)
            keys.append(kw)
            tr = np.empty((len(t), 3), np.int64)
            tr[:, 0] = t.msb.view(np.int64)
            tr[:, 1] = t.lsb.view(np.int64)
            tr[:, 2] = t.node
            ids.append(tr.reshape(-1))
            k2t.append(np.asarray(o, np.int32))
            counts[d] += [1, len(kw), len(t), len(o)]
    cat = lambda xs, dt: np.concatenate(xs).astype(dt) if xs else np.zeros(0, dt)  # noqa: E731
    return np.asarray(hdr, np.int64), cat(keys, np.int64), cat(ids, np.int64), cat(k2t, np.int32), counts


def decode(hdr, keys, ids, k2t, src_parts, txn_base, n_owned):
    """Received parts -> one PartialDepsBatch of the owned requests per source."""
    hdr = hdr.reshape(-1, 4)
    per_src = []
    p = kw_at = id_at = o_at = 0
    for s, np_s in enumerate(src_parts):
        rows = {m: [[] for _ in range(n_owned)] for m in range(3)}
        for _ in range(int(np_s)):
            h0, nk, ni, no = (int(x) for x in hdr[p])
            t, m = h0 >> 2, h0 & 3
            w = 2 if m == A.AD_MAP_RANGE else 1
            kw = keys[kw_at:kw_at + w * nk]
            tr = ids[3 * id_at:3 * (id_at + ni)].reshape(-1, 3)
            rows[m][t - txn_base] = (kw, tr, k2t[o_at:o_at + no])
            p += 1
            kw_at += w * nk
            id_at += ni
            o_at += no
        maps = []
        for m in range(3):
            ko, to, oo = [0], [0], [0]
            kk, ke, tm, tl, tn, oo_v = [], [], [], [], [], []
            for row in rows[m]:
                if row:
                    kw, tr, o = row
                    if m == A.AD_MAP_RANGE:
                        kk.append(kw[0::2]); ke.append(kw[1::2])
                    else:
                        kk.append(kw)
                    tm.append(tr[:, 0].view(np.uint64)); tl.append(tr[:, 1].view(np.uint64))
                    tn.append(tr[:, 2].astype(np.int32)); oo_v.append(o)
                    ko.append(ko[-1] + (len(kw) // (2 if m == A.AD_MAP_RANGE else 1)))
                    to.append(to[-1] + len(tr)); oo.append(oo[-1] + len(o))
                else:
                    ko.append(ko[-1]); to.append(to[-1]); oo.append(oo[-1])
            cat = lambda xs, dt: np.concatenate(xs).astype(dt) if xs else np.zeros(0, dt)  # noqa: E731
            maps.append(DepsMap(np.asarray(ko, np.uint64), cat(kk, np.int64),
                                cat(ke, np.int64) if m == A.AD_MAP_RANGE else None,
                                np.asarray(to, np.uint64),
                                Tids(cat(tm, np.uint64), cat(tl, np.uint64), cat(tn, np.int32)),
                                np.asarray(oo, np.uint64), cat(oo_v, np.int32)))
        per_src.append(PartialDepsBatch(maps))
    return per_src


class OracleEngine:
    """CPU engine for ShardExchange: resolve with the oracle, transport format via encode/decode,
    merge with the oracle's PartialDeps.with."""

    def __init__(self, local_workload, txn_index):
        self.w = local_workload
        self.txn_index = np.asarray(txn_index, np.int64)

    def resolve(self):
        self.res = pyoracle.resolve(self.w)

    def export(self, dest_first):
        h, k, i, o, counts = encode(self.res, self.txn_index, dest_first)
        return dict(hdr=torch.from_numpy(h), keys=torch.from_numpy(k), ids=torch.from_numpy(i),
                    k2t=torch.from_numpy(o)), counts

    def recv_buffers(self, totals):
        p, kw, ni, no = (int(x) for x in totals)
        self.recv = dict(hdr=torch.zeros(4 * p, dtype=torch.int64), keys=torch.zeros(kw, dtype=torch.int64),
                         ids=torch.zeros(3 * ni, dtype=torch.int64), k2t=torch.zeros(no, dtype=torch.int32))
        return self.recv

    def merge(self, totals, src_parts, txn_base, n_owned):
        r = {k: v.numpy() for k, v in self.recv.items()}
        per_src = decode(r["hdr"], r["keys"], r["ids"], r["k2t"], src_parts, txn_base, n_owned)
        return pyoracle.merge_batches(per_src)
