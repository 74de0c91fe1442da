"""Multi-GPU path: one CommandStore per GPU, per-store partials exchanged over RCCL and merged
on the GPU that owns each request.

Reference shape: a node's key space is split into contiguous range slices, one CommandStore each
(CommandStores.java:453-471, ShardDistributor.EvenSplit.split ShardDistributor.java:106-156); a
PreAccept is sent to every store owning one of its keys, each computes its PartialDeps
(PreAccept.calculatePartialDeps, PreAccept.java:245-267) and the results are reduced with
PartialDeps.with (CommandStores.mapReduce :576-593, PreAccept.reduce PreAccept.java:140-156).

Here rank g of `world` owns token slice g. One step:
  1. resolve the local batch (requests touching slice g) on the GPU        (ad_deps_batch_device)
  2. export the non-empty maps as parts, grouped by owning rank            (ad_parts_export)
  3. all-to-all of part counts, then of hdr / keys / ids / k2t             (RCCL via torch.distributed)
  4. K3: merge the parts of the owned requests                             (ad_parts_merge)
Request t (global index) is owned by rank `owner(t)`: contiguous blocks of the global batch.

The exchange protocol (`ShardExchange`) is independent of where parts come from: the product
engine is `GpuEngine` (libaccord_deps); the CPU tests drive the same protocol over gloo with a
CPU engine built on the oracle.
"""
import numpy as np
import torch
import torch.distributed as dist

from . import _abi as A
from .model import Queries


def owner_bases(n_total, world):
    """First global request index owned by each rank (+ n_total): contiguous blocks."""
    return [(d * n_total) // world for d in range(world)] + [n_total]


def route(queries, lo, hi, start_inclusive=False):
    """The requests a store owning the token slice from lo to hi receives, with their keys
    restricted to the slice (mapReduceForKey skips keys the store does not own,
    InMemoryCommandStore.java:280; CommandStores.mapReduce only asks stores that intersect).
    Returns (local Queries, global request index int64 ascending)."""
    k = queries.keys
    sel = ((k >= lo) & (k < hi)) if start_inclusive else ((k > lo) & (k <= hi))
    cs = np.zeros(len(k) + 1, np.int64)
    np.cumsum(sel, out=cs[1:])
    ko = queries.key_off.astype(np.int64)
    counts = cs[ko[1:]] - cs[ko[:-1]]
    touch = counts > 0
    ro = rs = re_ = None
    if queries.range_off is not None:
        # a Range-domain request goes to every store whose slice one of its ranges intersects, ranges
        # unchanged (the store slices them, InMemoryCommandStore.java:291)
        hit = np.maximum(queries.range_start, lo) < np.minimum(queries.range_end, hi)
        rc = np.zeros(len(hit) + 1, np.int64)
        np.cumsum(hit, out=rc[1:])
        roff = queries.range_off.astype(np.int64)
        touch |= (rc[roff[1:]] - rc[roff[:-1]]) > 0
    idx = np.nonzero(touch)[0].astype(np.int64)
    key_off = np.zeros(len(idx) + 1, np.uint64)
    key_off[1:] = np.cumsum(counts[idx])
    me = None if queries.min_epoch is None else queries.min_epoch[idx]
    if queries.range_off is not None:
        ro, (rs, re_) = Queries._gather(queries.range_off, [queries.range_start, queries.range_end], idx)
    return Queries(queries.txn.take(idx), queries.exec.take(idx), key_off, k[sel], me, ro, rs, re_), idx


def build_global_dict(dicts):
    """The global TxnId dictionary of a multi-store exchange: the ascending, duplicate-free union in
    Timestamp order (msb unsigned, then (lsb >>> 16, identity flags) unsigned, then node signed;
    Timestamp.compareTo / equals) of every store's dictionary (DeviceCommandStore.dictionary()),
    the raw fields of an id taken from the first store holding it. Ingest-time work, run
    identically on every rank. `dicts`: list of Tids in store order. Returns Tids."""
    from .model import Tids
    msb = np.concatenate([np.asarray(d.msb, np.uint64) for d in dicts]) if dicts else np.zeros(0, np.uint64)
    lsb = np.concatenate([np.asarray(d.lsb, np.uint64) for d in dicts]) if dicts else np.zeros(0, np.uint64)
    node = np.concatenate([np.asarray(d.node, np.int32) for d in dicts]) if dicts else np.zeros(0, np.int32)
    lo = ((lsb >> np.uint64(16)) << np.uint64(4)) | ((lsb >> np.uint64(1)) & np.uint64(0xF))
    src = np.concatenate([np.full(len(d.msb), i, np.int64) for i, d in enumerate(dicts)]) if dicts else \
        np.zeros(0, np.int64)
    order = np.lexsort((src, node, lo, msb))          # last key primary; equal ids: earliest store first
    m, l_, n_ = msb[order], lo[order], node[order]
    first = np.ones(len(order), bool)
    first[1:] = (m[1:] != m[:-1]) | (l_[1:] != l_[:-1]) | (n_[1:] != n_[:-1])
    keep = order[first]
    return Tids(msb[keep].copy(), lsb[keep].copy(), node[keep].copy())


class PartsBuffers:
    """Growable device arrays in the ad_parts transport format (ids as {msb, lsb, node} int64
    triplets, or as uint32 global ranks when `rank_ids`)."""

    def __init__(self, device, rank_ids=False):
        self.device = device
        self.rank_ids = rank_ids
        self.hdr = self.keys = self.ids = self.k2t = None
        self.ensure(1, 1, 1, 1)

    @property
    def id_mult(self):
        return 1 if self.rank_ids else 3

    def ensure(self, parts, key_words, ids, k2t):
        def grow(t, n, dtype):
            if t is None or t.numel() < n or t.dtype != dtype:
                return torch.empty(max(int(n * 1.25), 16), dtype=dtype, device=self.device)
            return t
        self.hdr = grow(self.hdr, 4 * parts, torch.int64)
        self.keys = grow(self.keys, key_words, torch.int64)
        self.ids = grow(self.ids, self.id_mult * ids, torch.int32 if self.rank_ids else torch.int64)
        self.k2t = grow(self.k2t, k2t, torch.int32)

    def soa(self, n=None):
        p = A.AdParts()
        p.hdr, p.keys, p.ids, p.k2t = (self.hdr.data_ptr(), self.keys.data_ptr(), self.ids.data_ptr(),
                                       self.k2t.data_ptr())
        p.cap_parts = self.hdr.numel() // 4
        p.cap_key_words = self.keys.numel()
        p.cap_ids = self.ids.numel() // self.id_mult
        p.cap_k2t = self.k2t.numel()
        p.id_format = A.AD_IDS_RANK if self.rank_ids else A.AD_IDS_TRIPLET
        if n is not None:
            p.n_parts, p.n_key_words, p.n_ids, p.n_k2t = (int(x) for x in n)
        return p


class GpuEngine:
    """Product engine: a DeviceCommandStore with its local batch resident in HBM."""

    def __init__(self, store, qdev, txn_index, device, stream=None, parts_only=True):
        self.store = store
        self.parts_only = parts_only      # the batch result is only exported (no packed arrays)
        self.qdev = qdev
        self.device = device
        self.txn_index = torch.from_numpy(np.ascontiguousarray(txn_index, np.int64)).to(device)
        self.stream = stream
        self.send = PartsBuffers(device)
        self.recv = PartsBuffers(device)
        self.last_stats = None

    @property
    def id_mult(self):
        return self.send.id_mult

    def dictionary(self):
        return self.store.dictionary()

    def set_global_dict(self, g):
        """Parts travel as uint32 global ranks from now on (ad_set_global_dict)."""
        self.store.set_global_dict(g)
        self.send = PartsBuffers(self.device, rank_ids=True)
        self.recv = PartsBuffers(self.device, rank_ids=True)

    def resolve(self):
        self.res, self.last_stats = self.store.deps_batch_device(self.qdev, self.stream, self.parts_only)

    def export(self, dest_first):
        """-> (dict of 1-D send tensors, counts[n_dest, 4] int64)."""
        while True:
            p = self.send.soa()
            rc, counts = self.store.export_parts(self.res, self.txn_index.data_ptr(), dest_first, p, self.stream)
            if rc == A.AD_OK:
                break
            self.send.ensure(p.n_parts, p.n_key_words, p.n_ids, p.n_k2t)
        return dict(hdr=self.send.hdr, keys=self.send.keys, ids=self.send.ids, k2t=self.send.k2t), \
            counts.astype(np.int64)

    def recv_buffers(self, totals):
        self.recv.ensure(*totals)
        return dict(hdr=self.recv.hdr, keys=self.recv.keys, ids=self.recv.ids, k2t=self.recv.k2t)

    def merge(self, totals, src_parts, txn_base, n_owned):
        return self.store.merge_parts(self.recv.soa(totals), src_parts, txn_base, n_owned, self.stream)


def _units(id_mult):
    """element multiplicity of each transport array per counted unit"""
    return (("hdr", 4), ("keys", 1), ("ids", id_mult), ("k2t", 1))


class ShardExchange:
    """The all-to-all + merge protocol of one rank."""

    def __init__(self, engine, txn_index, n_total, rank, world, group=None, count_device=None, stage_cpu=False):
        self.engine = engine
        self.stage_cpu = stage_cpu          # gloo over device buffers: payload staged through host memory
        self.rank, self.world = rank, world
        self.group = group
        bases = owner_bases(n_total, world)
        self.txn_base = bases[rank]
        self.n_owned = bases[rank + 1] - bases[rank]
        ti = np.asarray(txn_index, np.int64)
        if len(ti) > 1 and not np.all(ti[1:] > ti[:-1]):
            raise ValueError("local requests must be in ascending global order")
        self.dest_first = np.searchsorted(ti, np.asarray(bases[:world] + [n_total], np.int64)).astype(np.uint64)
        self.dest_first[-1] = len(ti)
        self.count_device = count_device

    def install_global_dict(self):
        """Ingest-time collective (once per snapshot): gather every store's dictionary, build the
        global one identically on every rank and install it, so that the per-step all-to-all moves
        4-byte id ranks instead of 24-byte ids and K3 merges integers."""
        mine = self.engine.dictionary()
        got = [None] * self.world
        dist.all_gather_object(got, (mine.msb, mine.lsb, mine.node), group=self.group)
        from .model import Tids
        g = build_global_dict([Tids(*t) for t in got])
        self.engine.set_global_dict(g)
        return len(g.msb)

    def step(self):
        e = self.engine
        e.resolve()
        send, counts = e.export(self.dest_first)                      # counts[d] = parts, words, ids, k2t
        dev = self.count_device
        sc = torch.from_numpy(counts.reshape(-1).copy())
        rc = torch.empty_like(sc)
        if dev is not None:
            sc, rc = sc.to(dev), rc.to(dev)
        dist.all_to_all_single(rc, sc, group=self.group)
        rcounts = rc.cpu().numpy().reshape(self.world, 4)
        totals = rcounts.sum(axis=0)
        recv = e.recv_buffers(totals)
        for a, (name, mult) in enumerate(_units(getattr(e, "id_mult", 3))):
            in_splits = [int(x) * mult for x in counts[:, a]]
            out_splits = [int(x) * mult for x in rcounts[:, a]]
            si = send[name][:sum(in_splits)]
            ro = recv[name][:sum(out_splits)]
            if self.stage_cpu and ro.is_cuda:
                rh = torch.empty(ro.shape, dtype=ro.dtype)
                dist.all_to_all_single(rh, si.cpu(), out_splits, in_splits, group=self.group)
                ro.copy_(rh)
            else:
                dist.all_to_all_single(ro, si, out_splits, in_splits, group=self.group)
        return e.merge(totals, rcounts[:, 0], self.txn_base, self.n_owned)


class NodeExchange:
    """The multi-GPU step on the library's own transport (accord_deps.h ad_exchange): one process per
    GPU, an RCCL communicator inside libaccord_deps over the node's stores (rank = slice order); per
    step the store resolves its local batch (parts only), then ad_exchange exports, moves (RCCL
    grouped send/recv over xGMI) and merges (K3) the requests this rank owns. torch.distributed is only
    the out-of-band channel for the communicator id and the ingest-time global dictionary."""

    def __init__(self, store, qdev, txn_index, n_total, rank, world, device, stream=None, group=None):
        import torch
        self.store, self.qdev, self.rank, self.world, self.stream = store, qdev, rank, world, stream
        bases = owner_bases(n_total, world)
        self.txn_base = bases[rank]
        self.n_owned = bases[rank + 1] - bases[rank]
        ti = np.asarray(txn_index, np.int64)
        self.dest_first = np.searchsorted(ti, np.asarray(bases[:world], np.int64)).astype(np.uint64).tolist() + [len(ti)]
        self.ti = torch.from_numpy(np.ascontiguousarray(ti)).to(device)
        from . import native
        uid = [native.comm_unique_id() if rank == 0 else None]
        if world > 1:
            dist.broadcast_object_list(uid, src=0, group=group)
        store.comm_init(uid[0], rank, world)
        self.last_stats = None
        self.last_exchange = None

    def step(self):
        res, self.last_stats = self.store.deps_batch_device(self.qdev, self.stream, parts_only=True)
        self.last_res = res
        mg, self.last_exchange = self.store.exchange(res, self.ti.data_ptr(), self.dest_first, self.txn_base,
                                                     self.n_owned, self.stream)
        return mg
