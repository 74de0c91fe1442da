"""(De)serialisation of golden fixtures: a workload (or waitingOn graph) and its expected output,
as flat numpy arrays in one .npz (loaded with allow_pickle=False). Test infrastructure only."""
import json

import numpy as np

from accord_deps.model import (CfkSnapshot, DepsMap, Graph, PartialDepsBatch, Queries, RangeCommands, Redundant,
                               Tids, Workload)


def _tids(d, p):
    return Tids(d[p + ".msb"], d[p + ".lsb"], d[p + ".node"])


def _put_tids(d, p, t):
    d[p + ".msb"], d[p + ".lsb"], d[p + ".node"] = t.msb, t.lsb, t.node


def _opt(d, k):
    return d[k] if k in d else None


def workload_arrays(w):
    d = {}
    c = w.cfk
    d["cfk.keys"], d["cfk.seg"], d["cfk.status"] = c.keys, c.seg, c.status
    _put_tids(d, "cfk.txn", c.txn)
    _put_tids(d, "cfk.exec", c.exec)
    if c.pruned_before is not None:
        d["cfk.pruned"] = c.pruned_before
    r = w.cmds
    _put_tids(d, "cmds.txn", r.txn)
    d["cmds.off"], d["cmds.start"], d["cmds.end"] = r.range_off, r.range_start, r.range_end
    if r.erased is not None:
        d["cmds.erased"] = r.erased
    if r.historical is not None:
        d["cmds.historical"] = r.historical
    if r.rec_status is not None:
        d["cmds.rec_status"], d["cmds.rec_has_deps"], d["cmds.rec_dep_off"] = r.rec_status, r.rec_has_deps, r.rec_dep_off
        _put_tids(d, "cmds.rec_exec", r.rec_exec)
        _put_tids(d, "cmds.rec_deps", r.rec_deps)
    if c.miss_off is not None:
        d["cfk.miss_off"] = c.miss_off
        _put_tids(d, "cfk.miss", c.miss)
    b = w.redundant
    d["rb.start"], d["rb.end"], d["rb.e0"], d["rb.e1"] = b.range_start, b.range_end, b.start_epoch, b.end_epoch
    _put_tids(d, "rb.wm", b.wm)
    q = w.queries
    _put_tids(d, "q.txn", q.txn)
    _put_tids(d, "q.exec", q.exec)
    d["q.key_off"], d["q.keys"] = q.key_off, q.keys
    if q.min_epoch is not None:
        d["q.min_epoch"] = q.min_epoch
    if q.range_off is not None:
        d["q.range_off"], d["q.range_start"], d["q.range_end"] = q.range_off, q.range_start, q.range_end
    if w.slices is not None:
        d["slices"] = np.asarray(w.slices, np.int64)
    d["meta"] = np.frombuffer(json.dumps(dict(name=w.name, flags=int(w.flags), params=w.params,
                                               range_start_inclusive=int(w.range_start_inclusive)),
                                          default=str).encode(), np.uint8)
    return d


def arrays_workload(d):
    meta = json.loads(bytes(d["meta"]).decode())
    miss = "cfk.miss_off" in d
    cfk = CfkSnapshot(d["cfk.keys"], d["cfk.seg"], _tids(d, "cfk.txn"), _tids(d, "cfk.exec"), d["cfk.status"],
                      _opt(d, "cfk.pruned"), _opt(d, "cfk.miss_off"), _tids(d, "cfk.miss") if miss else None)
    rec = "cmds.rec_status" in d
    cmds = RangeCommands(_tids(d, "cmds.txn"), d["cmds.off"], d["cmds.start"], d["cmds.end"], _opt(d, "cmds.erased"),
                         _opt(d, "cmds.historical"), _opt(d, "cmds.rec_status"), _opt(d, "cmds.rec_has_deps"),
                         _tids(d, "cmds.rec_exec") if rec else None, _opt(d, "cmds.rec_dep_off"),
                         _tids(d, "cmds.rec_deps") if rec else None)
    rb = Redundant(d["rb.start"], d["rb.end"], d["rb.e0"], d["rb.e1"], _tids(d, "rb.wm"))
    q = Queries(_tids(d, "q.txn"), _tids(d, "q.exec"), d["q.key_off"], d["q.keys"], _opt(d, "q.min_epoch"),
                _opt(d, "q.range_off"), _opt(d, "q.range_start"), _opt(d, "q.range_end"))
    return Workload(meta["name"], cfk, cmds, rb, q, flags=meta["flags"], params=meta["params"],
                    range_start_inclusive=meta["range_start_inclusive"], slices=_opt(d, "slices"))


def batch_arrays(b, prefix=""):
    d = {}
    for m, mm in enumerate(b.maps):
        p = prefix + "out%d." % m
        d[p + "keys_off"], d[p + "keys"] = mm.keys_off, mm.keys
        if mm.keys_end is not None:
            d[p + "keys_end"] = mm.keys_end
        d[p + "txn_off"], d[p + "k2t_off"], d[p + "k2t"] = mm.txn_off, mm.k2t_off, mm.k2t
        _put_tids(d, p + "txn", mm.txn)
    return d


def arrays_batch(d, prefix=""):
    maps = []
    for m in range(3):
        p = prefix + "out%d." % m
        maps.append(DepsMap(d[p + "keys_off"], d[p + "keys"], _opt(d, p + "keys_end"), d[p + "txn_off"],
                            _tids(d, p + "txn"), d[p + "k2t_off"], d[p + "k2t"]))
    return PartialDepsBatch(maps)


def graph_arrays(g, levels):
    d = {"g.kind": g.kind, "g.key_off": g.key_off, "g.keys": g.keys, "levels": levels}
    _put_tids(d, "g.exec", g.exec)
    if g.dep_off is not None:
        d["g.dep_off"], d["g.deps"] = g.dep_off, g.deps
    return d


def arrays_graph(d):
    g = Graph(_tids(d, "g.exec"), d["g.kind"], d["g.key_off"], d["g.keys"], _opt(d, "g.dep_off"), _opt(d, "g.deps"))
    return g, d["levels"]


def load(path):
    with np.load(path, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}
