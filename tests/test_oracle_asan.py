"""The CPU restatement (oracle/refcpu.c) under AddressSanitizer + LeakSanitizer + UBSan.

oracle/asan_driver.c links refcpu.c into a sanitized executable (oracle/Makefile target `asan`)
and replays a dump of oracle calls: every golden deps fixture, a sharded resolve with its
request-wise merge (rc_result_merge), the four recovery scans, preaccept and levels. Each input
array is its own heap block of exactly its size, so an out-of-bounds read of any SoA array, a
leak or undefined behaviour fails the run; each answer is folded into a hash that must equal the
same fold over the normal build's answer (oracle/librefcpu.so through pyoracle)."""
import ctypes as C
import dataclasses
import os
import struct
import subprocess
import sys

import numpy as np
import pytest

from accord_deps import _abi as A
from accord_deps import synth
from accord_deps.model import RangeMap

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(ROOT, "oracle")
DRIVER = os.path.join(ORACLE, "build", "asan_driver")
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import golden_io  # noqa: E402

OP_CREATE, OP_CFK, OP_RANGES, OP_REDUNDANT, OP_MISSING, OP_DEPS, OP_RECOVERY, OP_MERGE, OP_PREACCEPT, \
    OP_LEVELS, OP_DESTROY = range(1, 12)
MASK = (1 << 64) - 1
PRIME = 0x100000001b3


@pytest.fixture(scope="module")
def driver(oracle):
    oracle.build("asan")
    return DRIVER


# ---- the fold of asan_driver.c -------------------------------------------------------------
def fold(h, a):
    a = np.asarray(a)
    if a.dtype.kind == "i":
        u = a.astype(np.int64).view(np.uint64)
    else:
        u = a.astype(np.uint64)
    n = len(u)
    w = (2 * np.arange(n, dtype=np.uint64) + 1)
    with np.errstate(over="ignore"):
        s = int((u * w).sum(dtype=np.uint64)) if n else 0
    return (h * PRIME + s + n) & MASK


def fold_batch(b):
    h = b.n_txns
    for m, mm in enumerate(b.maps):
        h = fold(h, mm.keys_off)
        h = fold(h, mm.keys)
        if m == A.AD_MAP_RANGE:
            h = fold(h, mm.keys_end if mm.keys_end is not None else mm.keys)
        h = fold(h, mm.txn_off)
        h = fold(fold(fold(h, mm.txn.msb), mm.txn.lsb), mm.txn.node)
        h = fold(h, mm.k2t_off)
        h = fold(h, mm.k2t)
    return h


# ---- dump writer ---------------------------------------------------------------------------
def _arrays(obj, out):
    if isinstance(obj, np.ndarray):
        if obj.size or obj.ctypes.data not in out:
            out[obj.ctypes.data] = max(out.get(obj.ctypes.data, 0), obj.nbytes)
    elif dataclasses.is_dataclass(obj) and not isinstance(obj, type):
        for f in dataclasses.fields(obj):
            _arrays(getattr(obj, f.name), out)
    elif isinstance(obj, (list, tuple)):
        for x in obj:
            _arrays(x, out)
    return out


class Dump:
    def __init__(self):
        self.parts = []

    def u32(self, v):
        self.parts.append(struct.pack("<I", v))

    def u64(self, v):
        self.parts.append(struct.pack("<Q", v))

    def struct(self, s, *owners):
        if s is None:
            self.u32(0)
            return
        sizes = _arrays(list(owners), {})
        raw = bytes(memoryview(s).cast("B"))
        self.u32(len(raw))
        self.parts.append(raw)
        recs = []
        for name, typ in s._fields_:
            if typ is not A.P:
                continue
            p = getattr(s, name)
            if p is None:
                continue
            assert p in sizes, "pointer field %s of %s not backed by a known array" % (name, type(s).__name__)
            recs.append((getattr(type(s), name).offset, sizes[p], C.string_at(p, sizes[p])))
        self.u32(len(recs))
        for off, nb, data in recs:
            self.parts.append(struct.pack("<IQ", off, nb) + data)

    def op(self, code, *u32s):
        self.u32(code)
        for v in u32s:
            self.u32(v)

    def store(self, w, elide=1):
        from pyoracle import make_config
        cfg, keep = make_config(w.range_start_inclusive, elide, w.slices)
        self.op(OP_CREATE)
        self.struct(cfg, keep)
        self.op(OP_CFK)
        self.struct(w.cfk.soa(), w.cfk)
        self.op(OP_RANGES)
        self.struct(w.cmds.soa(), w.cmds)
        self.op(OP_REDUNDANT)
        self.struct(w.redundant.soa(), w.redundant)
        ms = w.cfk.missing_soa()
        if ms is not None:
            self.op(OP_MISSING)
            self.struct(ms, w.cfk)

    def write(self, path):
        with open(path, "wb") as f:
            f.write(b"".join(self.parts))


def run(driver, dump, tmp_path):
    p = str(tmp_path / "calls.bin")
    dump.write(p)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1:abort_on_error=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([driver, p], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, "sanitized oracle run failed (%d):\n%s" % (r.returncode, r.stderr[-4000:])
    assert "Sanitizer" not in r.stderr, r.stderr[-4000:]
    return [(ln.split()[0], int(ln.split()[1])) for ln in r.stdout.splitlines()]


DEPS = sorted(f for f, m in golden_io.json.load(open(os.path.join(ROOT, "tests", "golden", "MANIFEST.json"))).items()
              if m["kind"] == "deps")


def test_deps_fixtures_sanitized(driver, oracle, tmp_path):
    d = Dump()
    exp = []
    for f in DEPS:
        g = golden_io.load(os.path.join(ROOT, "tests", "golden", f))
        w = golden_io.arrays_workload(g)
        elide = int(g["elide"][0])
        d.store(w, elide)
        d.op(OP_DEPS, int(w.flags))
        d.struct(w.queries.soa(), w.queries)
        d.op(OP_DESTROY)
        exp.append(("deps", fold_batch(oracle.resolve(w, elide=elide))))
    assert run(driver, d, tmp_path) == exp


def test_sharded_merge_sanitized(driver, oracle, tmp_path):
    w = synth.random_small(11)
    n = 3
    lo, hi = synth.shard_bounds(n)
    d = Dump()
    for g in range(n):
        ws = synth.slice_workload(w, lo[g], hi[g])
        d.store(ws)
        d.op(OP_DEPS, int(ws.flags))
        d.struct(ws.queries.soa(), ws.queries)
    d.op(OP_MERGE, n)
    d.op(OP_DESTROY)
    got = run(driver, d, tmp_path)
    assert [t for t, _ in got] == ["deps"] * n + ["merge"]
    assert got[-1][1] == fold_batch(oracle.resolve_sharded(w, n))


def test_recovery_preaccept_levels_sanitized(driver, oracle, tmp_path):
    d = Dump()
    exp = []
    w = synth.recovery_workload(4, with_slices=True)
    d.store(w)
    for scan in A.RECOVER_SCANS:
        d.op(OP_RECOVERY, scan)
        d.struct(w.queries.soa(), w.queries)
        exp.append(("recovery", fold_batch(oracle.recover(w, scan))))
    d.op(OP_DESTROY)
    for seed, ie in ((1, 0), (2, 1)):
        q, mc, rb = synth.preaccept_workload(seed, inclusive_ends=ie, with_reject=True)
        for permit, ep in ((1, 0), (0, 3)):
            d.op(OP_PREACCEPT, permit)
            d.u64(ep)
            d.struct(mc.soa() if mc is not None else None, mc)
            d.struct(rb.soa() if rb is not None else None, rb)
            d.struct(q.soa(), q)
            t, fl = oracle.preaccept(mc, rb, q, permit, ep)
            exp.append(("preaccept", fold(fold(fold(fold(0, t.msb), t.lsb), t.node), fl)))
    q, _, _ = synth.preaccept_workload(1)
    d.op(OP_PREACCEPT, 1)
    d.u64(0)
    empty = RangeMap.empty()
    d.struct(empty.soa(), empty)
    d.struct(None)
    d.struct(q.soa(), q)
    t, fl = oracle.preaccept(empty, None, q, 1, 0)
    exp.append(("preaccept", fold(fold(fold(fold(0, t.msb), t.lsb), t.node), fl)))
    for seed in (1, 5):
        gph = synth.random_graph(seed, n_txns=300, n_keys=20, long_runs=(seed == 5))
        d.op(OP_LEVELS)
        d.struct(gph.soa(), gph)
        exp.append(("levels", fold(0, oracle.levels(gph))))
    assert run(driver, d, tmp_path) == exp
