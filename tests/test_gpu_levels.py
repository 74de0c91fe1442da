"""GPU parity of K5 (execution-ordering levels): ad_levels / ad_levels_device vs
the CPU restatement (oracle rc_levels), bit-exact u32 level per txn."""
import numpy as np
import pytest

from accord_deps import _abi as A
from accord_deps import native, synth
from accord_deps.model import Graph, make_timestamps

pytestmark = pytest.mark.gpu


def _check(g, oracle):
    exp = oracle.levels(g)
    got, st = native.levels(g)
    assert got.shape == exp.shape
    if not np.array_equal(got, exp):
        bad = np.nonzero(got != exp)[0]
        raise AssertionError("%d of %d levels differ, first txn %d: gpu %d oracle %d" %
                             (len(bad), len(exp), bad[0], got[bad[0]], exp[bad[0]]))
    return got, st


def _scheme(monkeypatch, scheme):
    # None: the rank-ordered dataflow over a predecessor CSR (k_level_pull, default); "frontier": the
    # level-synchronous frontier loop (the two schemes the library has)
    if scheme == "frontier":
        monkeypatch.setenv("AD_LEVELS_FRONTIER", "1")


@pytest.mark.parametrize("scheme", [None, "frontier"])
@pytest.mark.parametrize("seed", range(12))
def test_random_graph_all_kinds(oracle, seed, scheme, monkeypatch):
    _scheme(monkeypatch, scheme)
    g = synth.random_graph(seed, n_txns=500 + 300 * seed, n_keys=10 + 7 * seed, long_runs=(seed % 4 == 3))
    _check(g, oracle)


@pytest.mark.parametrize("per_cu", ["1", "8"])
def test_pull_occupancy(oracle, per_cu, monkeypatch):
    # fewer and more resident waves than the default (every wait still on a lower rank)
    monkeypatch.setenv("AD_LEVELS_PULL_PER_CU", per_cu)
    monkeypatch.setenv("AD_LEVELS_PULL_THREADS", "256")
    g = synth.random_graph(17, n_txns=40_000, n_keys=300, long_runs=True)
    _check(g, oracle)


@pytest.mark.parametrize("scheme", ["frontier"])
def test_config5_full_other_schemes(oracle, scheme, monkeypatch):
    _scheme(monkeypatch, scheme)
    g, _ = synth.config5()
    got, st = _check(g, oracle)
    assert st["n_levels"] == int(got.max()) + 1


def test_many_sources_spill_path(oracle, monkeypatch):
    # 3M sources (nothing witnesses a Read on a key) and a hub with a fan-out of 60k: 2% of the later
    # Reads directly depend on txn 0
    n = 3_000_000
    rng = np.random.default_rng(7)
    hlc = np.arange(1, n + 1, dtype=np.uint64)
    ex = make_timestamps(np.ones(n, np.uint64), hlc, np.zeros(n, np.uint64), rng.integers(1, 9, n).astype(np.int32))
    key_off = np.arange(n + 1, dtype=np.uint64)
    keys = rng.integers(0, 1 << 40, n).astype(np.int64)
    hub = rng.random(n) < 0.02
    hub[0] = False
    dep_off = np.zeros(n + 1, np.uint64)
    dep_off[1:] = np.cumsum(hub)
    deps = np.zeros(int(hub.sum()), np.uint32)
    g = Graph(ex, np.zeros(n, np.uint8), key_off, keys, dep_off, deps)
    for df in (None, "frontier"):
        monkeypatch.delenv("AD_LEVELS_FRONTIER", raising=False)
        _scheme(monkeypatch, df)
        got, st = _check(g, oracle)
        assert st["n_levels"] == 2


def test_config5_scaled(oracle):
    g, _ = synth.config5(n_txns=50_000, n_keys=5_000)
    got, st = _check(g, oracle)
    assert st["n_levels"] == int(got.max()) + 1


def test_config5_full(oracle):
    # BASELINE.json config 5 at full size: 1M txns x 4 keys over 100k keys
    g, _ = synth.config5()
    got, st = _check(g, oracle)
    assert st["n_txns"] == 1_000_000 and st["n_probes"] == 4_000_000


def test_multi_block_sort_and_no_keys(oracle):
    # > 1 radix tile per pass and txns without keys / only direct deps
    g = synth.random_graph(99, n_txns=20_000, n_keys=50, max_keys=2, direct_frac=0.5)
    _check(g, oracle)


def test_device_entry_point(oracle):
    import torch
    g, _ = synth.config5(n_txns=20_000, n_keys=2_000)
    dev = torch.device("cuda", 0)
    gdev, keep = native.device_graph(g, dev)
    out = torch.zeros(len(g.kind), dtype=torch.int32, device=dev)
    st = native.DeviceCommandStore(0)
    try:
        stats = st.levels_device(gdev, out.data_ptr(), torch.cuda.current_stream(dev).cuda_stream)
        torch.cuda.synchronize(dev)
        # the device entry point leaves a usable ctx: run it twice (buffers reused)
        stats = st.levels_device(gdev, out.data_ptr(), torch.cuda.current_stream(dev).cuda_stream)
        torch.cuda.synchronize(dev)
    finally:
        st.close()
    assert np.array_equal(out.cpu().numpy().view(np.uint32), oracle.levels(g))
    assert stats["ms_device"] > 0


def test_empty_graph():
    z = np.zeros(0, np.uint64)
    g = Graph(make_timestamps(z, z, z, np.zeros(0, np.int32)), np.zeros(0, np.uint8), np.zeros(1, np.uint64),
              np.zeros(0, np.int64))
    got, st = native.levels(g)
    assert len(got) == 0 and st["n_levels"] == 0


def test_single_txn_and_no_deps(oracle):
    g = synth.random_graph(5, n_txns=1, n_keys=3, max_keys=3)
    _check(g, oracle)


def test_duplicate_execute_at_rejected():
    g = synth.random_graph(3, n_txns=50, n_keys=5)
    g.exec.msb[7], g.exec.lsb[7], g.exec.node[7] = g.exec.msb[3], g.exec.lsb[3], g.exec.node[3]
    with pytest.raises(native.AccordDepsError) as e:
        native.levels(g)
    assert e.value.code == A.AD_E_DUP_EXEC


def test_dep_out_of_range_rejected():
    g = synth.random_graph(4, n_txns=50, n_keys=5, direct_frac=0.5)
    g.deps[0] = 50
    with pytest.raises(native.AccordDepsError) as e:
        native.levels(g)
    assert e.value.code == A.AD_E_INVAL
