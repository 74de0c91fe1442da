#!/usr/bin/env python3
"""Regenerate the golden fixtures of tests/golden/ from the CPU restatement (oracle/refcpu.c).

The reference (Java) cannot run in this image (no JDK) and holds no golden vectors
of its own, so these fixtures are outputs of the oracle (round 6: regenerated when the oracle began
to restate SafeCommandStore.maybeTruncate -- the synthetic stores are now generated truncated, and the
truncate_* / recovery_truncate cases hold stores read before truncation), which is itself pinned by the
reference's known answers (PreAcceptTest, see kats.json) and ported model tests
(tests/test_oracle.py). They freeze the oracle's answers so that (a) any later change to the
oracle or the generators is caught, and (b) the GPU path is checked against committed data.

Usage: python tests/golden/make_golden.py [--all]  (writes the missing tests/golden/*.npz -- every one
       with --all -- and MANIFEST.json)
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "cassandra-accord_amd"), os.path.join(ROOT, "oracle"), HERE]

import numpy as np  # noqa: E402

import golden_io  # noqa: E402
import pyoracle  # noqa: E402
from accord_deps import synth  # noqa: E402


def deps_cases():
    """(file stem, workload, elide) — one per behaviour the reference tests exercise."""
    yield "random_small_s0", synth.random_small(1000), 1
    yield "random_small_s1_slices", synth.random_small(1001, with_slices=True), 1
    yield "random_small_s2_start_inclusive", synth.random_small(1002, start_inclusive=True), 1
    yield "random_small_s3_no_elision", synth.random_small(1003), 0
    yield "random_small_s4_big", synth.random_small(1004, n_keys=60, n_hist_txns=1500, n_txns=300, max_keys=12,
                                                    n_range_cmds=80), 1
    # stores read before truncation: every batch sees them truncated to the RedundantBefore
    # (SafeCommandStore.maybeTruncate -> CommandsForKey.withRedundantBeforeAtLeast)
    yield "truncate_snapshot", synth.random_small(1005, n_keys=40, n_hist_txns=400, n_txns=160, n_redundant=6,
                                                  truncated=False), 1
    yield "truncate_sequential", synth.sequential_ranges(1006, n_keys=40, n_hist_txns=400, n_txns=160, n_redundant=6,
                                                         range_frac=0.2, truncated=False), 1
    yield "config1_n2000", synth.config1(n_txns=2000, n_keys=200), 1
    yield "config2_small", synth.config2(n_txns=2000, n_keys=3000, n_hist_entries=40_000, esp_frac=0.05), 1
    yield "config4_small", synth.config4(n_txns=1500, n_keys=3000, n_ranges=400, n_hist_txns=3000), 1
    # Range-domain txns (sync points, ExclusiveSyncPoints, range reads / writes over Ranges): SNAPSHOT and
    # SEQUENTIAL (each registering as a range command), sliced stores, both inclusivities
    yield "ranges_snapshot_slices", synth.random_small(1010, n_keys=60, n_hist_txns=400, n_txns=160, n_range_cmds=40,
                                                       n_redundant=5, range_frac=0.5, with_slices=True), 1
    yield "ranges_snapshot_start_inclusive", synth.random_small(1011, n_keys=60, n_hist_txns=400, n_txns=160,
                                                                n_range_cmds=40, n_redundant=5, range_frac=0.5,
                                                                start_inclusive=True), 1
    yield "ranges_sequential_slices", synth.sequential_ranges(1012, n_keys=60, n_hist_txns=400, n_txns=160,
                                                              n_range_cmds=40, n_redundant=5, range_frac=0.5,
                                                              with_slices=True), 1
    yield "ranges_sequential_start_inclusive", synth.sequential_ranges(1013, n_keys=60, n_hist_txns=400, n_txns=160,
                                                                       n_range_cmds=40, n_redundant=5, range_frac=0.5,
                                                                       start_inclusive=True), 1


def recovery_cases():
    """(file stem, workload): the four BeginRecovery scans of key- and Range-domain recovering txns."""
    yield "recovery_truncate", synth.recovery_workload(1022, n_redundant=6, range_frac=0.3, truncated=False)
    yield "recovery_ranges_slices", synth.recovery_workload(1020, n_range_cmds=30, range_frac=0.5, n_txns=100,
                                                            with_slices=True)
    yield "recovery_ranges_start_inclusive", synth.recovery_workload(1021, n_range_cmds=30, range_frac=0.5,
                                                                     n_txns=100, start_inclusive=True)


def level_cases():
    g, _ = synth.config5(n_txns=20_000, n_keys=2_000)
    yield "levels_config5_n20000", g
    yield "levels_random_all_kinds", synth.random_graph(2000, n_txns=3000, n_keys=40)


def main():
    # existing fixtures are kept as committed (their hashes are part of the record); --all rewrites them
    rewrite = "--all" in sys.argv
    pyoracle.build()
    mpath = os.path.join(HERE, "MANIFEST.json")
    manifest = {} if rewrite or not os.path.exists(mpath) else json.load(open(mpath))

    def todo(stem):
        return rewrite or not os.path.exists(os.path.join(HERE, stem + ".npz")) or stem + ".npz" not in manifest

    for stem, w, elide in deps_cases():
        if not todo(stem):
            continue
        exp = pyoracle.resolve(w, elide=elide)
        d = golden_io.workload_arrays(w)
        d.update(golden_io.batch_arrays(exp))
        d["elide"] = np.array([elide], np.int32)
        path = os.path.join(HERE, stem + ".npz")
        np.savez_compressed(path, **d)
        manifest[stem + ".npz"] = dict(kind="deps", requests=len(w.queries), pairs=[exp.pair_count(m) for m in range(3)])
    for stem, w in recovery_cases():
        if not todo(stem):
            continue
        d = golden_io.workload_arrays(w)
        pairs = []
        for scan in range(4):
            exp = pyoracle.recover(w, scan)
            d.update(golden_io.batch_arrays(exp, "scan%d." % scan))
            pairs.append([exp.pair_count(m) for m in range(3)])
        path = os.path.join(HERE, stem + ".npz")
        np.savez_compressed(path, **d)
        manifest[stem + ".npz"] = dict(kind="recovery", requests=len(w.queries), pairs=pairs)
    for stem, g in level_cases():
        if not todo(stem):
            continue
        lv = pyoracle.levels(g)
        path = os.path.join(HERE, stem + ".npz")
        np.savez_compressed(path, **golden_io.graph_arrays(g, lv))
        manifest[stem + ".npz"] = dict(kind="levels", txns=len(g.kind), levels=int(lv.max()) + 1)
    for f in sorted(manifest):
        with open(os.path.join(HERE, f), "rb") as fh:
            manifest[f]["sha256"] = hashlib.sha256(fh.read()).hexdigest()
    with open(os.path.join(HERE, "MANIFEST.json"), "w") as fh:
        json.dump(manifest, fh, indent=1, sort_keys=True)
    print(json.dumps(manifest, indent=1))


if __name__ == "__main__":
    main()
