#!/usr/bin/env python3
"""Store upkeep cost on a config-2 store: a RedundantBefore advance in place
(ad_redundant_advance: watermark dictionary growth + device truncation) against the rebuild a full
ad_redundant_load costs (the whole snapshot rebuilt from the host copies, then truncated).

  python scripts/bench_upkeep.py [--hist 16000000 --keys 1000000 --txns 200000 --advances 4]

Prints one JSON line per measurement and a summary line."""
import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cassandra-accord_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

from accord_deps import native, synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--hist", type=int, default=16_000_000)
    ap.add_argument("--keys", type=int, default=1_000_000)
    ap.add_argument("--txns", type=int, default=200_000)
    ap.add_argument("--entries", type=int, default=64, help="RedundantBefore entries")
    ap.add_argument("--advances", type=int, default=4)
    ap.add_argument("--registry", action="store_true", help="range-command registry upkeep on config 4 instead")
    ap.add_argument("--rows", type=int, default=1000, help="registry rows per upkeep batch")
    a = ap.parse_args()
    if a.registry:
        return registry(a)
    t0 = time.time()
    w = synth.with_redundant_ranges(synth.config2(n_txns=a.txns, n_keys=a.keys, n_hist_entries=a.hist), a.entries,
                                    seed=5, wm_frac=0.2)
    print("# workload %.1fs: %d entries, %d RedundantBefore entries" % (time.time() - t0, w.cfk.n_entries,
                                                                        len(w.redundant.range_start)), flush=True)
    hist = int(synth._hlc(w.cfk.txn).max())
    st = native.DeviceCommandStore(0)
    L = native.lib()
    try:
        t = time.time()
        st.load(w)
        load_ms = (time.time() - t) * 1e3
        print(json.dumps(dict(what="load+prepare", ms=round(load_ms, 2))), flush=True)
        red = w.redundant
        adv, reb = [], []
        for i in range(a.advances):
            red = synth.advance_redundant(red, 100 + i, step_frac=0.03, hist_hlc=hist)
            t = time.time()
            s = st.redundant_advance(red)
            ms = (time.time() - t) * 1e3
            adv.append(ms)
            print(json.dumps(dict(what="advance", step=i, ms=round(ms, 2), ms_device=round(s["ms_device"], 3),
                                  ms_dict=round(s["ms_stage"][0], 3), removed=int(s["n_keys"][0]),
                                  keys_changed=int(s["n_keys"][1]), new_ids=int(s["n_keys"][2]))), flush=True)
            # the same state through the full-replacement route: ad_redundant_load + the rebuild it forces
            t = time.time()
            st._check(L.ad_redundant_load(st.h, C.byref(red.soa())))
            st._check(L.ad_prepare(st.h))
            ms = (time.time() - t) * 1e3
            reb.append(ms)
            print(json.dumps(dict(what="redundant_load+rebuild", step=i, ms=round(ms, 2))), flush=True)
        print(json.dumps(dict(metric="redundant_before_upkeep", entries=int(w.cfk.n_entries),
                              advance_ms_median=round(sorted(adv)[len(adv) // 2], 2),
                              rebuild_ms_median=round(sorted(reb)[len(reb) // 2], 2))), flush=True)
    finally:
        st.close()


def registry(a):
    """config 4 (100k range commands over 1M keys): ad_range_cmds_update batches of `rows` registrations / unions /
    erasures / historical merges against the ad_range_cmds_load (full rebuild) of the same registry."""
    import refmodel
    t0 = time.time()
    w = synth.config4()
    lo, hi = int(w.cfk.keys.min()), int(w.cfk.keys.max())
    print("# config4 %.1fs: %d entries, %d range commands" % (time.time() - t0, w.cfk.n_entries, len(w.cmds.txn.msb)),
          flush=True)
    st = native.DeviceCommandStore(0)
    L = native.lib()
    try:
        st.load(w)
        cmds = w.cmds
        upd, reb = [], []
        for i in range(a.advances):
            u = synth.range_cmd_updates(cmds, 200 + i, a.rows, lo=lo, hi=hi, hlc_hi=90000, max_width=(hi - lo) // 20000)
            t = time.time()
            s = st.range_cmds_update(u)
            ms = (time.time() - t) * 1e3
            upd.append(ms)
            cmds = refmodel.range_cmds_update(cmds, u)
            print(json.dumps(dict(what="range_cmds_update", step=i, ms=round(ms, 2), ms_host=round(s["ms_stage"][0], 2),
                                  ms_refresh=round(s["ms_stage"][1], 2), registered=int(s["n_keys"][0]),
                                  range_entries=int(s["n_keys"][1]), new_ids=int(s["n_keys"][2]))), flush=True)
            t = time.time()
            st._check(L.ad_range_cmds_load(st.h, C.byref(cmds.soa())))
            st._check(L.ad_prepare(st.h))
            ms = (time.time() - t) * 1e3
            reb.append(ms)
            print(json.dumps(dict(what="range_cmds_load+rebuild", step=i, ms=round(ms, 2))), flush=True)
        print(json.dumps(dict(metric="range_registry_upkeep", rows=a.rows, commands=int(len(cmds.txn.msb)),
                              update_ms_median=round(sorted(upd)[len(upd) // 2], 2),
                              rebuild_ms_median=round(sorted(reb)[len(reb) // 2], 2))), flush=True)
    finally:
        st.close()


if __name__ == "__main__":
    main()
