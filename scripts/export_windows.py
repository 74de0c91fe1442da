#!/usr/bin/env python3
"""Per-step windows of the export and K3-copy kernels from scripts/export_ab.sh traces (W=8 emulation:
the 8 stores' exports run concurrently, so a step's window is the cost): python scripts/export_windows.py NAME..."""
import csv
import sys


def windows(rows, pat, per):
    ex = sorted((r for r in rows if any(p in r["Kernel_Name"] for p in pat)), key=lambda r: int(r["Start_Timestamp"]))
    w = []
    for i in range(0, len(ex) - per + 1, per):
        g = ex[i:i + per]
        w.append((max(int(r["End_Timestamp"]) for r in g) - min(int(r["Start_Timestamp"]) for r in g)) / 1e6)
    return w[1:]


for v in sys.argv[1:]:
    for d, per in (("xab_%s" % v, 8), ("xab1_%s" % v, 1)):
        rows = list(csv.DictReader(open("gpurun_out/%s/run_kernel_trace.csv" % d)))
        ex = windows(rows, ("k_export_groups", "k_export_tiles"), per)
        mc = windows(rows, ("k_rmerge_copy",), 1)
        print("%-8s %-10s export %s | k3 copy (per owner) %s" % (v, d, " ".join("%.4f" % x for x in ex),
                                                               " ".join("%.4f" % x for x in mc[-per:])))
