#!/usr/bin/env python3
"""Per-step export windows from scripts/export_ab.sh traces: python scripts/export_windows.py t 4 8"""
import csv
import sys

for v in sys.argv[1:]:
    for d, per in (("xab_%s" % v, 8), ("xab1_%s" % v, 1)):
        rows = list(csv.DictReader(open("gpurun_out/%s/run_kernel_trace.csv" % d)))
        ex = sorted((r for r in rows if "k_export_groups" in r["Kernel_Name"] or "k_export_tiles" in r["Kernel_Name"]),
                    key=lambda r: int(r["Start_Timestamp"]))
        w = []
        for i in range(0, len(ex) - per + 1, per):
            g = ex[i:i + per]
            w.append((max(int(r["End_Timestamp"]) for r in g) - min(int(r["Start_Timestamp"]) for r in g)) / 1e6)
        print(v, d, "windows ms", " ".join("%.4f" % x for x in w[1:]))
