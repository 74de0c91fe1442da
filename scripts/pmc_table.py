"""Per-kernel sums of every counter in a pmc_lean-style output directory (p1..pN passes).
Usage: python scripts/pmc_table.py gpurun_out/pmc_lean_TAG [kernel-substring ...]"""
import collections
import csv
import glob
import os
import sys


def short(name):
    return name.split("(")[0].replace("void ", "").replace("adx::", "")


def main(d, pats):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    calls = collections.defaultdict(set)
    for f in sorted(glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            if pats and not any(p in k for p in pats):
                continue
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            calls[(k, r["Counter_Name"])].add(r.get("Dispatch_Id", ""))
    for k, c in agg.items():
        print(k)
        for n, v in sorted(c.items()):
            print("   %-36s %16.0f  (per launch %14.0f)" % (n, v, v / max(1, len(calls[(k, n)]))))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
