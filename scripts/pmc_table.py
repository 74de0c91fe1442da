"""Per-kernel table of the PMC passes written by scripts/pmc_r2.sh (counter values summed over the
dispatches of a kernel, averaged per dispatch). Usage: python scripts/pmc_table.py gpurun_out/pmc_<tag> [kernel-substring ...]"""
import csv
import glob
import os
import sys
from collections import defaultdict


def short(name):
    n = name.replace("(anonymous namespace)::", "").split("(")[0]
    return n.replace("void ", "").replace("adx::", "")


def main(d, filt):
    vals = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for f in glob.glob(os.path.join(d, "p*", "run_counter_collection.csv")):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = short(row["Kernel_Name"])
                if filt and not any(x in k for x in filt):
                    continue
                vals[k][row["Counter_Name"]] += float(row["Counter_Value"])
                disp[(k, row["Counter_Name"])].add(row["Dispatch_Id"])
    for k, cs in sorted(vals.items()):
        print("##", k)
        for c, v in sorted(cs.items()):
            n = max(1, len(disp[(k, c)]))
            print("  %-32s %16.0f" % (c, v / n))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
