"""Summarise a rocprofv3 profile directory (written by scripts/profile.sh) into profiles/.

Usage: python scripts/summarize_prof.py gpurun_out/prof_<tag> profiles/<round>_<tag>

Copies the kernel-stats CSV and writes <dst>.md: per kernel the average duration
(--kernel-trace --stats) and the average FETCH_SIZE / WRITE_SIZE per launch (KB as rocprofv3
reports them; on gfx950 FETCH_SIZE under-reports wide streaming reads by 2x, see
MI355X_MICROARCH.md — the corrected column doubles it).
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    n = name.split("(")[0]
    return n.replace("void ", "").replace("adx::", "")


def counters(path, counter):
    agg = defaultdict(list)
    if not os.path.exists(path):
        return agg
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] == counter:
                agg[short(row["Kernel_Name"])].append(float(row["Counter_Value"]))
    return agg


def main(src, dst):
    os.makedirs(os.path.dirname(dst) or ".", exist_ok=True)
    stats = os.path.join(src, "trace", "run_kernel_stats.csv")
    shutil.copy(stats, dst + "_kernel_stats.csv")
    fetch = counters(os.path.join(src, "pmc_fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = counters(os.path.join(src, "pmc_write", "run_counter_collection.csv"), "WRITE_SIZE")
    lines = ["# rocprofv3 summary: %s" % os.path.basename(dst), "",
             "Source: `%s` (kernel trace + stats; FETCH_SIZE and WRITE_SIZE in separate --pmc passes)." % src, "",
             "| kernel | calls | avg ms | FETCH_SIZE KB/launch | corrected read MB/launch | WRITE_SIZE KB/launch |",
             "|---|---|---|---|---|---|"]
    with open(stats) as f:
        for row in csv.DictReader(f):
            k = short(row["Name"])
            fl = fetch.get(k, [])
            wl = write.get(k, [])
            fa = sum(fl) / len(fl) if fl else None
            wa = sum(wl) / len(wl) if wl else None
            lines.append("| %s | %s | %.4f | %s | %s | %s |" % (
                k, row["Calls"], float(row["AverageNs"]) / 1e6,
                "%.0f" % fa if fa is not None else "-",
                "%.1f" % (2 * fa / 1024) if fa is not None else "-",
                "%.0f" % wa if wa is not None else "-"))
    js = {}
    for k in set(fetch) | set(write):
        fl, wl = fetch.get(k, []), write.get(k, [])
        js[k] = {"fetch_bytes_per_launch": 1024 * sum(fl) / len(fl) if fl else None,
                 "write_bytes_per_launch": 1024 * sum(wl) / len(wl) if wl else None}
    with open(dst + "_pmc.json", "w") as f:
        json.dump(js, f, indent=1, sort_keys=True)
    with open(dst + ".md", "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
