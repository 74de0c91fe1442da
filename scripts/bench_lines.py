#!/usr/bin/env python3
"""One line per bench log: ms/step, roofline frac and traffic, stages. python scripts/bench_lines.py gpurun_out/b_*.log"""
import json
import sys

for f in sys.argv[1:]:
    try:
        line = [x for x in open(f).read().splitlines() if x.startswith("{")][-1]
    except (OSError, IndexError):
        print(f, "missing")
        continue
    d = json.loads(line)
    r = d.get("roofline", {})
    print(f, round(d["ms_per_step"], 4), round(r.get("frac", 0), 4), r.get("traffic"),
          {k[:24]: v for k, v in d.get("stages_ms", {}).items()}, d.get("exchange", {}).get("ms_export"))
