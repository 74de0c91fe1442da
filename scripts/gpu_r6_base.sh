#!/bin/bash
# Round-6 baseline: full GPU suite (one process) then the default bench line. Log names carry a tag so a
# failing log is never overwritten by a later passing run.
set -o pipefail
T=${1:-r6a}
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_full.log 2>&1 || { tail -40 gpurun_out/${T}_full.log; exit 1; }
tail -2 gpurun_out/${T}_full.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 > gpurun_out/${T}_bench.log 2>&1 || { tail -20 gpurun_out/${T}_bench.log; exit 2; }
tail -1 gpurun_out/${T}_bench.log
