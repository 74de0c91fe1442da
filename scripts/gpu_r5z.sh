#!/bin/bash
# round 5 final tree: full GPU suite + smoke, then the headline and config-4 lines
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5zz_full.log 2>&1 || { tail -30 gpurun_out/r5zz_full.log; exit 1; }
tail -1 gpurun_out/r5zz_full.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5zz_smoke.log 2>&1 || { tail -20 gpurun_out/r5zz_smoke.log; exit 2; }
tail -1 gpurun_out/r5zz_smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/r5zz_c2.log 2>&1 || exit 3
grep '^{' gpurun_out/r5zz_c2.log | tail -1 | cut -c1-400
bash scripts/gpu_ab.sh r5zz_c4 "--config 4" -
