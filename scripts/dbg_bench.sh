#!/bin/bash
# timing experiments: k_resolve with phases skipped (AD_DBG=1: no CSR build, 2: no list loads, 3: lookups only)
for d in 0 1 2 3; do
  AD_DBG=$d timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/dbg_$d.log 2>&1 || exit 1
done
echo dbg-done
