#!/bin/bash
# round 5: config-4 lean pass 1 variants by environment (requests per wave, residency)
mkdir -p gpurun_out
for v in "" "AD_LEAN_RPW=4" "AD_LEAN_RPW=8" "AD_RNG64=1"; do
  echo "== $v"
  env $v timeout -k 10 200 python -u scripts/lean_lab.py --config 4 --steps 10 2>/dev/null | grep '^{' | head -1 | cut -c1-300
done
