#!/bin/bash
# lean blocks-per-CU sweep on the config-2 (and config-4) bench. Usage: scripts/occ_sweep.sh TAG
set -o pipefail
TAG=${1:-x}
for pc in 3 4 5 6 7; do
  AD_LEAN_PER_CU=$pc timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/occ_${TAG}_$pc.log 2>&1 || exit 1
  AD_LEAN_PER_CU=$pc timeout -k 10 200 python -u bench.py --config 4 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/occ4_${TAG}_$pc.log 2>&1 || exit 1
done
echo sweep-done
