#!/bin/bash
# config-5 leveling sweep of the rank-ordered dataflow: resident blocks per CU x block size (poll naps 1)
set -o pipefail
mkdir -p gpurun_out
for cfg in "1 256" "1 128" "1 64" "2 64" "4 64" "2 128"; do set -- $cfg
  AD_LEVELS_PULL_PER_CU=$1 AD_LEVELS_PULL_THREADS=$2 timeout -k 10 120 python -u bench.py --config 5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/c5s.log 2>&1 || exit 1
  echo "per_cu=$1 threads=$2 $(python3 -c "import json,sys; r=json.loads(open('gpurun_out/c5s.log').read().strip().splitlines()[-1]); print(r['ms_per_step'], r['stages_ms'])")"
done
