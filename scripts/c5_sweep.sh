#!/bin/bash
# config-5 leveling schemes: the CSR dataflow (default) over residency, the frontier loop
set -o pipefail
mkdir -p gpurun_out
run() {
  timeout -k 10 120 python -u bench.py --config 5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/c5s.log 2>&1 || exit 1
  echo "$1 $(python3 -c "import json,sys; r=json.loads(open('gpurun_out/c5s.log').read().strip().splitlines()[-1]); print(r['ms_per_step'], r['stages_ms'], r['edges'])")"
}
run csr-64x1
AD_LEVELS_PULL_THREADS=128 run csr-128x1
AD_LEVELS_PULL_PER_CU=2 run csr-64x2
AD_LEVELS_FRONTIER=1 run frontier
