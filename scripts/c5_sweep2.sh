#!/bin/bash
# config 5 leveling residency / polling sweep (record kernel)
set -o pipefail
mkdir -p gpurun_out
run() {
  timeout -k 10 120 python -u bench.py --config 5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/c5w.log 2>&1 || { tail -20 gpurun_out/c5w.log; exit 1; }
  echo "$1 $(python3 -c "import json,sys; r=json.loads(open('gpurun_out/c5w.log').read().strip().splitlines()[-1]); print(round(r['ms_per_step'],4), r['stages_ms'])")"
}
run x4-default
AD_LEVELS_PULL_NAPS=0 run x4-nap0
AD_LEVELS_PULL_NAPS=4 run x4-nap4
AD_LEVELS_PULL_PER_CU=8 run x8
AD_LEVELS_PULL_PER_CU=6 run x6
AD_LEVELS_LOCAL=1 AD_LEVELS_PULL_THREADS=64 AD_LEVELS_PULL_PER_CU=8 run local-64x8
AD_LEVELS_LOCAL=1 AD_LEVELS_PULL_THREADS=64 AD_LEVELS_PULL_PER_CU=8 AD_LEVELS_PULL_NAPS=0 run local-64x8-nap0
