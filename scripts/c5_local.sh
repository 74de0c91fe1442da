#!/bin/bash
# config-5 leveling: the XCD-local dataflow (AD_LEVELS_LOCAL) over residency against the fabric one
set -o pipefail
mkdir -p gpurun_out
run() {
  timeout -k 10 120 python -u bench.py --config 5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/c5l.log 2>&1 || exit 1
  echo "$1 $(python3 -c "import json,sys; r=json.loads(open('gpurun_out/c5l.log').read().strip().splitlines()[-1]); print(r['ms_per_step'], r['stages_ms'])")"
}
AD_LEVELS_LOCAL=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_levels.py > gpurun_out/c5l_tests.log 2>&1 || { tail -30 gpurun_out/c5l_tests.log; exit 1; }
tail -2 gpurun_out/c5l_tests.log
run fabric-64x1
AD_LEVELS_PULL_PER_CU=2 run fabric-64x2
AD_LEVELS_PULL_THREADS=256 run fabric-256x1
for cfg in "256 1" "256 2" "256 4" "64 8"; do
  set -- $cfg
  AD_LEVELS_LOCAL=1 AD_LEVELS_PULL_THREADS=$1 AD_LEVELS_PULL_PER_CU=$2 run local-$1x$2
done
AD_LEVELS_LOCAL=1 AD_LEVELS_PULL_NAPS=0 run local-256x2-nap0
AD_LEVELS_LOCAL=1 AD_LEVELS_PULL_NAPS=4 run local-256x2-nap4
