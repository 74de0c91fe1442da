#!/bin/bash
# config 5: the packed K5 path (keys-only sorts, one walk into predecessor records) against the CSR
# path, fabric and XCD-local leveling; levels tests under both
set -o pipefail
mkdir -p gpurun_out
run() {
  timeout -k 10 120 python -u bench.py --config 5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/c5p.log 2>&1 || { tail -20 gpurun_out/c5p.log; exit 1; }
  echo "$1 $(python3 -c "import json,sys; r=json.loads(open('gpurun_out/c5p.log').read().strip().splitlines()[-1]); print(r['ms_per_step'], r['stages_ms'], r.get('edges'))")"
}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_levels.py > gpurun_out/c5p_tests.log 2>&1 || { tail -30 gpurun_out/c5p_tests.log; exit 1; }
tail -1 gpurun_out/c5p_tests.log
AD_LEVELS_LOCAL=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_levels.py > gpurun_out/c5p_tests2.log 2>&1 || { tail -30 gpurun_out/c5p_tests2.log; exit 1; }
tail -1 gpurun_out/c5p_tests2.log
AD_LEVELS_PACKED=0 run csr-fabric
run packed-fabric
AD_LEVELS_PULL_PER_CU=2 run packed-fabric-x2
AD_LEVELS_PULL_PER_CU=4 run packed-fabric-x4
AD_LEVELS_PULL_PER_CU=2 AD_LEVELS_PULL_THREADS=128 run packed-fabric-128x2
AD_LEVELS_LOCAL=1 run packed-local-256x2
AD_LEVELS_LOCAL=1 AD_LEVELS_PULL_PER_CU=4 run packed-local-256x4
