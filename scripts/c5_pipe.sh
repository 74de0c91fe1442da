#!/bin/bash
# config-5 leveling with pipelined polls (AD_LEVELS_PIPE) against the default
set -o pipefail
mkdir -p gpurun_out
AD_LEVELS_PIPE=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_levels.py tests/test_golden.py > gpurun_out/c5pipe_tests.log 2>&1 || { tail -30 gpurun_out/c5pipe_tests.log; exit 1; }
tail -1 gpurun_out/c5pipe_tests.log
run() {
  timeout -k 10 120 python -u bench.py --config 5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/c5pp.log 2>&1 || { tail -20 gpurun_out/c5pp.log; exit 1; }
  echo "$1 $(python3 -c "import json,sys; r=json.loads(open('gpurun_out/c5pp.log').read().strip().splitlines()[-1]); print(round(r['ms_per_step'],4), r['stages_ms'])")"
}
run default
AD_LEVELS_PIPE=1 run pipe-x4
AD_LEVELS_PIPE=1 AD_LEVELS_PULL_NAPS=0 run pipe-x4-nap0
AD_LEVELS_PIPE=1 AD_LEVELS_PULL_PER_CU=2 run pipe-x2
AD_LEVELS_PIPE=1 AD_LEVELS_PULL_PER_CU=6 run pipe-x6
AD_LEVELS_PIPE=1 AD_LEVELS_PULL_NAPS=2 run pipe-x4-nap2
