#!/bin/bash
# K5 packed path: levels tests, config-5 bench line, kernel trace + PMC passes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_levels.py tests/test_golden.py > gpurun_out/k5_tests.log 2>&1 || { tail -30 gpurun_out/k5_tests.log; exit 1; }
tail -1 gpurun_out/k5_tests.log
timeout -k 10 200 python -u bench.py --config 5 --steps 20 --warmup 3 > gpurun_out/k5_bench.log 2>&1 || { tail -20 gpurun_out/k5_bench.log; exit 2; }
tail -1 gpurun_out/k5_bench.log
scripts/profile.sh r5_config5 --config 5 || exit 3
echo all-done
