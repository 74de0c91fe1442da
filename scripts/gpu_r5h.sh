#!/bin/bash
# host API: into-path tests, then the timeline lab (pipelined path and the legacy one)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_host_api.py > gpurun_out/h_tests.log 2>&1 || { tail -40 gpurun_out/h_tests.log; exit 1; }
tail -3 gpurun_out/h_tests.log
timeout -k 10 300 python -u scripts/host_api_lab.py --slices 0 4 16 > gpurun_out/h_lab.log 2>&1 || { tail -30 gpurun_out/h_lab.log; exit 2; }
grep -E "^slices|total" gpurun_out/h_lab.log | tail -24
AD_INTO_LEGACY=1 timeout -k 10 300 python -u scripts/host_api_lab.py --slices 0 --reps 2 > gpurun_out/h_lab_legacy.log 2>&1 || exit 3
grep -E "^slices" gpurun_out/h_lab_legacy.log
