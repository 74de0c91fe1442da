#!/bin/bash
# range expansion by waves: the Range-domain and recovery parity, then the mixed-batch bench lines
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ranges.py tests/test_gpu_recovery.py tests/test_gpu_recovery_live.py tests/test_golden.py tests/test_gpu_host_api.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5x_t.log 2>&1 || { tail -30 gpurun_out/r5x_t.log; exit 1; }
tail -1 gpurun_out/r5x_t.log
bash scripts/gpu_ab.sh r5x_c2r "--range-frac 0.01" - && bash scripts/gpu_ab.sh r5x_c4r "--config 4 --range-frac 0.01" -
