#!/bin/bash
# Range-domain requests in the general kernel (stores with range commands, no RedundantBefore): parity, then the
# mixed config-4 line and the request mix (the general kernel's cost for key requests)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ranges.py tests/test_gpu_recovery.py tests/test_golden.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5y_t.log 2>&1 || { tail -30 gpurun_out/r5y_t.log; exit 1; }
tail -1 gpurun_out/r5y_t.log
bash scripts/gpu_ab.sh r5y_c4r "--config 4 --range-frac 0.01" - && bash scripts/gpu_ab.sh r5y_mix "--accept-frac 0.3 --unordered-frac 0.1" -
