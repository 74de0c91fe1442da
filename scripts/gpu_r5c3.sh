#!/bin/bash
# four requests per wave up to 4.5 keys per request: parity (lean paths, full-size config 3 / multi), then the
# config-3 exchange line and the headline
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py tests/test_gpu_multi.py tests/test_gpu_fullsize.py tests/test_gpu_ranges.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5c3_t.log 2>&1 || { tail -30 gpurun_out/r5c3_t.log; exit 1; }
tail -1 gpurun_out/r5c3_t.log
bash scripts/gpu_ab.sh r5c3_x "--config 3 --exchange" - && bash scripts/gpu_ab.sh r5c3_c2 "" -
