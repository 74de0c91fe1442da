#!/bin/bash
# config 4's wide range round: its parity (full size sampled + dense scaled, every range test), then the bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py -k config4 -x -q --timeout 300 --timeout-method thread > gpurun_out/r5w_t1.log 2>&1 || { tail -30 gpurun_out/r5w_t1.log; exit 1; }
tail -1 gpurun_out/r5w_t1.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_ranges.py tests/test_golden.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5w_t2.log 2>&1 || { tail -30 gpurun_out/r5w_t2.log; exit 2; }
tail -1 gpurun_out/r5w_t2.log
bash scripts/gpu_ab.sh r5w_c4 "--config 4" -
