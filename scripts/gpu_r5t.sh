#!/bin/bash
# round 5: the Range-domain edge-case tests, then the W = 8 node emulation on the final tree
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ranges.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r5t_ranges.log 2>&1 || { tail -30 gpurun_out/r5t_ranges.log; exit 1; }
tail -1 gpurun_out/r5t_ranges.log
timeout -k 10 400 python -u scripts/emulate_config3.py --world 8 --scale 0.25 --steps 5 > gpurun_out/r5t_emulate_w8.log 2>&1 || { tail -20 gpurun_out/r5t_emulate_w8.log; exit 2; }
tail -1 gpurun_out/r5t_emulate_w8.log | cut -c1-400
