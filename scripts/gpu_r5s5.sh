#!/bin/bash
# round 5 (session 2): Range-domain requests beside the lean passes -- parity, then config 2 and config 4
# with 1 % of the requests Range-domain
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5s5_full.log 2>&1 || { tail -30 gpurun_out/r5s5_full.log; exit 1; }
tail -1 gpurun_out/r5s5_full.log
bash scripts/gpu_ab.sh r5s5_c2r "--range-frac 0.01" - && bash scripts/gpu_ab.sh r5s5_c4r "--config 4 --range-frac 0.01" - && bash scripts/gpu_ab.sh r5s5_c4 "--config 4" -
