#!/bin/bash
# Iteration loop on one GPU box: parity (core + f1 + full size), then the headline and request-mix
# bench lines (short CPU baseline). Stops at the first failing step.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-i}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multi.py tests/test_gpu_recovery.py tests/test_gpu_cfk_update.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/parity_$TAG.log 2>&1
rc=$?; echo parity=$rc; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --cpu-budget 3 > gpurun_out/bench_$TAG.log 2>&1
rc=$?; echo bench=$rc; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --accept-frac 0.3 --unordered-frac 0.1 --cpu-budget 3 > gpurun_out/bench_mix_$TAG.log 2>&1
rc=$?; echo bench_mix=$rc; exit $rc
