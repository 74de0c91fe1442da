#!/bin/bash
# batch-end wait: hipStreamSynchronize vs event spin (AD_SPIN_WAIT) on config 2; the multi-GPU / exchange tests
set -o pipefail
mkdir -p gpurun_out
B="timeout -k 10 300 python -u bench.py --no-cpu-baseline"
$B > gpurun_out/c4_sync.log 2>&1 && grep '^{' gpurun_out/c4_sync.log | tail -1 | head -c 260 && echo &&
AD_SPIN_WAIT=1 $B > gpurun_out/c4_spin.log 2>&1 && grep '^{' gpurun_out/c4_spin.log | tail -1 | head -c 260 && echo &&
$B --config 3 --exchange > gpurun_out/c4_c3x.log 2>&1 && grep '^{' gpurun_out/c4_c3x.log | tail -1 > gpurun_out/c4_c3x.json && head -c 260 gpurun_out/c4_c3x.json && echo &&
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_multi.py > gpurun_out/t_c4.log 2>&1; rc=$?; echo tests=$rc; tail -2 gpurun_out/t_c4.log
