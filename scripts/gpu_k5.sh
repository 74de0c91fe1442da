#!/bin/bash
# K5 / radix check: the tests of every radix-sort user, then config 5 with the onesweep sort and with
# the per-pass sort (AD_RADIX_PER_PASS), then the config-2 ingest (its dictionary sort) via the bench.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-k5}
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_levels.py tests/test_gpu_ingest.py tests/test_gpu_cfk_update.py tests/test_gpu_recovery_live.py > gpurun_out/t_${TAG}.log 2>&1
rc=$?; echo tests=$rc; tail -3 gpurun_out/t_${TAG}.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u bench.py --config 5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/c5_${TAG}.log 2>&1 || exit 2
grep -o '"ms_per_step": [0-9.]*\|"stages_ms": {[^}]*}' gpurun_out/c5_${TAG}.log
AD_RADIX_ONESWEEP=1 timeout -k 10 300 python -u bench.py --config 5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/c5pp_${TAG}.log 2>&1 || exit 3
grep -o '"ms_per_step": [0-9.]*\|"stages_ms": {[^}]*}' gpurun_out/c5pp_${TAG}.log
