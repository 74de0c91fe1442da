#!/bin/bash
# round 5: range recovery / SEQUENTIAL ranges tests, lean gather+build parity, bench A/B
mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_golden.py > gpurun_out/r5a_parity.log 2>&1 || { echo PARITY_FAIL; exit 1; }
$T 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_recovery.py tests/test_gpu_ranges.py tests/test_gpu_recovery_live.py > gpurun_out/r5a_tests.log 2>&1 || { echo TESTS_FAIL; exit 1; }
$T 300 python bench.py > gpurun_out/r5a_bench_gb.log 2>&1 || { echo BENCH_FAIL; exit 1; }
AD_LEAN_GB=0 $T 300 python bench.py > gpurun_out/r5a_bench_old.log 2>&1 || { echo BENCH0_FAIL; exit 1; }
echo ALL_OK
