#!/bin/bash
# round 5: lean gather+build parity (parity + golden + fullsize) then a kernel trace of the config-2 batch
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-r5c}
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_golden.py ${EXTRA_TESTS} > gpurun_out/${TAG}_parity.log 2>&1 || { echo PARITY_FAIL; tail -30 gpurun_out/${TAG}_parity.log; exit 1; }
tail -1 gpurun_out/${TAG}_parity.log
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_${TAG}/trace -o run -- python3 scripts/lean_lab.py --steps 10 > gpurun_out/${TAG}_lab.log 2>&1 || { echo LAB_FAIL; exit 2; }
grep "^{" gpurun_out/${TAG}_lab.log | head -3
head -12 gpurun_out/prof_${TAG}/trace/run_kernel_stats.csv | cut -d, -f1-4
