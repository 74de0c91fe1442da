#!/bin/bash
# round 5: range-path parity (lean ranges, ranges, fullsize config 4) + config-4 bench line and kernel trace
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-r5e}
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_ranges.py tests/test_golden.py -k "range or golden or fixture or config4" > gpurun_out/${TAG}_parity.log 2>&1 || { echo PARITY_FAIL; tail -30 gpurun_out/${TAG}_parity.log; exit 1; }
tail -1 gpurun_out/${TAG}_parity.log
timeout -k 10 300 python -u bench.py --config 4 --no-cpu-baseline > gpurun_out/${TAG}_c4.log 2>&1 || { echo BENCH_FAIL; tail -5 gpurun_out/${TAG}_c4.log; exit 2; }
grep '^{' gpurun_out/${TAG}_c4.log | tail -1 | head -c 600; echo
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_${TAG}/trace -o run -- python3 bench.py --config 4 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_trace.log 2>&1 || { echo TRACE_FAIL; exit 3; }
head -6 gpurun_out/prof_${TAG}/trace/run_kernel_stats.csv | cut -d, -f1-4
