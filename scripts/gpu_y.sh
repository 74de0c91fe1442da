#!/bin/bash
# recovery (new scan kernel) + exchange (tiled export) checks
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-y}
timeout -k 10 300 python -u -m pytest tests/test_gpu_recovery.py tests/test_gpu_multi.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ytests_$TAG.log 2>&1
rc=$?; echo tests=$rc; [ $rc -eq 0 ] || exit $rc
for s in 3 0; do
  timeout -k 10 300 python -u bench.py --recovery 65536 --recovery-scan $s --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/rbench_${TAG}_$s.log 2>&1
  rc=$?; echo bench$s=$rc; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python -u scripts/node_local_bench.py --stores 8 --scale 0.5 > gpurun_out/node8_$TAG.log 2>&1
rc=$?; echo node8=$rc; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --config 3 --exchange --no-cpu-baseline > gpurun_out/c3x_$TAG.log 2>&1
rc=$?; echo bench_c3_x=$rc; exit $rc
