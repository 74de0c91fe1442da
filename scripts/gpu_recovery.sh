#!/bin/bash
# Recovery scans on one GPU box: parity tests, then the --recovery bench for each scan.
set -o pipefail
TAG=${1:-x}
timeout -k 10 300 python -u -m pytest tests/test_gpu_recovery.py -x -v --timeout 120 --timeout-method thread > gpurun_out/rtests_$TAG.log 2>&1
rc=$?; echo tests=$rc; [ $rc -eq 0 ] || exit $rc
for s in 3 0 1 2; do
  timeout -k 10 300 python -u bench.py --recovery 65536 --recovery-scan $s --steps 3 --warmup 1 --cpu-budget 8 > gpurun_out/rbench_${TAG}_$s.log 2>&1
  rc=$?; echo bench$s=$rc; [ $rc -eq 0 ] || exit $rc
done
