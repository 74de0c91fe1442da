#!/bin/bash
# Quick GPU check after a kernel change: smoke, then the core parity tests (stops at the first failure).
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-q}
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
rc=$?; echo smoke=$rc; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multi.py tests/test_gpu_recovery.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/parity_$TAG.log 2>&1
rc=$?; echo parity=$rc; exit $rc
