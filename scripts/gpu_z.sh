#!/bin/bash
# headline path after a pack / resolve change: smoke, parity (incl. full size), bench, kernel trace
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-z}
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
rc=$?; echo smoke=$rc; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/parity_$TAG.log 2>&1
rc=$?; echo parity=$rc; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.log 2>&1
rc=$?; echo bench=$rc; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_trace.sh $TAG
