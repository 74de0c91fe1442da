#!/bin/bash
# One GPU-box round trip: parity tests (-m gpu) then a config-2 bench. Usage: scripts/gpu_check.sh TAG [bench args]
# The bench runs only if the tests ended normally (pass or ordinary failures, exit 0/1): after a
# timeout, abort or fault nothing more touches the GPU in this call.
set -o pipefail
TAG=${1:-x}; shift
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1
rc=$?
echo tests=$rc
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/bench_$TAG.log 2>&1
rc=$?
echo bench=$rc
exit $rc
