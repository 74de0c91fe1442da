#!/bin/bash
# Round-end rehearsal on one GPU box: every -m gpu test, smoke(), then the default bench line
# (with the CPU baseline). Stops at the first step that does not end normally.
set -o pipefail
TAG=${1:-x}
timeout -k 10 700 python -u -m pytest tests/ -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1
rc=$?; echo tests=$rc; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
rc=$?; echo smoke=$rc; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$TAG.log 2>&1
rc=$?; echo bench=$rc; exit $rc
