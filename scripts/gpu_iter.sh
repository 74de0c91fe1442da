#!/bin/bash
# One GPU call of an iteration: the test files named in $TESTS (default: all -m gpu), then the
# optional config-5 bench under both leveling schemes and the lean-kernel lab over variants/*.so given
# in $LAB. Stops at the first step that does not end normally.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-it}
TESTS=${TESTS:-tests/}
timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1
rc=$?; echo tests=$rc; tail -3 gpurun_out/t_$TAG.log; [ $rc -eq 0 ] || exit $rc
if [ -n "$C5" ]; then
  timeout -k 10 300 python -u bench.py --config 5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/c5_pull_$TAG.log 2>&1 || exit 3
  AD_LEVELS_FRONTIER=1 timeout -k 10 300 python -u bench.py --config 5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/c5_front_$TAG.log 2>&1 || exit 4
  tail -c 600 gpurun_out/c5_pull_$TAG.log; tail -c 300 gpurun_out/c5_front_$TAG.log
fi
if [ -n "$LAB" ]; then
  timeout -k 10 400 python -u scripts/lean_lab.py --steps 20 $LABARGS $LAB > gpurun_out/lab_$TAG.log 2>&1 || exit 5
  cat gpurun_out/lab_$TAG.log
fi
exit 0
