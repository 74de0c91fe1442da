#!/bin/bash
# Whole -m gpu suite (no serialization), then the default bench, the steady state with recovery and
# config 5. Stops at the first step that does not end normally.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_full3.log 2>&1
rc=$?; tail -2 gpurun_out/t_full3.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/b_f3.log 2>&1 || exit 2
timeout -k 10 300 python -u bench.py --steady 16384 --steady-recovery 2 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/st_f3.log 2>&1 || exit 3
timeout -k 10 300 python -u bench.py --config 5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/c5_f3.log 2>&1 || exit 4
echo ok
