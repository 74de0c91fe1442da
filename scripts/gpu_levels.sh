#!/bin/bash
# K5 round trip: levels parity tests, config-5 bench, kernel-trace profile. Usage: scripts/gpu_levels.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-x}
timeout -k 10 300 python -u -m pytest tests/test_gpu_levels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/lvtests_$TAG.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --config 5 --steps 5 --warmup 2 > gpurun_out/lvbench_$TAG.log 2>&1 || exit 2
mkdir -p gpurun_out/prof_lv_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_lv_$TAG/trace -o run -- python3 bench.py --config 5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_lv_$TAG/trace.log 2>&1 || exit 3
echo levels-done
