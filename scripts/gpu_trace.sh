#!/bin/bash
# kernel trace (+stats) of one bench configuration. Usage: scripts/gpu_trace.sh TAG [bench args]
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-t}
shift
OUT=gpurun_out/trace_$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline "$@" > $OUT/trace.log 2>&1
rc=$?; echo trace=$rc; exit $rc
