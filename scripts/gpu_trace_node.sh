#!/bin/bash
# kernel trace of the N-store node rehearsal. Usage: scripts/gpu_trace_node.sh TAG STORES SCALE
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/trace_$1
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT -o run -- python3 scripts/node_local_bench.py --stores $2 --scale $3 --steps 3 --warmup 1 > $OUT/trace.log 2>&1
rc=$?; echo trace=$rc; exit $rc
