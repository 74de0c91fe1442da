#!/bin/bash
# round rehearsal (tests, smoke, default bench) then a kernel trace of the f1 update bench
set -o pipefail
bash scripts/gpu_round.sh r1c || exit $?
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_f1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_f1/trace -o run -- python3 bench.py --cfk-update 1000000 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_f1/trace.log 2>&1
echo prof=$?
