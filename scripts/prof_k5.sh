#!/bin/bash
# Kernel traces of config 5: the onesweep sort and the per-pass sort (AD_RADIX_PER_PASS).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-k5}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_${T}_os/trace -o run -- python3 bench.py --config 5 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_${T}_os.log 2>&1 || exit 1
AD_RADIX_ONESWEEP=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_${T}_pp/trace -o run -- python3 bench.py --config 5 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_${T}_pp.log 2>&1 || exit 2
echo done
