#!/bin/bash
# config-5 kernel traces: packed path and CSR path
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/c5t_packed -o run -- python3 bench.py --config 5 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/c5t_packed.log 2>&1 || exit 1
AD_LEVELS_PACKED=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/c5t_csr -o run -- python3 bench.py --config 5 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/c5t_csr.log 2>&1 || exit 2
echo done
