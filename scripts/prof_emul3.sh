#!/bin/bash
# Kernel trace of the W=8 config-3 emulation (scripts/emulate_config3.py, scale 0.25)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-e3}
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_${T}/trace -o run -- python3 scripts/emulate_config3.py --world 8 --scale 0.25 --steps 3 > gpurun_out/prof_${T}.log 2>&1 || exit 1
tail -2 gpurun_out/prof_${T}.log
