#!/bin/bash
# kernel trace of the N-store emulation. Usage: scripts/prof_emu.sh TAG N [scale]
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-x}; N=${2:-8}; SC=${3:-0.25}
OUT=gpurun_out/prof_emu_$TAG
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $OUT -o run -- python3 scripts/emulate_shards.py --n $N --scale $SC --steps 2 > $OUT/log.txt 2>&1
