#!/bin/bash
# rocprofv3 kernel trace + PMC passes of the config-2 bench. Usage: scripts/profile.sh TAG [bench args]
# Writes gpurun_out/prof_TAG/ (summarise with scripts/summarize_prof.py).
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r1}
shift
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline "$@" > $OUT/trace.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -f csv -d $OUT/pmc_fetch -o run -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline "$@" > $OUT/pmc_fetch.log 2>&1 || exit 2
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -f csv -d $OUT/pmc_write -o run -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline "$@" > $OUT/pmc_write.log 2>&1 || exit 3
echo profile-done
