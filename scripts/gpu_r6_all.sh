#!/bin/bash
# Round 6: the whole GPU suite without stopping at the first failure (one process), failures listed.
#   bash scripts/gpu_r6_all.sh TAG [extra pytest args]
set -o pipefail
T=$1
shift
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread "$@" > gpurun_out/${T}_all.log 2>&1
rc=$?
grep -E "^FAILED|^ERROR|passed|failed" gpurun_out/${T}_all.log | tail -40
exit $rc
