#!/bin/bash
# Round 6: named GPU test files (fast iteration), then optionally the full suite. Logs carry a tag.
#   bash scripts/gpu_r6_tests.sh TAG "tests/test_a.py tests/test_b.py" [full]
set -o pipefail
T=$1
FILES=$2
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest $FILES -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_sel.log 2>&1 || { tail -60 gpurun_out/${T}_sel.log; exit 1; }
tail -3 gpurun_out/${T}_sel.log
if [ "$3" = "full" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_full.log 2>&1 || { tail -40 gpurun_out/${T}_full.log; exit 2; }
  tail -2 gpurun_out/${T}_full.log
fi
