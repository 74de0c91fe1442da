#!/bin/bash
# Round-4 closing call 1: the whole -m gpu suite on the defaults, the headline bench line, its profile
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_r4e.log 2>&1
rc=$?; echo suite=$rc; tail -2 gpurun_out/t_r4e.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/r4_config2.log 2>&1 || exit 2
grep '^{' gpurun_out/r4_config2.log | tail -1 > gpurun_out/r4_config2.json; head -c 600 gpurun_out/r4_config2.json; echo
bash scripts/profile.sh r4_config2 || exit 3
echo c1-done
