#!/bin/bash
# recovery benches (f4) then a fresh config-2 profile (trace + FETCH/WRITE passes)
set -o pipefail
for s in 3 0 1 2; do
  timeout -k 10 300 python -u bench.py --recovery 65536 --recovery-scan $s --steps 5 --warmup 2 --cpu-budget 8 > gpurun_out/rbench_r1b_$s.log 2>&1
  rc=$?; echo bench$s=$rc; [ $rc -eq 0 ] || exit $rc
done
bash scripts/profile.sh v7
