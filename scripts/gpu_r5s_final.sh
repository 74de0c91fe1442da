#!/bin/bash
# round 5 (session 2) evidence on the final tree: full GPU suite + smoke, every bench line, the
# Range-domain mixed-batch lines, the config-2 profile (trace + FETCH_SIZE + WRITE_SIZE)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5z_full.log 2>&1 || { tail -30 gpurun_out/r5z_full.log; exit 1; }
tail -1 gpurun_out/r5z_full.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5z_smoke.log 2>&1 || { tail -20 gpurun_out/r5z_smoke.log; exit 2; }
tail -1 gpurun_out/r5z_smoke.log
bash scripts/gpu_r5_final.sh A || exit 3
B="timeout -k 10 300 python -u bench.py --no-cpu-baseline"
$B --range-frac 0.01 > gpurun_out/r5f_config2_ranges.log 2>&1 && grep '^{' gpurun_out/r5f_config2_ranges.log | tail -1 > gpurun_out/r5f_config2_ranges.json || exit 4
$B --config 4 --range-frac 0.01 > gpurun_out/r5f_config4_ranges.log 2>&1 && grep '^{' gpurun_out/r5f_config4_ranges.log | tail -1 > gpurun_out/r5f_config4_ranges.json || exit 5
bash scripts/profile.sh r5z_config2 || exit 6
echo FINAL_OK
