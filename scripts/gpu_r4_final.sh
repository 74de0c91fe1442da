#!/bin/bash
# Round-4 evidence: the bench lines of every config (A) and the rocprofv3 profiles behind them (B).
#   bash scripts/gpu_r4_final.sh A   -> gpurun_out/r4_<name>.json lines
#   bash scripts/gpu_r4_final.sh B   -> gpurun_out/prof_r4_<name>/ (scripts/summarize_prof.py -> profiles/)
set -o pipefail
mkdir -p gpurun_out
B="timeout -k 10 300 python -u bench.py --no-cpu-baseline"
line() { grep '^{' "$1" | tail -1 > "${1%.log}.json"; head -c 400 "${1%.log}.json"; echo; }
if [ "$1" = A ]; then
  $B > gpurun_out/r4_config2.log 2>&1 && line gpurun_out/r4_config2.log &&
  $B --output packed > gpurun_out/r4_config2_packed.log 2>&1 && line gpurun_out/r4_config2_packed.log &&
  $B --accept-frac 0.3 --unordered-frac 0.1 > gpurun_out/r4_mix.log 2>&1 && line gpurun_out/r4_mix.log &&
  $B --config 4 > gpurun_out/r4_config4.log 2>&1 && line gpurun_out/r4_config4.log &&
  $B --config 5 --steps 10 --warmup 2 > gpurun_out/r4_config5.log 2>&1 && line gpurun_out/r4_config5.log &&
  $B --config 3 --exchange > gpurun_out/r4_config3x.log 2>&1 && line gpurun_out/r4_config3x.log &&
  $B --steady 16384 --steps 8 --warmup 2 > gpurun_out/r4_steady.log 2>&1 && line gpurun_out/r4_steady.log
  exit $?
fi
if [ "$1" = B ]; then
  bash scripts/profile.sh r4_config2 && bash scripts/profile.sh r4_mix --accept-frac 0.3 --unordered-frac 0.1 &&
  bash scripts/profile.sh r4_config4 --config 4 && bash scripts/profile.sh r4_config5 --config 5
  exit $?
fi
