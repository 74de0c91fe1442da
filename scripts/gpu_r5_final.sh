#!/bin/bash
# Round-5 evidence: the bench lines of every config (A), the rocprofv3 profiles behind them (B), the
# one-GPU emulation of the N = 8 config-3 node (C).
#   bash scripts/gpu_r5_final.sh A   -> gpurun_out/r5f_<name>.json lines (config 2 as the driver runs it)
#   bash scripts/gpu_r5_final.sh B   -> gpurun_out/prof_r5f_<name>/ (scripts/summarize_prof.py -> profiles/)
#   bash scripts/gpu_r5_final.sh C   -> gpurun_out/r5f_emulate_config3_w8.log
set -o pipefail
mkdir -p gpurun_out
B="timeout -k 10 300 python -u bench.py --no-cpu-baseline"
line() { grep '^{' "$1" | tail -1 > "${1%.log}.json"; head -c 300 "${1%.log}.json"; echo; }
for part in "$@"; do
  case $part in
  A)
    timeout -k 10 400 python -u bench.py > gpurun_out/r5f_config2.log 2>&1 && line gpurun_out/r5f_config2.log &&
    $B --output packed > gpurun_out/r5f_config2_packed.log 2>&1 && line gpurun_out/r5f_config2_packed.log &&
    $B --accept-frac 0.3 --unordered-frac 0.1 > gpurun_out/r5f_mix.log 2>&1 && line gpurun_out/r5f_mix.log &&
    $B --config 4 > gpurun_out/r5f_config4.log 2>&1 && line gpurun_out/r5f_config4.log &&
    $B --config 5 --steps 10 --warmup 2 > gpurun_out/r5f_config5.log 2>&1 && line gpurun_out/r5f_config5.log &&
    $B --config 3 --exchange > gpurun_out/r5f_config3x.log 2>&1 && line gpurun_out/r5f_config3x.log &&
    $B --steady 16384 --steps 8 --warmup 2 > gpurun_out/r5f_steady.log 2>&1 && line gpurun_out/r5f_steady.log || exit 1 ;;
  B)
    bash scripts/profile.sh r5f_config2 && bash scripts/profile.sh r5f_config3x --config 3 --exchange || exit 2 ;;
  C)
    timeout -k 10 400 python -u scripts/emulate_config3.py --world 8 --scale 0.25 --steps 5 > gpurun_out/r5f_emulate_config3_w8.log 2>&1 &&
    tail -5 gpurun_out/r5f_emulate_config3_w8.log || exit 3 ;;
  esac
done
