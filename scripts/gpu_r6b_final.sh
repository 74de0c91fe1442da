#!/bin/bash
# Round-6 (second session) evidence: rocprofv3 profiles of the final tree (B1, B2), then the bench lines of every config (A) whose
# roofline traffic comes from those profiles (commit the summaries between B and A).
#   bash scripts/gpu_r6b_final.sh B1|B2|A|C
set -o pipefail
mkdir -p gpurun_out
B="timeout -k 10 300 python -u bench.py --no-cpu-baseline"
line() { grep '^{' "$1" | tail -1 > "${1%.log}.json"; head -c 400 "${1%.log}.json"; echo; }
for part in "$@"; do
  case $part in
  B1)
    bash scripts/profile.sh r6b_config2 && bash scripts/profile.sh r6b_config4 --config 4 &&
    bash scripts/profile.sh r6b_mix --accept-frac 0.3 --unordered-frac 0.1 || exit 2 ;;
  B2)
    bash scripts/profile.sh r6b_config3x --config 3 --exchange &&
    bash scripts/profile.sh r6b_steady --steady 16384 || exit 3 ;;
  A)
    timeout -k 10 400 python -u bench.py > gpurun_out/r6bf_config2.log 2>&1 && line gpurun_out/r6bf_config2.log &&
    $B --output packed > gpurun_out/r6bf_config2_packed.log 2>&1 && line gpurun_out/r6bf_config2_packed.log &&
    $B --accept-frac 0.3 --unordered-frac 0.1 > gpurun_out/r6bf_mix.log 2>&1 && line gpurun_out/r6bf_mix.log &&
    $B --config 4 > gpurun_out/r6bf_config4.log 2>&1 && line gpurun_out/r6bf_config4.log &&
    $B --config 5 --steps 10 --warmup 2 > gpurun_out/r6bf_config5.log 2>&1 && line gpurun_out/r6bf_config5.log &&
    $B --config 3 --exchange > gpurun_out/r6bf_config3x.log 2>&1 && line gpurun_out/r6bf_config3x.log &&
    $B --steady 16384 --steps 8 --warmup 2 > gpurun_out/r6bf_steady.log 2>&1 && line gpurun_out/r6bf_steady.log || exit 1 ;;
  C)
    timeout -k 10 400 python -u scripts/emulate_config3.py --world 8 --scale 0.25 --steps 5 > gpurun_out/r6bf_emulate_config3_w8.log 2>&1 &&
    tail -5 gpurun_out/r6bf_emulate_config3_w8.log || exit 4 ;;
  esac
done
