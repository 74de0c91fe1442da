#!/bin/bash
# wide kernels at 5 waves per SIMD (spilling) vs 4 on config 2; batch-end wait by event spin vs
# hipStreamSynchronize; config 3 with the exchange; the multi-GPU tests; the config-2 profile
set -o pipefail
mkdir -p gpurun_out
B="timeout -k 10 300 python -u bench.py --no-cpu-baseline"
timeout -k 10 300 python -u scripts/lean_lab.py --steps 20 variants/wide5.so variants/ppt1.so variants/ppt4.so > gpurun_out/lab_wide5.log 2>&1 && grep '^{' gpurun_out/lab_wide5.log &&
$B > gpurun_out/c4_sync.log 2>&1 && grep '^{' gpurun_out/c4_sync.log | tail -1 | head -c 260 && echo &&
AD_SPIN_WAIT=1 $B > gpurun_out/c4_spin.log 2>&1 && grep '^{' gpurun_out/c4_spin.log | tail -1 | head -c 260 && echo &&
$B --config 3 --exchange > gpurun_out/c4_c3x.log 2>&1 && grep '^{' gpurun_out/c4_c3x.log | tail -1 > gpurun_out/c4_c3x.json && head -c 260 gpurun_out/c4_c3x.json && echo &&
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_multi.py > gpurun_out/t_c4.log 2>&1 && tail -2 gpurun_out/t_c4.log &&
bash scripts/profile.sh r4b_config2
