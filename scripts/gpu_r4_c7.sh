#!/bin/bash
# K5: the level tests (incl. the lane-refilled dataflow), then config 5 with and without lane refill
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_levels.py > gpurun_out/t_c7.log 2>&1; rc=$?; echo tests=$rc; tail -2 gpurun_out/t_c7.log
case $rc in 0) ;; *) exit $rc;; esac
B="timeout -k 10 300 python -u bench.py --no-cpu-baseline --config 5 --steps 10 --warmup 2"
$B > gpurun_out/c7_c5.log 2>&1 && grep '^{' gpurun_out/c7_c5.log | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); print('wave', d['ms_per_step'], d['stages_ms'])" &&
AD_LEVELS_PULL_LANE=1 $B > gpurun_out/c7_c5l.log 2>&1 && grep '^{' gpurun_out/c7_c5l.log | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); print('lane', d['ms_per_step'], d['stages_ms'])" &&
AD_LEVELS_PULL_LANE=1 AD_LEVELS_PULL_PER_CU=2 $B > gpurun_out/c7_c5l2.log 2>&1 && grep '^{' gpurun_out/c7_c5l2.log | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); print('lane2', d['ms_per_step'], d['stages_ms'])"
timeout -k 10 300 python -u scripts/lean_lab.py --steps 20 --regions variants/packa.so > gpurun_out/lab_packa.log 2>&1 && grep '^{' gpurun_out/lab_packa.log &&
timeout -k 10 300 python -u scripts/lean_lab.py --steps 20 --config 3 variants/packa.so > gpurun_out/lab_packa3.log 2>&1 && grep '^{' gpurun_out/lab_packa3.log
