#!/bin/bash
# Lab + parity: the in-tree library against the variants named in LAB (scripts/lean_lab.py), then the
# lean-path parity tests (stops at a crash, abort or time limit).
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-lab}
crashed() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 300 python -u scripts/lean_lab.py --steps 20 ${REGIONS:+--regions} ${CONFIG:+--config $CONFIG} $LAB > gpurun_out/lab_${TAG}.log 2>&1
rc=$?; echo lab=$rc; grep "^{" gpurun_out/lab_${TAG}.log; crashed $rc && exit 8
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_ranges.py tests/test_gpu_multi.py} > gpurun_out/t_${TAG}.log 2>&1
rc=$?; echo tests=$rc; tail -3 gpurun_out/t_${TAG}.log
