#!/bin/bash
# XCD relabel / wide pass-1 A/B on configs 2 and 3, then the lean parity tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/lean_lab.py --steps 20 --config 3 variants/noxcd.so variants/narrow1.so > gpurun_out/lab_xcd3.log 2>&1 &&
grep "^{" gpurun_out/lab_xcd3.log &&
LAB="variants/noxcd.so variants/narrow1.so" bash scripts/gpu_lab.sh xcd2
