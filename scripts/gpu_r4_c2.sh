#!/bin/bash
# Full -m gpu suite, then the headline and config-3 bench lines (adaptive lean pass-1 width, XCD relabel)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_r4_c2.log 2>&1
rc=$?; echo suite=$rc; tail -3 gpurun_out/t_r4_c2.log
case $rc in 0) ;; *) exit $rc;; esac
B="timeout -k 10 300 python -u bench.py --no-cpu-baseline"
$B > gpurun_out/r4_config2.log 2>&1 && grep '^{' gpurun_out/r4_config2.log | tail -1 > gpurun_out/r4_config2.json && head -c 600 gpurun_out/r4_config2.json && echo &&
$B --config 3 --exchange > gpurun_out/r4_config3x.log 2>&1 && grep '^{' gpurun_out/r4_config3x.log | tail -1 > gpurun_out/r4_config3x.json && head -c 300 gpurun_out/r4_config3x.json && echo
$B --accept-frac 0.3 --unordered-frac 0.1 > gpurun_out/r4_mix.log 2>&1 && grep '^{' gpurun_out/r4_mix.log | tail -1 > gpurun_out/r4_mix.json && head -c 300 gpurun_out/r4_mix.json && echo &&
$B --config 4 > gpurun_out/r4_config4.log 2>&1 && grep '^{' gpurun_out/r4_config4.log | tail -1 > gpurun_out/r4_config4.json && head -c 300 gpurun_out/r4_config4.json && echo &&
timeout -k 10 300 python -u scripts/lean_lab.py --steps 20 --config 4 --regions variants/rng4.so > gpurun_out/lab_rng4.log 2>&1 && grep '^{' gpurun_out/lab_rng4.log
