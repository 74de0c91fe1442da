#!/bin/bash
# the full suite, then the bench lines with the stage split outside the timed steps (config 4, config 3 with
# the exchange, the request mix, config 2 as the driver runs it)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_c10.log 2>&1; rc=$?; echo suite=$rc; tail -2 gpurun_out/t_c10.log
case $rc in 0) ;; *) exit $rc;; esac
B="timeout -k 10 300 python -u bench.py --no-cpu-baseline"
line() { grep '^{' "$1" | tail -1 > "${1%.log}.json"; python3 -c "import json; d=json.load(open('${1%.log}.json')); print(d['ms_per_step'], d['roofline']['frac'], d['roofline']['traffic'], d['stages_ms'])"; }
$B --config 4 > gpurun_out/c8_config4.log 2>&1 && line gpurun_out/c8_config4.log &&
$B --config 3 --exchange > gpurun_out/c8_config3x.log 2>&1 && line gpurun_out/c8_config3x.log &&
$B --accept-frac 0.3 --unordered-frac 0.1 > gpurun_out/c10_mix.log 2>&1 && line gpurun_out/c10_mix.log &&
timeout -k 10 400 python -u bench.py > gpurun_out/c8_config2f.log 2>&1 && line gpurun_out/c8_config2f.log
