#!/bin/bash
# the round's last checks on the final tree: smoke, the full suite, the bench lines, the config-2 profile
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/last_smoke.log 2>&1 && tail -1 gpurun_out/last_smoke.log || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_last.log 2>&1; rc=$?; echo suite=$rc; tail -2 gpurun_out/t_last.log
case $rc in 0) ;; *) exit $rc;; esac
B="timeout -k 10 300 python -u bench.py --no-cpu-baseline"
line() { grep '^{' "$1" | tail -1 > "${1%.log}.json"; python3 -c "import json; d=json.load(open('${1%.log}.json')); print(d['ms_per_step'], d['roofline']['frac'], d['roofline']['traffic'], d['stages_ms'])"; }
timeout -k 10 400 python -u bench.py > gpurun_out/last_config2.log 2>&1 && line gpurun_out/last_config2.log &&
$B --accept-frac 0.3 --unordered-frac 0.1 > gpurun_out/last_mix.log 2>&1 && line gpurun_out/last_mix.log &&
$B --config 3 --exchange > gpurun_out/last_config3x.log 2>&1 && line gpurun_out/last_config3x.log &&
$B --config 4 > gpurun_out/last_config4.log 2>&1 && line gpurun_out/last_config4.log &&
bash scripts/profile.sh r4g_config2
