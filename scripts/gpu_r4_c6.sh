#!/bin/bash
# smoke, the full suite, the default bench (host_api + cpu_baseline), then the K5 lane-refill and the
# packed key-start experiments
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/c6_smoke.log 2>&1 && tail -1 gpurun_out/c6_smoke.log || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_c6.log 2>&1; rc=$?; echo suite=$rc; tail -2 gpurun_out/t_c6.log
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 400 python -u bench.py > gpurun_out/c6_config2.log 2>&1 && grep '^{' gpurun_out/c6_config2.log | tail -1 > gpurun_out/c6_config2.json &&
python3 -c "import json; d=json.load(open('gpurun_out/c6_config2.json')); print(d['ms_per_step'], d['host_api'])" || exit 2
B="timeout -k 10 300 python -u bench.py --no-cpu-baseline --config 5 --steps 10 --warmup 2"
$B > gpurun_out/c7_c5.log 2>&1 && grep '^{' gpurun_out/c7_c5.log | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); print('wave', d['ms_per_step'], d['stages_ms'])" &&
AD_LEVELS_PULL_LANE=1 $B > gpurun_out/c7_c5l.log 2>&1 && grep '^{' gpurun_out/c7_c5l.log | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); print('lane', d['ms_per_step'], d['stages_ms'])" &&
AD_LEVELS_PULL_LANE=1 AD_LEVELS_PULL_PER_CU=2 $B > gpurun_out/c7_c5l2.log 2>&1 && grep '^{' gpurun_out/c7_c5l2.log | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); print('lane2', d['ms_per_step'], d['stages_ms'])" &&
timeout -k 10 300 python -u scripts/lean_lab.py --steps 20 --regions variants/packa.so > gpurun_out/lab_packa.log 2>&1 && grep '^{' gpurun_out/lab_packa.log &&
timeout -k 10 300 python -u scripts/lean_lab.py --steps 20 --config 3 variants/packa.so > gpurun_out/lab_packa3.log 2>&1 && grep '^{' gpurun_out/lab_packa3.log
