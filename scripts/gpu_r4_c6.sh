#!/bin/bash
# host paths after the huge-page result arrays / threaded staging (default bench: host_api + cpu_baseline),
# smoke, then the full suite
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/c6_config2.log 2>&1 && grep '^{' gpurun_out/c6_config2.log | tail -1 > gpurun_out/c6_config2.json &&
python3 -c "import json; d=json.load(open('gpurun_out/c6_config2.json')); print(d['ms_per_step'], d['host_api'])" &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/c6_smoke.log 2>&1 && tail -1 gpurun_out/c6_smoke.log &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_c6.log 2>&1; rc=$?; echo suite=$rc; tail -2 gpurun_out/t_c6.log
