#!/bin/bash
# K5 after the single-round-trip plan: levels tests on the packed, CSR and frontier paths, config-5 line
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_levels.py tests/test_golden.py"
$T > gpurun_out/k5b_1.log 2>&1 || { tail -30 gpurun_out/k5b_1.log; exit 1; }
AD_LEVELS_PACKED=0 $T > gpurun_out/k5b_2.log 2>&1 || { tail -30 gpurun_out/k5b_2.log; exit 2; }
AD_LEVELS_FRONTIER=1 $T > gpurun_out/k5b_3.log 2>&1 || { tail -30 gpurun_out/k5b_3.log; exit 3; }
tail -qn1 gpurun_out/k5b_1.log gpurun_out/k5b_2.log gpurun_out/k5b_3.log
timeout -k 10 200 python -u bench.py --config 5 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/k5b_bench.log 2>&1 || exit 4
python3 -c "import json; r=json.loads(open('gpurun_out/k5b_bench.log').read().strip().splitlines()[-1]); print(r['ms_per_step'], r['stages_ms'])"
