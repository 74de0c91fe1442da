#!/bin/bash
# lean deferrals to the split kernels (AD_DEFER_SPLIT) against the general fused kernel: parity + mix
set -o pipefail
mkdir -p gpurun_out
AD_DEFER_SPLIT=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fullsize.py > gpurun_out/ds_tests.log 2>&1 || { tail -30 gpurun_out/ds_tests.log; exit 1; }
tail -1 gpurun_out/ds_tests.log
line() { python3 -c "import json,sys; r=json.loads(open('$1').read().strip().splitlines()[-1]); print(r['ms_per_step'], r['stages_ms'], r.get('deferred'))"; }
AD_DEFER_SPLIT=1 timeout -k 10 300 python -u bench.py --accept-frac 0.3 --unordered-frac 0.1 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ds_mix.log 2>&1 && line gpurun_out/ds_mix.log || exit 2
