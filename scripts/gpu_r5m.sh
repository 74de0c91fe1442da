#!/bin/bash
# current config-4 and request-mix bench lines (stage splits)
set -o pipefail
mkdir -p gpurun_out
line() { python3 -c "import json,sys; r=json.loads(open('$1').read().strip().splitlines()[-1]); print(r['ms_per_step'], r['roofline']['frac'], r['stages_ms'], r.get('deferred'))"; }
timeout -k 10 300 python -u bench.py --config 4 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/m_c4.log 2>&1 && line gpurun_out/m_c4.log || exit 1
timeout -k 10 300 python -u bench.py --accept-frac 0.3 --unordered-frac 0.1 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/m_mix.log 2>&1 && line gpurun_out/m_mix.log || exit 2
