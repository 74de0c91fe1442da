#!/bin/bash
# full GPU suite (one process), then the config-2 bench line (host_api included)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/full_gpu.log 2>&1 || { tail -40 gpurun_out/full_gpu.log; exit 1; }
tail -2 gpurun_out/full_gpu.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 > gpurun_out/bench_c2.log 2>&1 || { tail -20 gpurun_out/bench_c2.log; exit 2; }
tail -1 gpurun_out/bench_c2.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['ms_per_step'], r['roofline']['frac'], r.get('host_api'))"
