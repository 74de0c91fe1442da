#!/bin/bash
# round 5: the merge split into a queued phase and its tail (owners on distinct GPUs merge at once) -- the
# multi-GPU and union tests, then the W = 8 emulation and the config-3 line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_multi.py tests/test_gpu_union.py -x -q --timeout 200 --timeout-method thread > gpurun_out/rw_t.log 2>&1 || { tail -30 gpurun_out/rw_t.log; exit 1; }
tail -1 gpurun_out/rw_t.log
timeout -k 10 400 python -u scripts/emulate_config3.py --world 8 --scale 0.25 --steps 5 > gpurun_out/rw_emulate_w8.log 2>&1 || { tail -20 gpurun_out/rw_emulate_w8.log; exit 2; }
tail -1 gpurun_out/rw_emulate_w8.log | cut -c1-400
timeout -k 10 400 python -u bench.py --config 3 --exchange --no-cpu-baseline > gpurun_out/rw_c3x.log 2>&1 || { tail -20 gpurun_out/rw_c3x.log; exit 3; }
grep '^{' gpurun_out/rw_c3x.log | tail -1 | cut -c1-300
