#!/bin/bash
# Parity files touched by the resolve / exchange, two default bench lines, the bench with the separate
# slot launch (AD_SLOTS_KERNEL), the config-3 share, and the config-2 profile under TAG.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-r3_final2}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_host_api.py tests/test_gpu_fullsize.py tests/test_gpu_multi.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_s.log 2>&1
rc=$?; tail -2 gpurun_out/t_s.log; [ $rc -eq 0 ] || exit 1
for i in 1 2; do timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/b_s$i.log 2>&1 || exit 2; done
AD_SLOTS_KERNEL=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/b_s0.log 2>&1 || exit 3
timeout -k 10 300 python -u bench.py --config 3 --exchange --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/c3_s.log 2>&1 || exit 4
bash scripts/profile.sh ${TAG}_config2 || exit 5
echo ok
