#!/bin/bash
# host API: into-path tests, then the timeline lab over slicings and copy-kernel grids
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_host_api.py > gpurun_out/h_tests.log 2>&1 || { tail -40 gpurun_out/h_tests.log; exit 1; }
tail -1 gpurun_out/h_tests.log
timeout -k 10 300 python -u scripts/host_api_lab.py --slices 0 4 8 12 > gpurun_out/h_lab.log 2>&1 || { tail -30 gpurun_out/h_lab.log; exit 2; }
grep -E "^slices" gpurun_out/h_lab.log
for b in 64 256; do
AD_COPY_BLOCKS=$b timeout -k 10 300 python -u scripts/host_api_lab.py --slices 0 8 > gpurun_out/h_lab_b$b.log 2>&1 || exit 3
echo "blocks $b: $(grep -E '^slices' gpurun_out/h_lab_b$b.log | tr '\n' ' ')"
done
AD_INTO_WIRE=0 timeout -k 10 300 python -u scripts/host_api_lab.py --slices 0 > gpurun_out/h_lab_nowire.log 2>&1 || exit 4
echo "no wire: $(grep -E '^slices' gpurun_out/h_lab_nowire.log | tr '\n' ' ')"
grep -B9 "slices=0 rep 2" gpurun_out/h_lab.log
