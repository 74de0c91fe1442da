#!/bin/bash
# round 5: hot lines in LDS for lean pass 1 -- parity on the lean tests + full-size config 2, then the
# config-2 lab (in-tree = hot lines, variants/nohot.so = before) and the request-mix / config-3 lines
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/rh_t.log 2>&1 || { tail -30 gpurun_out/rh_t.log; exit 1; }
tail -1 gpurun_out/rh_t.log
timeout -k 10 400 python -u scripts/lean_lab.py --steps 20 variants/nohot.so > gpurun_out/rh_lab.log 2>&1 || { tail -20 gpurun_out/rh_lab.log; exit 2; }
grep '^{' gpurun_out/rh_lab.log | cut -c1-300
bash scripts/gpu_ab.sh rh_mix "--accept-frac 0.3 --unordered-frac 0.1" - variants/nohot.so || exit 3
bash scripts/gpu_ab.sh rh_c2 "" - variants/nohot.so - variants/nohot.so || exit 4
