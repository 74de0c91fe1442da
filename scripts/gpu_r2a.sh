#!/bin/bash
# Round 2, first GPU pass: full-size parity tests, the default bench (multi-store CPU baseline with
# its parity sample), the request-mix bench and its kernel trace.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/full_r2a.log 2>&1
rc=$?; echo fullsize=$rc; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/bench_r2a.log 2>&1
rc=$?; echo bench=$rc; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --accept-frac 0.3 --unordered-frac 0.1 --cpu-budget 6 > gpurun_out/bench_mix_r2a.log 2>&1
rc=$?; echo bench_mix=$rc; [ $rc -eq 0 ] || exit $rc
bash scripts/profile.sh r2a_mix --accept-frac 0.3 --unordered-frac 0.1
