#!/bin/bash
# exchange path: multi-store + union parity, the config-3 bench through the node exchange, and the
# N-store node rehearsal on one GPU (ad_exchange_local)
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-x}
timeout -k 10 500 python -u -m pytest tests/test_gpu_multi.py tests/test_gpu_union.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/multi_$TAG.log 2>&1
rc=$?; echo multi=$rc; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --config 3 --exchange --no-cpu-baseline > gpurun_out/c3x_$TAG.log 2>&1
rc=$?; echo bench_c3_x=$rc; [ $rc -eq 0 ] || exit $rc
for N in 2 8; do
  timeout -k 10 300 python -u scripts/node_local_bench.py --stores $N --scale 0.5 > gpurun_out/node${N}_$TAG.log 2>&1
  rc=$?; echo node$N=$rc; [ $rc -eq 0 ] || exit $rc
done
