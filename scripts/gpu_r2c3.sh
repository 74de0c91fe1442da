#!/bin/bash
# config 3 path on one GPU: multi-store parity (library exchange), the 1/8 config-3 bench line plain and
# through the RCCL node exchange (world 1), and a 2-rank gloo rehearsal of the N > 1 flow.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_multi.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/c3_multi.log 2>&1
rc=$?; echo multi=$rc; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --config 3 --cpu-budget 4 > gpurun_out/c3_bench.log 2>&1
rc=$?; echo bench_c3=$rc; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --config 3 --exchange --no-cpu-baseline > gpurun_out/c3_bench_x.log 2>&1
rc=$?; echo bench_c3_x=$rc; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29633 bench.py --gpus 2 --dist-backend gloo --scale 0.25 --steps 3 --warmup 1 > gpurun_out/c3_gloo2.log 2>&1
rc=$?; echo gloo2=$rc; exit $rc
