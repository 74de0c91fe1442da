#!/bin/bash
# Rehearsal of the N>1 bench path on a 1-GPU box: N ranks share the GPU, the exchange runs over gloo
# staged through host memory (RCCL itself is not exercised). Usage: scripts/rehearse_multi.sh N [bench args]
set -o pipefail
N=${1:-2}; shift
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus $N --dist-backend gloo --no-cpu-baseline "$@" > gpurun_out/rehearse_$N.log 2>&1
rc=$?
echo rehearse=$rc
exit $rc
