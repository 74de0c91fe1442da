#!/bin/bash
# one box: smoke, every GPU test file, the headline bench + trace, recovery bench scan 3, node rehearsal
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-all}
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
rc=$?; echo smoke=$rc; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputests_$TAG.log 2>&1
rc=$?; echo gputests=$rc; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.log 2>&1
rc=$?; echo bench=$rc; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --recovery 65536 --recovery-scan 3 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/rbench_$TAG.log 2>&1
rc=$?; echo rbench=$rc; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_trace.sh $TAG
