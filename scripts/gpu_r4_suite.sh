#!/bin/bash
# Round-4 GPU check: the new Range-domain request tests first (a plain failure does not stop the run;
# a crash, abort or time limit does), then the whole -m gpu suite with device guard bands (AD_GUARD=1:
# every allocation's tail band checked after each test and at every free), then the plain
# unserialized suite, then the default bench line.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-r4}
crashed() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_ranges.py tests/test_gpu_multi.py -k "range" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_${TAG}_ranges.log 2>&1
rc=$?; echo ranges=$rc; tail -3 gpurun_out/t_${TAG}_ranges.log; crashed $rc && exit 9
# kernel lab: the in-tree library against the variants named in LAB (built by scripts/build_variant.sh)
if [ -n "$LAB" ]; then
  timeout -k 10 300 python -u scripts/lean_lab.py --steps 20 $LAB > gpurun_out/lab_${TAG}.log 2>&1
  rc=$?; echo lab=$rc; cat gpurun_out/lab_${TAG}.log | grep "^{" ; crashed $rc && exit 8
fi
AD_GUARD=1 timeout -k 10 1000 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_${TAG}_guard.log 2>&1
rc=$?; echo guard=$rc; tail -3 gpurun_out/t_${TAG}_guard.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 1000 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_${TAG}_plain.log 2>&1
rc=$?; echo plain=$rc; tail -3 gpurun_out/t_${TAG}_plain.log; [ $rc -eq 0 ] || exit 2
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/b_${TAG}.log 2>&1 || exit 3
tail -c 1500 gpurun_out/b_${TAG}.log
timeout -k 10 300 python -u bench.py --config 5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/c5_${TAG}.log 2>&1 || exit 4
tail -c 1200 gpurun_out/c5_${TAG}.log
# optional counter passes (PMC=1): lean pass 1's read/write access split
if [ -n "$PMC" ]; then
  bash scripts/pmc_split.sh split_${TAG} && python3 scripts/pmc_table.py gpurun_out/pmc_split_${TAG} resolve_lean > gpurun_out/pmc_split_${TAG}.txt
fi
