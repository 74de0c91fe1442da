#!/bin/bash
# bench the in-tree library and each variants/*.so (same tree, ACCORD_DEPS_LIB override)
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/var_base.log 2>&1 || exit 1
for f in variants/*.so; do
  b=$(basename $f .so)
  ACCORD_DEPS_LIB=$PWD/$f timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/var_$b.log 2>&1 || exit 1
done
echo variants-done
