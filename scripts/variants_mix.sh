#!/bin/bash
# bench the in-tree library and each variants/*.so on the config-2 request mix (ACCORD_DEPS_LIB override)
ARGS="--steps 5 --warmup 2 --no-cpu-baseline --config 2 --accept-frac 0.3 --unordered-frac 0.1"
timeout -k 10 300 python -u bench.py $ARGS > gpurun_out/varm_base.log 2>&1 || exit 1
for f in variants/*.so; do
  b=$(basename $f .so)
  ACCORD_DEPS_LIB=$PWD/$f timeout -k 10 300 python -u bench.py $ARGS > gpurun_out/varm_$b.log 2>&1 || exit 1
done
echo variants-done
