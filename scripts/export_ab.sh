#!/bin/bash
# export kernel A/B: per-step window of the 8 stores' exports in the W=8 emulation (kernel trace) and
# the config-3 N=1 share, for AD_EXPORT_TILES / AD_EXPORT_G variants given as arguments (e.g. t 4 8)
set -o pipefail
export TMPDIR=/tmp
for v in "$@"; do
  unset AD_EXPORT_TILES AD_EXPORT_G
  if [ "$v" = t ]; then export AD_EXPORT_TILES=1; else export AD_EXPORT_G=$v; fi
  mkdir -p gpurun_out/xab_$v gpurun_out/xab1_$v
  timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d gpurun_out/xab_$v -o run -- python3 scripts/emulate_config3.py --world 8 --scale 0.25 --steps 3 > gpurun_out/xab_$v/log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d gpurun_out/xab1_$v -o run -- python3 bench.py --config 3 --exchange --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/xab1_$v/log 2>&1 || exit 2
done
echo done
