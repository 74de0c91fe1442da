#!/bin/bash
# export / K3-copy kernel A/B: kernel traces of the W=8 emulation and of the config-3 N=1 share per
# variant. A variant is NAME or NAME:VAR=val,VAR=val (e.g. tiles:AD_EXPORT_TILES=1,AD_RMERGE_TILES=1).
set -o pipefail
export TMPDIR=/tmp
for spec in "$@"; do
  v=${spec%%:*}
  envs=""
  [ "$spec" != "$v" ] && envs=${spec#*:}
  mkdir -p gpurun_out/xab_$v gpurun_out/xab1_$v
  ( IFS=,; for e in $envs; do export "$e"; done
    timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d gpurun_out/xab_$v -o run -- python3 scripts/emulate_config3.py --world 8 --scale 0.25 --steps 3 > gpurun_out/xab_$v/log 2>&1 || exit 1
    timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d gpurun_out/xab1_$v -o run -- python3 bench.py --config 3 --exchange --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/xab1_$v/log 2>&1 || exit 2 ) || exit 1
done
echo done
