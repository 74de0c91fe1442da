#!/bin/bash
# config 5 with the in-tree library and variants/<name>.so (ACCORD_DEPS_LIB)
set -o pipefail
mkdir -p gpurun_out
run() {
  timeout -k 10 120 python -u bench.py --config 5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/c5v.log 2>&1 || { tail -20 gpurun_out/c5v.log; exit 1; }
  echo "$1 $(python3 -c "import json,sys; r=json.loads(open('gpurun_out/c5v.log').read().strip().splitlines()[-1]); print(round(r['ms_per_step'],4), r['stages_ms'])")"
}
run base
for v in "$@"; do ACCORD_DEPS_LIB=$PWD/variants/$v.so run $v; done
