#!/bin/bash
# A/B of library variants on one bench line: scripts/gpu_ab.sh TAG "bench args" lib1 lib2 ...
# (lib "-" = the in-tree library); prints ms_per_step and the stage split per library
set -o pipefail
mkdir -p gpurun_out
T=$1; ARGS=$2; shift 2
i=0
for L in "$@"; do
  i=$((i+1))
  if [ "$L" = "-" ]; then unset ACCORD_DEPS_LIB; else export ACCORD_DEPS_LIB=$PWD/$L; fi
  timeout -k 10 300 python -u bench.py --no-cpu-baseline $ARGS > gpurun_out/${T}_$i.log 2>&1 || { echo "FAIL $L"; tail -5 gpurun_out/${T}_$i.log; exit 1; }
  python3 -c "
import json
r=json.loads([l for l in open('gpurun_out/${T}_$i.log') if l.startswith('{')][-1])
print('$L', round(r['ms_per_step'],4), {k.split('(')[0].strip()[:24]:v for k,v in r.get('stages_ms',{}).items() if v})"
done
