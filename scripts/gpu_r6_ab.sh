#!/bin/bash
# A/B of library variants on the config-2 bench (and optional extra bench args): each variant's bench line.
#   bash scripts/gpu_r6_ab.sh TAG "lib_a.so lib_b.so ..." [bench args]
set -o pipefail
T=$1; LIBS=$2; shift 2
mkdir -p gpurun_out
for L in $LIBS; do
  n=$(basename $L .so)
  ACCORD_DEPS_LIB=$PWD/$L timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 30 --warmup 3 "$@" > gpurun_out/${T}_${n}.log 2>&1 || { tail -20 gpurun_out/${T}_${n}.log; exit 1; }
  grep '^{' gpurun_out/${T}_${n}.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); s=d.get("stages_ms",{}); print(sys.argv[1], d["ms_per_step"], "resolve", d["roofline"]["launch_ms"], "frac", round(d["roofline"]["frac"],4), "pass1", s.get("lean resolve pass 1"), "pass2", s.get("lean resolve pass 2 (2 requests/wave, 2 emissions/lane)"), "prep", s.get("prepare (request records: S / self ranks; probe KeyLines for the lean passes)"))' $n
done
