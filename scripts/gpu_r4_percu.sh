#!/bin/bash
# lean pass 1 residency: blocks per CU 4 (default for the wide kernel) vs 3 vs 2 on config 2
set -o pipefail
mkdir -p gpurun_out
B="timeout -k 10 300 python -u bench.py --no-cpu-baseline"
line() { grep '^{' "$1" | tail -1 > "${1%.log}.json"; python3 -c "import json; d=json.load(open('${1%.log}.json')); print('$2', d['ms_per_step'], d['stages_ms']['lean resolve pass 1'])"; }
$B > gpurun_out/pc4.log 2>&1 && line gpurun_out/pc4.log 4 &&
AD_LEAN_PER_CU=3 $B > gpurun_out/pc3.log 2>&1 && line gpurun_out/pc3.log 3 &&
AD_LEAN_PER_CU=2 $B > gpurun_out/pc2.log 2>&1 && line gpurun_out/pc2.log 2 &&
$B > gpurun_out/pc4b.log 2>&1 && line gpurun_out/pc4b.log 4b
