#!/bin/bash
# the N = 8 emulation with lean pass 1 at 4 (default) / 8 requests per wave (AD_LEAN_RPW=8), and 8 per wave at 4
# waves per SIMD (variants/occ4n.so)
set -o pipefail
mkdir -p gpurun_out
E="timeout -k 10 300 python -u scripts/emulate_config3.py --world 8 --scale 0.25 --steps 5"
$E > gpurun_out/rpw_def.log 2>&1 && tail -1 gpurun_out/rpw_def.log | cut -c1-200 &&
AD_LEAN_RPW=8 $E > gpurun_out/rpw_8.log 2>&1 && tail -1 gpurun_out/rpw_8.log | cut -c1-200 &&
AD_LEAN_RPW=8 ACCORD_DEPS_LIB=$PWD/variants/occ4n.so $E > gpurun_out/rpw_8o4.log 2>&1 && tail -1 gpurun_out/rpw_8o4.log | cut -c1-200
