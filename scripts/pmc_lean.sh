#!/bin/bash
# PMC passes of a bench configuration, one counter group per run. Usage: scripts/pmc_lean.sh [TAG [bench args]]
# (no bench args: the config-2 headline)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmc_lean${1:+_$1}
[ $# -gt 0 ] && shift
mkdir -p $OUT
i=0
for P in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES" "SQ_INSTS_SMEM SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_INSTS_VMEM_WR" "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" "GRBM_GUI_ACTIVE SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -f csv -d $OUT/p$i -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline "$@" > $OUT/p$i.log 2>&1 || echo "pass $i failed"
done
echo pmc-done
