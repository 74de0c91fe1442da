#!/bin/bash
# PMC passes of the config-2 bench (one counter group per run), for the per-kernel tables in profiles/
# (scripts/pmc_table.py). Usage: scripts/pmc_r2.sh TAG [bench args]
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmc_${1:-r2}
shift
mkdir -p $OUT
i=0
for P in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" \
         "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" \
         "SQ_WAIT_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_BUSY_CYCLES" \
         "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $P -f csv -d $OUT/p$i -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline "$@" > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo pmc-done
