#!/bin/bash
# PMC passes of the request-mix bench line (the general kernel over the late PreAccepts): issue and wait
# counters, one counter group per run. Table: scripts/pmc_table.py gpurun_out/pmc_<tag>
set -o pipefail
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/pmc_${1:-mix}
mkdir -p $OUT
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC" \
         "SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM" \
         "GRBM_GUI_ACTIVE TA_TA_BUSY_sum TD_TD_BUSY_sum" \
         "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $P -f csv -d $OUT/p$i -o run -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline --accept-frac 0.3 --unordered-frac 0.1 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo pmc-done
