#!/bin/bash
# PMC passes of scripts/lean_lab.py (config-2 batch, the in-tree library; one counter group per run):
# stall / latency / TLB / issue counters for the resolve kernels. Table: scripts/pmc_table.py gpurun_out/pmc_<tag>
set -o pipefail
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/pmc_${1:-lab}
mkdir -p $OUT
i=0
for P in "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum" \
         "TD_TD_BUSY_sum TD_TC_STALL_sum" \
         "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum" \
         "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCP_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" \
         "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC" \
         "SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_LEVEL_WAVES SQ_INSTS_VMEM SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
         "GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -f csv -d $OUT/p$i -o run -- python3 scripts/lean_lab.py --steps 2 --warmup 1 "${@:2}" > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo pmc-done
