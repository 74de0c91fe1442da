#!/bin/bash
# Read/write split of lean pass 1's vector-memory accesses (config-2 batch of scripts/lean_lab.py, the
# in-tree library or the one given as $2): one counter group per run. Table: scripts/pmc_table.py gpurun_out/pmc_<tag>
set -o pipefail
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/pmc_${1:-split}
mkdir -p $OUT
i=0
for P in "TCP_TOTAL_READ_sum TCP_TOTAL_WRITE_sum TCP_TCC_WRITE_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" \
         "TCP_TCC_READ_REQ_sum TCP_UTCL1_REQUEST_sum" \
         "SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VMEM SQ_INSTS_VALU SQ_INSTS_LDS" \
         "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum" \
         "TD_TD_BUSY_sum TD_TC_STALL_sum" \
         "GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -f csv -d $OUT/p$i -o run -- python3 scripts/lean_lab.py --steps 2 --warmup 1 ${2:+--only $2} > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo pmc-done
