#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmc_sq
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES -f csv -d $OUT/p1 -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $OUT/p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SMEM SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY -f csv -d $OUT/p2 -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $OUT/p2.log 2>&1 || exit 2
echo pmc-done
