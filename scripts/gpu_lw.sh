#!/bin/bash
# lane-width tests, the export's ids-per-request at W = 8 and N = 1, and the 2-lane export A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_multi.py -m gpu -x -q --timeout 300 --timeout-method thread -k "lane_widths or node_exchange or exchange_local" > gpurun_out/t_lw.log 2>&1
rc=$?; tail -2 gpurun_out/t_lw.log; [ $rc -eq 0 ] || exit 1
AD_EXPORT_TRACE=1 timeout -k 10 300 python -u scripts/emulate_config3.py --world 8 --scale 0.25 --steps 1 > gpurun_out/emu_tr.log 2>&1 || exit 2
grep -m 3 "^export:" gpurun_out/emu_tr.log
AD_EXPORT_TRACE=1 timeout -k 10 300 python -u bench.py --config 3 --exchange --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/c3_tr.log 2>&1 || exit 3
grep -m 2 "^export:" gpurun_out/c3_tr.log
bash scripts/export_ab.sh g2:AD_EXPORT_G=2 || exit 4
