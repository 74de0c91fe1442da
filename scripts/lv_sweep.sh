#!/bin/bash
# levels: frontier loop vs dataflow with several step budgets (config 5 bench timings)
timeout -k 10 300 python -u -m pytest tests/test_gpu_levels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/lvsweep_tests.log 2>&1 || exit 1
for d in none 4 16 64; do
  if [ $d = none ]; then unset AD_LEVELS_DATAFLOW; else export AD_LEVELS_DATAFLOW=$d; fi
  timeout -k 10 300 python -u bench.py --config 5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/lvsweep_$d.log 2>&1 || exit 2
done
echo sweep-done
