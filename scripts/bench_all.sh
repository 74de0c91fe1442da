#!/bin/bash
# one bench line per BASELINE config that fits one GPU (config 2 is the headline, default line)
for c in 2 1 4 5; do
  timeout -k 10 400 python -u bench.py --config $c --steps 5 --warmup 2 > gpurun_out/benchall_c$c.log 2>&1 || { echo "config $c failed"; exit 1; }
done
echo bench-all-done
