#!/bin/bash
# Round-3 refresh of the side profiles: request mix, steady state, config 3 (N=1 share + library
# exchange), and the N=8 node emulation on one GPU. Stops at the first failing step.
set -o pipefail
mkdir -p gpurun_out
bash scripts/profile.sh r3_mix --accept-frac 0.3 --unordered-frac 0.1 || exit 1
bash scripts/profile.sh r3_steady --steady 16384 || exit 2
timeout -k 10 300 python -u bench.py --config 3 --exchange --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/c3x.log 2>&1 || exit 3
tail -c 2500 gpurun_out/c3x.log
bash scripts/profile.sh r3_config3x --config 3 --exchange || exit 4
timeout -k 10 300 python -u scripts/emulate_config3.py --world 8 --scale 0.25 > gpurun_out/emu_c3.log 2>&1 || exit 5
tail -2 gpurun_out/emu_c3.log
