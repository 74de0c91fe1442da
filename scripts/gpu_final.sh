#!/bin/bash
# Round-end evidence on one GPU: the whole -m gpu suite, smoke, the default bench line (with its
# cpu_baseline), rocprofv3 trace + FETCH/WRITE passes of the headline and of the config-3 share, and
# the W=8 node emulation. Stops at the first step that does not end normally.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-r3_final}
# TEST_ENV: extra environment for the test step only (e.g. AMD_SERIALIZE_KERNEL=3 to pin a device fault
# on the call that caused it)
env $TEST_ENV timeout -k 10 1000 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1
rc=$?; echo tests=$rc; tail -2 gpurun_out/t_$TAG.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit 2
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$TAG.log 2>&1 || exit 3
tail -c 600 gpurun_out/bench_$TAG.log
bash scripts/profile.sh ${TAG}_config2 || exit 4
bash scripts/profile.sh ${TAG}_config3x --config 3 --exchange || exit 5
timeout -k 10 300 python -u scripts/emulate_config3.py --world 8 --scale 0.25 > gpurun_out/emu_$TAG.log 2>&1 || exit 6
tail -1 gpurun_out/emu_$TAG.log
echo final-done
