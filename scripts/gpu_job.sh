# one GPU call of round-3 work: new tests, the lab A/B of the lean passes, the bench, counters, N=8 emulation
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/lean_lab.py --steps 20 variants/noslots.so > gpurun_out/lab3.log 2>&1; rc=$?; grep ms_per gpurun_out/lab3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_host_api.py tests/test_gpu_recovery_live.py tests/test_gpu_recovery.py tests/test_gpu_cfk_missing.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3_host.log 2>&1; rc=$?; tail -25 gpurun_out/r3_host.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-budget 2 > gpurun_out/r3_bench_host.log 2>&1; rc=$?; tail -c 1500 gpurun_out/r3_bench_host.log; [ $rc -eq 0 ] || exit $rc
scripts/pmc_lab.sh lab1 && python3 scripts/pmc_table.py gpurun_out/pmc_lab1 k_resolve_lean k_pack_tiles k_lean_slots > gpurun_out/pmc_lab1.txt || exit 1
timeout -k 10 300 python -u scripts/emulate_config3.py --world 8 --scale 0.25 > gpurun_out/emu_c3.log 2>&1; tail -3 gpurun_out/emu_c3.log
