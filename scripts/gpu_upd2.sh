cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/steady && timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_cfk_update.py > gpurun_out/upd2.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steady 16384 --steps 8 --warmup 2 > gpurun_out/steady/steady_16k_c.json 2> gpurun_out/steady/steady_16k_c.err && \
timeout -k 10 300 python -u bench.py --config 2 --cfk-update 1000000 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/steady/upd_1m_c.json 2> gpurun_out/steady/upd_1m_c.err
