cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/steady && \
timeout -k 10 400 python -u bench.py --steady 16384 --steps 8 --warmup 2 > gpurun_out/steady/steady_16k.json 2> gpurun_out/steady/steady_16k.err && \
bash scripts/profile.sh r2upd --config 2 --cfk-update 1000000 && \
bash scripts/profile.sh r2steady --steady 16384
