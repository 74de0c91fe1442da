cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/k5 && timeout -k 10 200 python -u bench.py --config 5 --no-cpu-baseline > gpurun_out/k5/frontier.json 2> gpurun_out/k5/frontier.err && \
for st in 4 8 32; do AD_LEVELS_DATAFLOW=$st timeout -k 10 200 python -u bench.py --config 5 --no-cpu-baseline > gpurun_out/k5/df$st.json 2> gpurun_out/k5/df$st.err || exit 1; done
