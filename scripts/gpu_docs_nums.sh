cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/nums && \
timeout -k 10 300 python -u bench.py > gpurun_out/nums/c2.json 2> gpurun_out/nums/c2.err && \
timeout -k 10 300 python -u bench.py --config 2 --accept-frac 0.3 --unordered-frac 0.2 --no-cpu-baseline > gpurun_out/nums/mix.json 2> gpurun_out/nums/mix.err && \
timeout -k 10 300 python -u bench.py --config 3 --exchange --no-cpu-baseline > gpurun_out/nums/c3x.json 2> gpurun_out/nums/c3x.err && \
timeout -k 10 300 python -u bench.py --recovery 65536 --recovery-scan 3 --no-cpu-baseline > gpurun_out/nums/rec3.json 2> gpurun_out/nums/rec3.err && \
timeout -k 10 300 python -u bench.py --config 5 --no-cpu-baseline > gpurun_out/nums/c5.json 2> gpurun_out/nums/c5.err && \
timeout -k 10 300 python -u bench.py --config 4 --no-cpu-baseline > gpurun_out/nums/c4.json 2> gpurun_out/nums/c4.err
