cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/gpu_all.log 2>&1
