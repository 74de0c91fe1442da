cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_cfk_update.py > gpurun_out/cfk1.log 2>&1
