timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5s3_full.log 2>&1; tail -3 gpurun_out/r5s3_full.log
bash scripts/gpu_ab.sh ab4 "--range-frac 0.01" variants/prerange.so - 
timeout -k 10 400 python -u scripts/lean_lab.py --config 2 --steps 10 --regions variants/exp16.so variants/exp4.so variants/exp1.so variants/exp21.so > gpurun_out/lab_exp.log 2>&1; grep "regions\": true" gpurun_out/lab_exp.log | cut -c1-200
