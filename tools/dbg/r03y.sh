set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 240 --timeout-method thread -k "random_job_tables" > gpurun_out/r03y_parity.log 2>&1
