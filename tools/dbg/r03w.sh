set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "item_kernel_jobs or batch_search or stripe_jobs" > gpurun_out/r03w_parity.log 2>&1
