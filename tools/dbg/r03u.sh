set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03u_pytest_gpu.log 2>&1
for c in 4k 8k 1080p; do
  timeout -k 10 300 python -u tools/stripe_sweep.py --config $c --frames 8 --ranks 1,2,4,8 --iters 10 >> gpurun_out/r03u_stripe_sweep.jsonl
done
