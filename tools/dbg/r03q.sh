set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 150 --timeout-method thread -k "batch or stripes or flow or jobs" > gpurun_out/r03q_parity.log 2>&1
timeout -k 10 150 python -u tools/stripe_sweep.py --config 1080p --ranks 1,2,4,8 --frames 8 > gpurun_out/r03q_sweep.jsonl
timeout -k 10 200 python -u tools/stripe_sweep.py --config 4k --ranks 1,2,4,8 --frames 8 >> gpurun_out/r03q_sweep.jsonl
timeout -k 10 300 python -u bench.py > gpurun_out/r03q_bench.json 2> gpurun_out/r03q_bench.err
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r03q_gpu.log 2>&1
