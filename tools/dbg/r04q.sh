#!/bin/bash
# Round 4: packed MV stores -- GPU suite; bench.py's host_stream leg alone and
# inside the default line; 8K SAD write bytes.
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04q_pytest_gpu.log 2>&1
timeout -k 10 200 python3 bench.py --no-cpu --no-ssd --no-4k --no-single --steps 10 > gpurun_out/r04q_bench_stream_only.json 2> gpurun_out/r04q_a.err
timeout -k 10 400 python3 bench.py > gpurun_out/r04q_bench.json 2> gpurun_out/r04q_b.err
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T -d gpurun_out/r04q_w8k -o run --output-format csv -- python3 bench.py --config 8k --steps 2 --warmup 0 --no-cpu --no-stream --no-4k --no-single --no-ssd > gpurun_out/r04q_w8k.log 2>&1
