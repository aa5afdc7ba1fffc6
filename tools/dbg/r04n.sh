#!/bin/bash
# Round 4: pair pipeline with per-batch record downloads and a 1.5x ramp;
# batched 8K SAD launches (whole frames per XCD band, row-major) -- GPU suite,
# pair rates and trace, 8K traffic; single-frame 8K strip widths.
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04n_pytest_gpu.log 2>&1
for n in 64 96; do timeout -k 10 120 python3 tools/dbg/stream_trace.py $n >> gpurun_out/r04n_stream_rates.txt 2>&1; done
timeout -k 10 120 python3 tools/dbg/stream_trace.py 64 352 288 >> gpurun_out/r04n_stream_rates.txt 2>&1
TAG=r04n bash tools/dbg/stream_trace.sh > gpurun_out/r04n_stream_trace.log 2>&1
VARIANTS="none" bash tools/dbg/pmc_variants.sh r04n_8k --config 8k --cost sad --steps 2 --warmup 0 --no-cpu --no-stream --no-4k --no-single --no-ssd > gpurun_out/r04n_variants_8k.txt 2>&1
VARIANTS="none;ME_STRIP=0;ME_STRIP=8" bash tools/dbg/pmc_variants.sh r04n_8k1 --config 8k --cost sad --frames-per-step 1 --steps 4 --warmup 1 --no-cpu --no-stream --no-4k --no-single --no-ssd > gpurun_out/r04n_variants_8k_f1.txt 2>&1
