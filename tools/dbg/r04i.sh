#!/bin/bash
# Round 4: the pair pipeline's ramped launches (1, 2, 4, 8 pairs) -- stream
# tests, pinned pan rates -- and request-size-calibrated read bytes of the
# 1080p and 4K SAD batches (tools/profile.sh SIZED=1).
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04i_stream_tests.log 2>&1
for n in 64 96; do timeout -k 10 120 python3 tools/dbg/stream_trace.py $n >> gpurun_out/r04i_stream_rates.txt 2>&1; done
timeout -k 10 120 python3 tools/dbg/stream_trace.py 64 352 288 >> gpurun_out/r04i_stream_rates.txt 2>&1
SIZED=1 bash tools/profile.sh r04i_4k_sad --config 4k --cost sad --steps 6 --warmup 2 --no-cpu --no-stream --no-4k --no-single --no-ssd > gpurun_out/r04i_prof4k.log 2>&1
SIZED=1 bash tools/profile.sh r04i_1080p_sad --steps 20 --warmup 3 --no-cpu --no-stream --no-4k --no-single --no-ssd > gpurun_out/r04i_prof1080.log 2>&1
