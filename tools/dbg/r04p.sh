#!/bin/bash
# Round 4: pair pipeline after a clock ramp -- launch size after the ramp
# (ME_STREAM_BATCH) with and without the ramp, 64 pinned 1080p pairs, and a
# trace of the default.
set -e
mkdir -p gpurun_out
OUT=gpurun_out/r04p_stream_sweep.txt
: > $OUT
for v in "ME_STREAM_BATCH=8" "ME_STREAM_BATCH=12" "ME_STREAM_BATCH=16" "ME_STREAM_BATCH=8 ME_STREAM_RAMP=0" "ME_STREAM_BATCH=16 ME_STREAM_RAMP=0"; do
  echo "$v" >> $OUT
  env ME_HIP_LIB=libme_hip_tune.so $v timeout -k 10 120 python3 tools/dbg/stream_trace.py 64 >> $OUT 2>&1
done
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace \
  --output-format csv -d gpurun_out/r04p_stream -o run -- python3 tools/dbg/stream_trace.py 64 > gpurun_out/r04p_trace.log 2>&1
