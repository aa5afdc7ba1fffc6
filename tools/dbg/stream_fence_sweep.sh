#!/bin/bash
# Pair pipeline: release scope of the ordering events (ME_STREAM_FENCE, tuning
# build: 0 system scope, 1 no system fence, 2 device-scope release), 1080p pan
# of 64 pairs, pinned frames; then a trace with the chosen setting.
set -e
export ME_HIP_LIB=libme_hip_tune.so TMPDIR=/tmp
for f in ${FENCE_SET:-0 1 2 0 1 2}; do
  echo "ME_STREAM_FENCE=$f"
  ME_STREAM_FENCE=$f timeout -k 10 120 python3 tools/dbg/stream_trace.py 64
done
ME_STREAM_FENCE=${TRACE_FENCE:-2} timeout -k 10 240 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace \
  --output-format csv -d gpurun_out/${TRACE_TAG:-r04e}_stream -o run -- python3 tools/dbg/stream_trace.py 16
