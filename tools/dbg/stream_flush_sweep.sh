#!/bin/bash
# Pair pipeline: how the copy stream's ready markers get pushed (ME_STREAM_FLUSH,
# tuning build), 1080p pan of 64 pairs, pinned frames; then a trace of the best.
set -e
export ME_HIP_LIB=libme_hip_tune.so TMPDIR=/tmp
for f in ${FLUSH_SET:-0 3 4 0 3 4}; do
  echo "ME_STREAM_FLUSH=$f"
  ME_STREAM_FLUSH=$f timeout -k 10 120 python3 tools/dbg/stream_trace.py 64
done
ME_STREAM_FLUSH=${TRACE_FLUSH:-2} timeout -k 10 240 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace \
  --output-format csv -d gpurun_out/${TRACE_TAG:-r04c}_stream -o run -- python3 tools/dbg/stream_trace.py 16
