#!/bin/bash
# Pair pipeline: pinned 1080p pan timings (64 pairs, 3 reps, twice) and a
# kernel + copy + HIP API trace of a 16-pair run (tools/stream_timeline.py,
# /tmp-free analysis in tools/stream_gaps.py).  TAG names the output dir.
set -e
export TMPDIR=/tmp
for i in 1 2; do timeout -k 10 120 python3 tools/dbg/stream_trace.py 64; done
timeout -k 10 240 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace \
  --output-format csv -d gpurun_out/${TAG:-r04g}_stream -o run -- python3 tools/dbg/stream_trace.py 16
