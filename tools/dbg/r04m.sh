#!/bin/bash
# Round 4: 8K 8x8 +-128 SAD -- 16 frames in one item-kernel launch
# (ME_ITEM_BATCH=1: every XCD band holds whole frames, no band halos) against
# one launch per frame, with strip widths.
set -e
mkdir -p gpurun_out
VARIANTS="none;ME_ITEM_BATCH=1;ME_ITEM_BATCH=1 ME_STRIP=0;ME_ITEM_BATCH=1 ME_STRIP=8;ME_ITEM_BATCH=1 ME_STRIP=32" \
  bash tools/dbg/pmc_variants.sh r04m_8k --config 8k --cost sad --steps 2 --warmup 0 --no-cpu --no-stream --no-4k --no-single --no-ssd > gpurun_out/r04m_variants_8k.txt 2>&1
TAG=r04m bash tools/dbg/stream_trace.sh > gpurun_out/r04m_stream_trace.log 2>&1
