#!/bin/bash
# Pair-pipeline sweep (tools/dbg/stream_trace.py, pinned pairs of a pan) over
# ME_STREAM_BATCH (pairs per search launch) through the tuning build, 1080p
# (96 pairs) and CIF (64 pairs).
mkdir -p gpurun_out
OUT=gpurun_out/${TAG:-r04h}_stream_batch.txt
: > $OUT
for SIZE in "1920 1080" "352 288"; do
  NP=64; [ "$SIZE" = "1920 1080" ] && NP=96
  for G in ${GSET:-4 6 8 12 16}; do
    echo "G=$G" >> $OUT
    ME_HIP_LIB=libme_hip_tune.so ME_STREAM_BATCH=$G timeout -k 10 120 python tools/dbg/stream_trace.py $NP $SIZE >> $OUT 2>&1 || exit $?
  done
done
