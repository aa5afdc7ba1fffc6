#!/bin/bash
# Round 4: pair records on the copy stream vs a stream of their own, after
# searches on a torch stream (tools/dbg/hs_probe.py), and the stream tests.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04s_stream_tests.log 2>&1
OUT=gpurun_out/r04s_hs_probe.txt
for m in batch_stream none; do
  echo "copy-stream records, $m" >> $OUT
  timeout -k 10 200 python3 tools/dbg/hs_probe.py $m >> $OUT 2>&1
  echo "own-stream records (ME_STREAM_D2H=1), $m" >> $OUT
  ME_HIP_LIB=libme_hip_tune.so ME_STREAM_D2H=1 timeout -k 10 200 python3 tools/dbg/hs_probe.py $m >> $OUT 2>&1
done
