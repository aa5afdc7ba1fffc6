# Pair-pipeline sweep (tools/dbg/stream_trace.py, pinned pairs of a pan) over
# ME_STREAM_BATCH (pairs per search launch) through the tuning build, at 1080p
# and CIF; the stream tests on the default build first.
mkdir -p gpurun_out
OUT=gpurun_out/${TAG:-r03bn}_stream_batch.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_ssim.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG:-r03bn}_stream_tests.log 2>&1 || exit $?
for SIZE in "1920 1080" "352 288"; do
  for G in 1 2 4 8; do
    echo "G=$G" >> $OUT
    ME_HIP_LIB=libme_hip_tune.so ME_STREAM_BATCH=$G timeout -k 10 120 python tools/dbg/stream_trace.py 64 $SIZE >> $OUT 2>&1 || exit $?
  done
done
