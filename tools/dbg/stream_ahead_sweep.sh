# Pair pipeline at 4 pairs per launch: host run-ahead (ME_STREAM_AHEAD, batches)
# and cooling slots (ME_STREAM_COOL) through the tuning build, 64 pinned 1080p pairs.
mkdir -p gpurun_out
OUT=gpurun_out/${TAG:-r03br}_stream_ahead.txt
for AC in "0 0" "3 0" "4 0" "2 12" "3 12" "4 16"; do
  set -- $AC
  echo "AHEAD=$1 COOL=$2" >> $OUT
  ME_HIP_LIB=libme_hip_tune.so ME_STREAM_AHEAD=$1 ME_STREAM_COOL=$2 timeout -k 10 120 python tools/dbg/stream_trace.py 64 >> $OUT 2>&1 || exit $?
done
