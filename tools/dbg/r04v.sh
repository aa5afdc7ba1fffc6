set -e
mkdir -p gpurun_out
OUT=gpurun_out/r04v_hs_batch.txt
for g in 8 12 16; do
  echo "ME_STREAM_BATCH=$g" >> $OUT
  ME_HIP_LIB=libme_hip_tune.so ME_STREAM_BATCH=$g timeout -k 10 200 python3 tools/dbg/hs_probe.py batch_stream >> $OUT 2>&1
done
