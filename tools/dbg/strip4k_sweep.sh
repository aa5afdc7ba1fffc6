#!/bin/bash
# 4K +-64 SAD (item kernel, 16 frames per launch): tile-strip walk widths
# (ME_STRIP, tuning build: 0 = row-major order, the automatic choice at 4K) --
# kernel time and PMC traffic per launch (tools/profile.sh, keys *_strip<W>).
set -e
export ME_HIP_LIB=libme_hip_tune.so
for w in ${STRIPS:-0 8 10 15}; do
  ME_STRIP=$w PMC_KEY_SUFFIX=_strip$w bash tools/profile.sh r04h_4k_sad_strip$w --config 4k --cost sad \
    --steps 6 --warmup 2 --no-cpu --no-stream --no-4k --no-single --no-ssd > gpurun_out/r04h_strip$w.log 2>&1
done
