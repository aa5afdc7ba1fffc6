#!/bin/bash
# Round 4: item kernel with two-ended band counters (thieves take a band's last
# tiles) -- GPU suite, then request-size-calibrated traffic and time of the 4K
# +-64 and 8K 8x8 +-128 SAD batches, and 4K with static bands only (ME_DYN=0).
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04j_pytest_gpu.log 2>&1
SIZED=1 bash tools/profile.sh r04j_4k_sad --config 4k --cost sad --steps 6 --warmup 2 --no-cpu --no-stream --no-4k --no-single --no-ssd > gpurun_out/r04j_prof4k.log 2>&1
ME_HIP_LIB=libme_hip_tune.so ME_DYN=0 PMC_KEY_SUFFIX=_dyn0 SIZED=1 bash tools/profile.sh r04j_4k_sad_dyn0 --config 4k --cost sad --steps 6 --warmup 2 --no-cpu --no-stream --no-4k --no-single --no-ssd > gpurun_out/r04j_prof4k_dyn0.log 2>&1
SIZED=1 bash tools/profile.sh r04j_8k_sad --config 8k --cost sad --steps 3 --warmup 1 --no-cpu --no-stream --no-4k --no-single --no-ssd > gpurun_out/r04j_prof8k.log 2>&1
