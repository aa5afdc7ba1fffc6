#!/bin/bash
# Round 4: where the 4K item kernel's extra L2 misses come from -- XCD
# placement of its workgroups (stamps build) and read bytes per plan variant.
set -e
mkdir -p gpurun_out
timeout -k 10 120 python3 tools/wave_stamps.py 4k > gpurun_out/r04k_stamps_4k.txt 2>&1
VARIANTS="none;ME_DYN=0;ME_PRIO=0;ME_PLAN=13,8,10,256,1;ME_PLAN=13,4,4,256,1;ME_PLAN=13,8,4,1024,1;ME_PLAN=13,8,2,256,1" \
  bash tools/dbg/pmc_variants.sh r04k_4k --config 4k --cost sad --steps 4 --warmup 1 --no-cpu --no-stream --no-4k --no-single --no-ssd > gpurun_out/r04k_variants_4k.txt 2>&1
