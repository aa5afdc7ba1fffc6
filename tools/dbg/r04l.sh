#!/bin/bash
# Round 4: item kernel claiming one tile ahead (tiles with >= 2 passes) --
# GPU suite, then read bytes / time at 4K +-64 and 8K 8x8 +-128 SAD against the
# two-ahead claim (ME_AHEAD=2) and a 512-thread plan.
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04l_pytest_gpu.log 2>&1
VARIANTS="none;ME_AHEAD=2;ME_PLAN=13,8,4,512,1;ME_PLAN=13,8,4,512,1 ME_AHEAD=2" \
  bash tools/dbg/pmc_variants.sh r04l_4k --config 4k --cost sad --steps 4 --warmup 1 --no-cpu --no-stream --no-4k --no-single --no-ssd > gpurun_out/r04l_variants_4k.txt 2>&1
VARIANTS="none;ME_AHEAD=2" \
  bash tools/dbg/pmc_variants.sh r04l_8k --config 8k --cost sad --steps 1 --warmup 0 --no-cpu --no-stream --no-4k --no-single --no-ssd > gpurun_out/r04l_variants_8k.txt 2>&1
