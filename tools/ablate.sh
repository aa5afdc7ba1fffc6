#!/bin/bash
# Time the fast kernel with parts removed (diagnostic builds, wrong results by
# design): abl1 = no epilogue, abl2 = xor instead of qsad, abl3 = no key atomics.
# usage (GPU box): bash tools/ablate.sh  -> gpurun_out/ablate.jsonl
set -e
cd "$(dirname "$0")/.."
out=gpurun_out/ablate.jsonl
mkdir -p gpurun_out
: > $out
for lib in libme_hip.so libme_hip_abl1.so libme_hip_abl2.so libme_hip_abl3.so; do
  for cost in sad ssd; do
    echo "{\"lib\": \"$lib\", \"cost\": \"$cost\"}" >> $out
    ME_HIP_LIB=$lib timeout -k 10 120 python3 tools/size_sweep.py --cost $cost --heights 1080,4320 --iters 50 2>/dev/null | grep '^{' >> $out
  done
done
cat $out
