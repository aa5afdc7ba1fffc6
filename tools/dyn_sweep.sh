#!/bin/bash
# Kernel time vs the dynamic-scheduling threshold (ME_DYN = tiles per workgroup
# from which tiles are pulled dynamically; 0 = static bands).
cd "$(dirname "$0")/.."
export ME_HIP_LIB=libme_hip_tune.so  # ME_DYN is read by the tuning build only
for d in 0 1 2 4 8; do
  for c in "--heights 1080" "--width 3840 --heights 2160 --span 64" "--width 7680 --heights 4320 --blk 8 --span 128 --iters 5"; do
    echo "{\"dyn\": $d, \"case\": \"$c\"}"
    ME_DYN=$d timeout -k 10 120 python3 tools/size_sweep.py --cost sad $c 2>/dev/null | grep '^{'
  done
done
