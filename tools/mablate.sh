#!/bin/bash
# Time the MFMA SSD path with parts removed (diagnostic builds, wrong results
# by design).  mablN, N a bit set: 1 no S2 loads, 2 epilogue cut to one min,
# 4 only the first chunk staged, 8 prepass staging only, 16 prepass without
# box sums, 32 no fragment loads, 64 no MFMA.
# usage (GPU box): bash tools/mablate.sh -> per-kernel averages per build
set -e
cd "$(dirname "$0")/.."
R=$(pwd)
out=$R/gpurun_out/mablate.txt
mkdir -p gpurun_out
: > $out
export TMPDIR=/tmp
for lib in libme_hip.so $(cd motionestimation_amd/lib && ls libme_hip_mabl*.so libme_hip_mdly*.so); do
  d=$R/gpurun_out/mabl_$lib
  (cd /tmp && ME_HIP_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- python3 $R/tools/size_sweep.py ${SWEEP_ARGS:---cost ssd --heights 1080 --iters 50} > $d.log 2>&1)
  echo "== $lib" >> $out
  find $d -name "*kernel_stats.csv" | xargs cat | awk -F'","' 'NR>1{printf "%-40s %s\n", substr($1,1,40), $4}' >> $out
done
cat $out
