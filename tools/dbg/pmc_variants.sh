#!/bin/bash
# One rocprofv3 pass of L2 fabric read requests (128 B / 64 B) per tuning-build
# variant of a bench workload; prints per variant the batch launches' mean
# request bytes and duration (tools/dbg/pmc_variants.py).
#   VARIANTS="ME_DYN=0;ME_PLAN=13,4,4,256,1" tools/dbg/pmc_variants.sh <tag> <bench args>
# (COUNTERS="..." replaces the counter set: one pass, within the block limits)
set -e
TAG=$1; shift
OUT=gpurun_out/pmcvar_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
IFS=';' read -ra VS <<< "${VARIANTS:-none}"
i=0
for v in "${VS[@]}"; do
  envs=(ME_HIP_LIB=libme_hip_tune.so)
  [ "$v" != none ] && envs+=($v)
  env "${envs[@]}" timeout -k 10 240 rocprofv3 --pmc ${COUNTERS:-TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_HIT_sum TCC_MISS_sum} \
    -T -d $OUT/v$i -o run --output-format csv -- python3 bench.py "$@" > $OUT/v$i.log 2>&1
  echo "$v" > $OUT/v$i.variant
  i=$((i+1))
done
python3 tools/dbg/pmc_variants.py $OUT
