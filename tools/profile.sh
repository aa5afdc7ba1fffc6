#!/bin/bash
# Profile the bench workload on the GPU box (run from the repo root):
#   tools/profile.sh <tag> [bench args...]
# 1) rocprofv3 --kernel-trace --stats  (per-kernel durations)
# 2) rocprofv3 --pmc FETCH_SIZE        (own pass: TCC slots, MI355X_MICROARCH.md)
# 3) rocprofv3 --pmc WRITE_SIZE        (own pass)
# 4) SIZED=1: the L2's fabric read requests by size (32/64/128 B) and the L2
#    hit/miss counts, two more passes (FETCH_SIZE is requests x 64 B, so the
#    doubling of MI355X_MICROARCH.md holds only if every request is 128 B)
# 5) VALU=1: SQ instruction counts, one more pass (below)
# then tools/pmc_summary.py folds them into profiles/pmc_summary.json and
# copies the stats CSVs to profiles/<tag>_*.
set -o pipefail
TAG=${1:-r01}
shift
ARGS=${@:---steps 20 --warmup 3 --no-cpu --no-stream --no-4k}
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d "$OUT/kt" -o run --output-format csv -- python3 bench.py $ARGS > "$OUT/kt.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T -d "$OUT/fetch" -o run --output-format csv -- python3 bench.py $ARGS > "$OUT/fetch.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T -d "$OUT/write" -o run --output-format csv -- python3 bench.py $ARGS > "$OUT/write.log" 2>&1 || exit $?
if [ "${SIZED:-0}" = 1 ]; then
  timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum -T -d "$OUT/rdreq" -o run --output-format csv -- python3 bench.py $ARGS > "$OUT/rdreq.log" 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -T -d "$OUT/hit" -o run --output-format csv -- python3 bench.py $ARGS > "$OUT/hit.log" 2>&1 || exit $?
fi
# 5) VALU=1: wave-level instruction counts of every kernel (VALU incl. MFMA,
#    MFMA, SALU) and waves -- the 8x8 SSD line's valu figure (bench.py)
if [ "${VALU:-0}" = 1 ]; then
  timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_WAVES -T -d "$OUT/valu" -o run --output-format csv -- python3 bench.py $ARGS > "$OUT/valu.log" 2>&1 || exit $?
fi
find "$OUT" -name "*.csv" | head -50
python3 tools/pmc_summary.py "$OUT" "$TAG" $ARGS
