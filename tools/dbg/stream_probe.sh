#!/bin/bash
# Streams of one RCCL stripe rank: a one-rank
# torch.distributed.run of bench.py in stripe mode with the HIP runtime's own
# API log (AMD_LOG_LEVEL=3) on stderr; tools/dbg/stream_probe.py counts the
# stream creations (torch's pool, RCCL's internal streams, the library's).
# Usage (GPU box, repo root): tools/dbg/stream_probe.sh <tag>
TAG=${1:-r05a}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export AMD_LOG_LEVEL=${LEVEL:-3}
timeout -k 10 180 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=1 \
  --master-addr=127.0.0.1 --master-port=29561 bench.py --mode stripe --steps 3 --warmup 1 \
  --no-cpu --no-4k --ramp-ms 5 > "$OUT/stripe_rank.out" 2> "$OUT/stripe_rank.log"
rc=$?
grep -c "" "$OUT/stripe_rank.log"
grep -o "hipStreamCreate[A-Za-z]*\|hipExtStreamCreate[A-Za-z]*" "$OUT/stripe_rank.log" | sort | uniq -c
exit $rc
