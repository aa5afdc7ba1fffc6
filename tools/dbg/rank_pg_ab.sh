#!/bin/bash
# One-rank RCCL stripe step (bench.py --mode stripe under torch.distributed.run)
# with torch's process group on gloo (default: one RCCL communicator per rank,
# the library's) and on nccl (round 4: a second communicator), interleaved
# twice; one JSON line per run -> gpurun_out/<tag>_rank_pg_ab.jsonl.
TAG=${1:-r05}
OUT=gpurun_out/${TAG}_rank_pg_ab.jsonl
: > "$OUT"
port=29571
for rep in 1 2; do
  for pg in gloo nccl; do
    port=$((port + 1))
    line=$(timeout -k 10 150 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=1 \
      --master-addr=127.0.0.1 --master-port=$port bench.py --mode stripe --steps 200 --warmup 10 \
      --no-cpu --no-4k --torch-pg $pg 2>/dev/null | grep '^{')
    rc=$?
    [ $rc -ne 0 ] && { echo "run $pg rc=$rc"; exit $rc; }
    python3 -c "
import json,sys; d=json.loads(sys.argv[1])
print(json.dumps({'torch_pg': sys.argv[2], 'rep': int(sys.argv[3]), 'ms_per_step': d['ms_per_step'],
                  'kernel_ms': d['kernel_ms'], 'parity': d['parity'], 'gather': d['config']['gather']}))" "$line" $pg $rep >> "$OUT"
  done
done
cat "$OUT"
