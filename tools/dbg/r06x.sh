# Round 6: pair pipeline batch-size sweep after the ramp (tuning build,
# ME_STREAM_BATCH = 8 / 12 / 16 / 24 / 32) with one-ahead uploads and merged copies.
set -e
mkdir -p gpurun_out
O=gpurun_out/r06x_stream_batch.jsonl
: > $O
for rep in 1 2; do
  for g in 8 12 16 24 32; do
    ME_STREAM_BATCH=$g ME_HIP_LIB=libme_hip_tune.so timeout -k 10 180 python3 bench.py --no-cpu --no-4k --no-single --no-ssd --no-ssim --steps 5 --warmup 1 2>>gpurun_out/r06x_err.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); s=d['host_stream']
print(json.dumps({'G': $g, 'pinned': s['pinned']['pairs_per_s'], 'pageable': s['pageable']['pairs_per_s'], 'batched': s['kernel_only_batched_pairs_per_s'], 'parity': s['parity']['ok']}))" >> $O
  done
done
