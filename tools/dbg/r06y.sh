# Round 6: full GPU suite on this build, then the stream A/B against the
# previous commit (pinned / pageable pairs/s), then the default bench line.
set -e
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06y_pytest.log 2>&1
O=gpurun_out/r06y_stream_ab.jsonl
: > $O
for rep in 1 2 3; do
  for lib in prev cur; do
    L=libme_hip_$lib.so; [ $lib = cur ] && L=libme_hip.so
    ME_HIP_LIB=$L timeout -k 10 180 python3 bench.py --no-cpu --no-4k --no-single --no-ssd --no-ssim --steps 5 --warmup 1 2>>gpurun_out/r06y_err.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); s=d['host_stream']
print(json.dumps({'tag': '$lib', 'pinned': s['pinned']['pairs_per_s'], 'pageable': s['pageable']['pairs_per_s'], 'batched': s['kernel_only_batched_pairs_per_s'], 'parity': s['parity']['ok']}))" >> $O
  done
done
timeout -k 10 400 python3 bench.py > gpurun_out/r06y_bench.json 2> gpurun_out/r06y_bench.err
