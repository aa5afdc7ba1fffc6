# Round 6: (1) pair pipeline, adjacent frames in one upload (slot chunks), and
# 16-pair batches (tuning build) -- host_stream A/B against the previous
# commit + a 64-pair trace; (2) SSIM plane prefetch two tiles ahead and the
# 16x16 statistics four positions per thread in two packed chains -- A/B.
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_ssim.py tests/test_gpu_fuzz.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06w_pytest.log 2>&1
O=gpurun_out/r06w_stream_ab.jsonl
: > $O
for rep in 1 2 3; do
  for lib in prev cur g16; do
    L=libme_hip_$lib.so; E=; [ $lib = cur ] && L=libme_hip.so; [ $lib = g16 ] && L=libme_hip_tune.so && E=ME_STREAM_BATCH=16
    env $E ME_HIP_LIB=$L timeout -k 10 180 python3 bench.py --no-cpu --no-4k --no-single --no-ssd --no-ssim --steps 5 --warmup 1 2>>gpurun_out/r06w_err.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); s=d['host_stream']
print(json.dumps({'tag': '$lib', 'pinned': s['pinned']['pairs_per_s'], 'pageable': s['pageable']['pairs_per_s'], 'batched': s['kernel_only_batched_pairs_per_s'], 'parity': s['parity']['ok']}))" >> $O
  done
done
O=gpurun_out/r06w_ssim_ab.jsonl
: > $O
for rep in 1 2; do
  for lib in prev cur; do
    L=libme_hip_$lib.so; [ $lib = cur ] && L=libme_hip.so
    ME_HIP_LIB=$L timeout -k 10 180 python3 bench.py --no-cpu --no-stream --no-4k --no-single --no-ssd --steps 10 --warmup 2 2>>gpurun_out/r06w_err.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); s=d['ssim']
print(json.dumps({'tag': '$lib', 'kernel_ms': s['kernel_ms'], 'parity': s['parity']['ok']}))" >> $O
  done
done
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r06w_stream -o run -- python3 tools/dbg/stream_trace.py 64 > gpurun_out/r06w_trace.log 2>&1
