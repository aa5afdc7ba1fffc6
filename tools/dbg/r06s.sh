# Round 6: (1) SSIM packed score epilogue + XCD-ordered blocks, (2) pair
# pipeline with uploads one batch ahead (no wait packet when they landed).
# GPU tests, then A/B: SSIM leg (previous commit / XCD + scalar epilogue /
# this build) and host_stream leg (previous commit / this build), alternating.
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_ssim.py tests/test_gpu_fuzz.py tests/test_gpu_stream.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06s_pytest.log 2>&1
O=gpurun_out/r06s_ssim_ab.jsonl
: > $O
for rep in 1 2; do
  for lib in prev oldep cur; do
    L=libme_hip_$lib.so; [ $lib = cur ] && L=libme_hip.so
    ME_HIP_LIB=$L timeout -k 10 180 python3 bench.py --no-cpu --no-stream --no-4k --no-single --no-ssd --steps 10 --warmup 2 2>>gpurun_out/r06s_err.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); s=d['ssim']
print(json.dumps({'tag': '$lib', 'kernel_ms': s['kernel_ms'], 'parity': s['parity']['ok']}))" >> $O
  done
done
O=gpurun_out/r06s_stream_ab.jsonl
: > $O
for rep in 1 2 3; do
  for lib in prev cur; do
    L=libme_hip_$lib.so; [ $lib = cur ] && L=libme_hip.so
    ME_HIP_LIB=$L timeout -k 10 180 python3 bench.py --no-cpu --no-4k --no-single --no-ssd --no-ssim --steps 5 --warmup 1 2>>gpurun_out/r06s_err.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); s=d['host_stream']
print(json.dumps({'tag': '$lib', 'pinned': s['pinned']['pairs_per_s'], 'pageable': s['pageable']['pairs_per_s'], 'batched': s['kernel_only_batched_pairs_per_s'], 'parity': s['parity']['ok']}))" >> $O
  done
done
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r06s_ssim -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --no-stream --no-4k --no-single --no-ssd --steps 10 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/r06s_prof.log 2>&1
