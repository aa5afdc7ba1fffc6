# Round 6: SSIM full 16x16 blocks on the matrix cores (exact integer cross
# variance) -- SSIM tests against the reference goldens and the oracle, then
# the bench's SSIM leg against the round-5 library on one box.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ssim.py tests/test_gpu_fuzz.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06l_pytest.log 2>&1
O=gpurun_out/r06l_ssim_ab.jsonl
: > $O
for rep in 1 2; do
  for lib in r5 cur; do
    L=libme_hip_$lib.so; [ $lib = cur ] && L=libme_hip.so
    ME_HIP_LIB=$L timeout -k 10 180 python3 bench.py --no-cpu --no-stream --no-4k --no-single --no-ssd --steps 10 --warmup 2 2>>gpurun_out/r06l_err.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); s=d['ssim']
print(json.dumps({'tag': '$lib', 'kernel_ms': s['kernel_ms'], 'frac': s['roofline']['frac'], 'parity': s['parity']['ok']}))" >> $O
  done
done
