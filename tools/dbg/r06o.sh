# Round 6: SSIM statistics in one launch, packed plane stats -- SSIM tests, bench
# SSIM leg A/B (previous commit's library, this build), kernel trace of the leg.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ssim.py tests/test_gpu_fuzz.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06o_pytest.log 2>&1
O=gpurun_out/r06o_ssim_ab.jsonl
: > $O
for rep in 1 2; do
  for lib in prev cur; do
    L=libme_hip_$lib.so; [ $lib = cur ] && L=libme_hip.so
    ME_HIP_LIB=$L timeout -k 10 180 python3 bench.py --no-cpu --no-stream --no-4k --no-single --no-ssd --steps 10 --warmup 2 2>>gpurun_out/r06o_err.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); s=d['ssim']
print(json.dumps({'tag': '$lib', 'kernel_ms': s['kernel_ms'], 'frac': s['roofline']['frac'], 'parity': s['parity']['ok']}))" >> $O
  done
done
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r06o_ssim -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --no-stream --no-4k --no-single --no-ssd --steps 10 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/r06o_prof.log 2>&1
