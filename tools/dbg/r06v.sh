# Round 6: pair pipeline, adjacent frames in one upload (slot chunks) --
# stream tests, host_stream A/B (previous commit / this build), and a kernel +
# copy + HIP API trace of a 64-pair pinned run (tools/stream_gaps.py).
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06v_pytest.log 2>&1
O=gpurun_out/r06v_stream_ab.jsonl
: > $O
for rep in 1 2 3; do
  for lib in prev cur g16; do
    L=libme_hip_$lib.so; E=; [ $lib = cur ] && L=libme_hip.so; [ $lib = g16 ] && L=libme_hip_tune.so && E=ME_STREAM_BATCH=16
    env $E ME_HIP_LIB=$L timeout -k 10 180 python3 bench.py --no-cpu --no-4k --no-single --no-ssd --no-ssim --steps 5 --warmup 1 2>>gpurun_out/r06v_err.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); s=d['host_stream']
print(json.dumps({'tag': '$lib', 'pinned': s['pinned']['pairs_per_s'], 'pageable': s['pageable']['pairs_per_s'], 'batched': s['kernel_only_batched_pairs_per_s'], 'parity': s['parity']['ok']}))" >> $O
  done
done
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r06v_stream -o run -- python3 tools/dbg/stream_trace.py 64 > gpurun_out/r06v_trace.log 2>&1
