# Round 6: one-box A/B of the 8x8 SSD switches (ME_SSD8_TAB / ME_SSD8_PIPE)
# and the SSIM switches (ME_SSIM_Q16 / _W0 / _FIT) against the round-5 library.
set -e
mkdir -p gpurun_out
O=gpurun_out/r06k_ssd8_ab.jsonl
: > $O
for rep in 1 2; do
  for lib in r5 cur tab0 pipe0 none; do
    L=libme_hip_$lib.so; [ $lib = cur ] && L=libme_hip.so
    ME_HIP_LIB=$L timeout -k 10 180 python3 tools/search_time.py --configs 8k --costs ssd --ms 400 --tag $lib >> $O 2>>gpurun_out/r06k_err.log
  done
done
O=gpurun_out/r06k_ssim_ab.jsonl
: > $O
for rep in 1 2; do
  for lib in r5 cur s12 s12w0 s12fit s14fit; do
    L=libme_hip_$lib.so; [ $lib = cur ] && L=libme_hip.so
    ME_HIP_LIB=$L timeout -k 10 180 python3 bench.py --no-cpu --no-stream --no-4k --no-single --no-ssd --steps 10 --warmup 2 2>>gpurun_out/r06k_err.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); s=d['ssim']
print(json.dumps({'tag': '$lib', 'kernel_ms': s['kernel_ms'], 'frac': s['roofline']['frac'], 'parity': s['parity']['ok']}))" >> $O
  done
done
