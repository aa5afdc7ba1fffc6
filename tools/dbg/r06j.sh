# Round 6: 8x8 SSD with the position term precomputed in the S2 table and
# the MFMAs one step ahead of their keys; SSIM workgroups sized to one round
# of lane-tasks, the block statistics on one wave -- tests, then one-box A/B
# against the round-5 library.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ssim.py tests/test_gpu_fullframe.py tests/test_gpu_mfma.py -x -q --timeout 300 --timeout-method thread -k "ssim or 8k or b8 or 8x8 or ssd8" > gpurun_out/r06j_pytest.log 2>&1
O=gpurun_out/r06j_ab.jsonl
: > $O
for rep in 1 2; do
  for lib in libme_hip_r5.so libme_hip.so; do
    ME_HIP_LIB=$lib timeout -k 10 180 python3 tools/search_time.py --configs 8k --costs ssd --ms 500 --tag $lib >> $O 2>>gpurun_out/r06j_err.log
    ME_HIP_LIB=$lib timeout -k 10 180 python3 bench.py --no-cpu --no-stream --no-4k --no-single --no-ssd --steps 10 --warmup 2 > gpurun_out/r06j_bench_${lib}_$rep.json 2>>gpurun_out/r06j_err.log
  done
done
