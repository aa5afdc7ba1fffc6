set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullframe.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "8k or 4k or fast_sad" > gpurun_out/r03r_parity.log 2>&1
for S in 16 0; do
  ME_HIP_LIB=libme_hip_tune.so ME_STRIP=$S timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r03r_fetch_8k_s$S -o run --output-format csv -- python3 tools/dbg/traffic_probe.py 8k sad 2 > /dev/null 2>&1
  ME_HIP_LIB=libme_hip_tune.so ME_STRIP=$S timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r03r_fetch_4k_s$S -o run --output-format csv -- python3 tools/dbg/traffic_probe.py 4k sad 3 > /dev/null 2>&1
  ME_HIP_LIB=libme_hip_tune.so ME_STRIP=$S timeout -k 10 200 python -u tools/stripe_sweep.py --config 8k --ranks 1 --iters 5 >> gpurun_out/r03r_time_s$S.jsonl
  ME_HIP_LIB=libme_hip_tune.so ME_STRIP=$S timeout -k 10 200 python -u tools/stripe_sweep.py --config 4k --ranks 1 --iters 10 >> gpurun_out/r03r_time_s$S.jsonl
done
