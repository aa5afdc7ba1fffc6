# split-mode flow kernel: parity suite, then stripe sweeps with split on / off
set -e
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "split or flow or fast_sad or stripe or ties" > gpurun_out/r03e_parity.log 2>&1
timeout -k 10 100 python -u tools/stripe_sweep.py --config 1080p --ranks 1,2,4,8 > gpurun_out/r03e_sweep.jsonl
timeout -k 10 100 python -u tools/stripe_sweep.py --config 4k --ranks 1,8 >> gpurun_out/r03e_sweep.jsonl
ME_HIP_LIB=libme_hip_tune.so ME_FLOW=2 timeout -k 10 100 python -u tools/stripe_sweep.py --config 1080p --ranks 1,2,4,8 > gpurun_out/r03e_sweep_nosplit.jsonl
ME_HIP_LIB=libme_hip_tune.so ME_PLAN=13,0,0,0 timeout -k 10 100 python -u tools/stripe_sweep.py --config 1080p --ranks 4,8 > gpurun_out/r03e_sweep_k13.jsonl
timeout -k 10 100 python -u tools/step_overhead.py --steps 2000 > gpurun_out/r03e_step.jsonl 2>/dev/null
#timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03e_gpu.log 2>&1
