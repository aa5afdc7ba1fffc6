set -e
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "split or flow or fast_sad or stripe or ties" > gpurun_out/r03i_parity.log 2>&1
timeout -k 10 100 python -u tools/stripe_sweep.py --config 1080p --ranks 1,2,4,8 > gpurun_out/r03i_sweep.jsonl
for KK in 5 4 13; do
ME_HIP_LIB=libme_hip_tune.so ME_PLAN=$KK,0,0,0 timeout -k 10 100 python -u tools/stripe_sweep.py --config 1080p --ranks 4,8 | sed "s/^/{\"K\": $KK, \"r\": /; s/$/}/" >> gpurun_out/r03i_sweep_k.jsonl
done
FLOW_STAMPS_SAVE=gpurun_out/r03i_flow_9_17.npy timeout -k 10 100 python -u tools/flow_stamps.py 9:17 > gpurun_out/r03i_flow_stamps.txt 2>&1
