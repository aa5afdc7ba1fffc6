set -e
mkdir -p gpurun_out
FLOW_STAMPS_SAVE=gpurun_out/r03n_flow_single.npy timeout -k 10 100 python -u tools/flow_stamps.py > gpurun_out/r03n_flow_stamps.txt 2>&1
FLOW_STAMPS_SAVE=gpurun_out/r03n_flow_batch8.npy timeout -k 10 100 python -u tools/flow_stamps.py batch8 >> gpurun_out/r03n_flow_stamps.txt 2>&1
