set -e
mkdir -p gpurun_out
FLOW_STAMPS_SAVE=gpurun_out/r03h_flow_9_17.npy timeout -k 10 100 python -u tools/flow_stamps.py 9:17 > /dev/null 2>&1
FLOW_STAMPS_SAVE=gpurun_out/r03h_flow_full.npy timeout -k 10 100 python -u tools/flow_stamps.py > /dev/null 2>&1
