set -e
mkdir -p gpurun_out
ITERS=100 bash tools/sq_counters.sh sad me_flow > gpurun_out/r03x_sq.txt 2>&1
