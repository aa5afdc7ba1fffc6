set -e
mkdir -p gpurun_out
SQ_ARGS="--blk 8 --span 128 --width 7680 --heights 4320" ITERS=3 bash tools/sq_counters.sh sad me_fast > gpurun_out/r03aq_sq_8k.txt 2>&1
cat gpurun_out/r03aq_sq_8k.txt
