set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/plan_sweep.py --width 7680 --height 4320 --blk 8 --span 128 --iters 5 --plans "26,8,1,256,1;26,10,1,256,1;26,6,1,256,1;26,12,1,256,1;26,16,1,256,1;13,8,0,256,1" > gpurun_out/r03ar_plan_8k.jsonl 2>&1
timeout -k 10 300 python -u tools/plan_sweep.py --width 7680 --height 4320 --blk 8 --span 128 --iters 5 --plans "26,10,1,256,1" >> gpurun_out/r03ar_plan_8k.jsonl 2>&1
cat gpurun_out/r03ar_plan_8k.jsonl
