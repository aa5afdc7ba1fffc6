set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/plan_sweep.py --width 7680 --height 4320 --blk 8 --span 128 --iters 5 --plans "26,8,1,256,1;13,8,0,256,1" > gpurun_out/r03as_plan_8k.jsonl 2>&1
cat gpurun_out/r03as_plan_8k.jsonl
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03as_pytest_gpu.log 2>&1
tail -2 gpurun_out/r03as_pytest_gpu.log
