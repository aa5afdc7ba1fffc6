# 8K frames of a batch launch one by one: job-table parity, then the 16-frame 8K SAD profile
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "job or batch or stripes" > gpurun_out/r03ax_parity.log 2>&1
tail -2 gpurun_out/r03ax_parity.log
bash tools/profile.sh r03ax_8k_sad --steps 2 --warmup 1 --no-cpu --no-stream --no-4k --no-single --no-ssd --config 8k > gpurun_out/r03ax_prof8k.txt 2>&1
tail -4 gpurun_out/r03ax_prof8k.txt
timeout -k 10 300 python bench.py --config 8k --steps 2 --warmup 1 --no-cpu --no-stream --no-4k --no-single --no-ssd > gpurun_out/r03ax_bench8k.json 2> gpurun_out/r03ax_bench8k.err
cat gpurun_out/r03ax_bench8k.json
