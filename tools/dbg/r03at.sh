set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03at_pytest_gpu.log 2>&1
tail -2 gpurun_out/r03at_pytest_gpu.log
bash tools/profile.sh r03at_8k_sad --steps 2 --warmup 1 --no-cpu --no-stream --no-4k --no-single --no-ssd --config 8k > gpurun_out/r03at_prof8k.txt 2>&1
tail -3 gpurun_out/r03at_prof8k.txt
timeout -k 10 400 python bench.py > gpurun_out/r03at_bench.json 2> gpurun_out/r03at_bench.err
cat gpurun_out/r03at_bench.json
