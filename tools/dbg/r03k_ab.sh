set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 150 python -u tools/stripe_sweep.py --config 1080p --ranks 1 --frames 1 --iters 100 > gpurun_out/r03k_sweep.jsonl
timeout -k 10 150 python -u tools/stripe_sweep.py --config 1080p --ranks 1,8 --frames 8 >> gpurun_out/r03k_sweep.jsonl
timeout -k 10 200 python -u bench.py --no-cpu --no-stream --no-4k --frames-per-step 8 > gpurun_out/r03k_bench_f8.json 2>/dev/null
timeout -k 10 200 python -u bench.py --no-cpu --no-stream --no-4k --frames-per-step 1 > gpurun_out/r03k_bench_f1.json 2>/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d gpurun_out/r03k_prof -o run --output-format csv -- python3 bench.py --no-cpu --no-stream --no-4k --no-ssd --frames-per-step 8 --steps 20 > gpurun_out/r03k_prof.log 2>&1
