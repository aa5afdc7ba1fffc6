# SSIM statistics prepass with LDS tiles: SSIM parity and the 1080p timing
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ssim.py tests/test_gpu_fuzz.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03bb_ssim_parity.log 2>&1
tail -2 gpurun_out/r03bb_ssim_parity.log
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r03bb_ssim_kt -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --cost ssim --steps 5 --warmup 1 --no-cpu --no-stream --no-4k --no-single --frames-per-step 1 > $GRAFT_REPO_ROOT/gpurun_out/r03bb_ssim_bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/r03bb_ssim_bench.err)
cut -c1-300 gpurun_out/r03bb_ssim_bench.json
find gpurun_out/r03bb_ssim_kt -name "*kernel_stats.csv" -exec cat {} \;
