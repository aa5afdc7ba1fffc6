# SSIM 16x16 rows in registers, 12 candidates per lane (product) vs 10: parity, then A/B on one box
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ssim.py tests/test_gpu_fuzz.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03be_ssim_parity.log 2>&1
tail -2 gpurun_out/r03be_ssim_parity.log
AB_LIBS="libme_hip.so libme_hip_ssim10.so" SWEEP_ARGS="--cost ssim --heights 1080 --iters 10" bash tools/dbg/ab.sh > gpurun_out/r03be_ssim_ab.txt 2>&1
cat gpurun_out/r03be_ssim_ab.txt
