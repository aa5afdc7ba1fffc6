# SSIM search variants, one box: product (8 candidates per lane, 256 threads), 12 and 16 per lane, 320 threads
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_LIBS="libme_hip.so libme_hip_ssim12.so libme_hip_ssim16.so libme_hip_ssim320.so" SWEEP_ARGS="--cost ssim --heights 1080 --iters 10" bash tools/dbg/ab.sh > gpurun_out/r03bd_ssim_ab.txt 2>&1
cat gpurun_out/r03bd_ssim_ab.txt
