# SSIM 16x16 lane layouts, one box: product (12 per lane, 256 threads: 2 rounds of 390 groups),
# 13 per lane x 384 threads (325 groups, one round), 17 per lane x 320 threads (260 groups, one round)
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_LIBS="libme_hip.so libme_hip_ssim13.so libme_hip_ssim17.so" SWEEP_ARGS="--cost ssim --heights 1080 --iters 10" bash tools/dbg/ab.sh > gpurun_out/r03bg_ssim_ab.txt 2>&1
cat gpurun_out/r03bg_ssim_ab.txt
