# SSIM search variants, one box: product (16x16 rows in registers, 6 candidates per lane),
# ssim8 (the same with 8), ssim0 (the generic plane path, 8 per lane, x loop rolled)
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_LIBS="libme_hip.so libme_hip_ssim8.so libme_hip_ssim0.so" SWEEP_ARGS="--cost ssim --heights 1080 --iters 10" bash tools/dbg/ab.sh > gpurun_out/r03bc_ssim_ab.txt 2>&1
cat gpurun_out/r03bc_ssim_ab.txt
