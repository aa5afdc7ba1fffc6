# Block-major SSD kernel ablations (diagnostic builds, timing only):
# abl1 no S2 loads, abl2 no key epilogue, abl3 a quarter of the B-fragment LDS reads
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_LIBS="libme_hip.so libme_hip_abl1.so libme_hip_abl2.so libme_hip_abl3.so" bash tools/dbg/ab.sh > gpurun_out/r03au_abl_1080p.txt 2>&1
cat gpurun_out/r03au_abl_1080p.txt
AB_LIBS="libme_hip.so libme_hip_abl1.so libme_hip_abl2.so libme_hip_abl3.so" SWEEP_ARGS="--cost ssd --width 3840 --heights 2160 --span 64 --iters 10" bash tools/dbg/ab.sh > gpurun_out/r03au_abl_4k.txt 2>&1
cat gpurun_out/r03au_abl_4k.txt
