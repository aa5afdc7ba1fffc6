# Final-build profile set: the six BASELINE workloads (16 frames per step), 1080p SAD one frame per step, default bench
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/profile_all.sh r03bh
