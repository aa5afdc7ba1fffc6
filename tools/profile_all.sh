# Profile the six BASELINE workloads (one frame per step, so every per-launch
# figure is per frame) and the default bench line on the GPU box:
#   bash tools/profile_all.sh <tag>
set -e
TAG=${1:-r01}
bash tools/profile.sh ${TAG}_1080p_sad --steps 20 --warmup 3 --no-cpu --no-stream --no-4k --no-ssd --frames-per-step 1 > gpurun_out/prof1.txt 2>&1
bash tools/profile.sh ${TAG}_1080p_ssd --steps 20 --warmup 3 --no-cpu --no-stream --no-4k --cost ssd --frames-per-step 1 > gpurun_out/prof2.txt 2>&1
bash tools/profile.sh ${TAG}_4k_sad --steps 10 --warmup 2 --no-cpu --no-stream --no-4k --no-ssd --config 4k --frames-per-step 1 > gpurun_out/prof3.txt 2>&1
bash tools/profile.sh ${TAG}_8k_sad --steps 3 --warmup 1 --no-cpu --no-stream --no-4k --no-ssd --config 8k --frames-per-step 1 > gpurun_out/prof4.txt 2>&1
bash tools/profile.sh ${TAG}_4k_ssd --steps 10 --warmup 2 --no-cpu --no-stream --no-4k --cost ssd --config 4k --frames-per-step 1 > gpurun_out/prof5.txt 2>&1
bash tools/profile.sh ${TAG}_8k_ssd --steps 3 --warmup 1 --no-cpu --no-stream --no-4k --cost ssd --config 8k --frames-per-step 1 > gpurun_out/prof6.txt 2>&1
timeout -k 10 400 python bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err
cat gpurun_out/bench_${TAG}.json
