# Profile the six BASELINE workloads as bench.py runs them (16 frames per step:
# a SAD launch holds all 16, an SSD search launches per frame), the 1080p SAD
# search one frame per launch, then the default bench line, on the GPU box:
#   bash tools/profile_all.sh <tag>
# (the single_frame / ssd / stripe_4k / stream legs are off in the profiled
# runs, so each kernel's launches are the timed workload's own)
set -e
TAG=${1:-r01}
C="--no-cpu --no-stream --no-4k --no-single --no-ssim"
bash tools/profile.sh ${TAG}_1080p_sad --steps 20 --warmup 3 $C --no-ssd > gpurun_out/prof1.txt 2>&1
bash tools/profile.sh ${TAG}_1080p_ssd --steps 20 --warmup 3 $C --cost ssd > gpurun_out/prof2.txt 2>&1
bash tools/profile.sh ${TAG}_4k_sad --steps 4 --warmup 1 $C --no-ssd --config 4k > gpurun_out/prof3.txt 2>&1
bash tools/profile.sh ${TAG}_8k_sad --steps 2 --warmup 1 $C --no-ssd --config 8k > gpurun_out/prof4.txt 2>&1
bash tools/profile.sh ${TAG}_4k_ssd --steps 4 --warmup 1 $C --cost ssd --config 4k > gpurun_out/prof5.txt 2>&1
bash tools/profile.sh ${TAG}_8k_ssd --steps 2 --warmup 1 $C --cost ssd --config 8k > gpurun_out/prof6.txt 2>&1
bash tools/profile.sh ${TAG}_1080p_sad_f1 --steps 20 --warmup 3 $C --no-ssd --frames-per-step 1 > gpurun_out/prof7.txt 2>&1
timeout -k 10 400 python bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err
cat gpurun_out/bench_${TAG}.json
