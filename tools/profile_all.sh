# Profile the six BASELINE workloads as bench.py runs them (16 frames per step),
# the 1080p SAD and the 1080p / 4K SSD searches one frame per launch (the
# bench's single_frame / ssd_single_frame legs read their traffic from these),
# the 8K 8x8 SSD with the SQ instruction pass (its valu figure), then the
# default bench line, on the GPU box:
#   bash tools/profile_all.sh <tag> [part: 1 | 2 | all]
# (the single_frame / ssd / stripe_4k / stream legs are off in the profiled
# runs, so each kernel's launches are the timed workload's own)
set -e
TAG=${1:-r01}
PART=${2:-all}
C="--no-cpu --no-stream --no-4k --no-single --no-ssim"
if [ $PART != 2 ]; then
bash tools/profile.sh ${TAG}_1080p_sad --steps 20 --warmup 3 $C --no-ssd > gpurun_out/prof1.txt 2>&1
bash tools/profile.sh ${TAG}_1080p_ssd --steps 20 --warmup 3 $C --cost ssd > gpurun_out/prof2.txt 2>&1
bash tools/profile.sh ${TAG}_4k_sad --steps 4 --warmup 1 $C --no-ssd --config 4k > gpurun_out/prof3.txt 2>&1
bash tools/profile.sh ${TAG}_8k_sad --steps 2 --warmup 1 $C --no-ssd --config 8k > gpurun_out/prof4.txt 2>&1
bash tools/profile.sh ${TAG}_4k_ssd --steps 4 --warmup 1 $C --cost ssd --config 4k > gpurun_out/prof5.txt 2>&1
fi
if [ $PART != 1 ]; then
VALU=1 bash tools/profile.sh ${TAG}_8k_ssd --steps 2 --warmup 1 $C --cost ssd --config 8k > gpurun_out/prof6.txt 2>&1
bash tools/profile.sh ${TAG}_1080p_sad_f1 --steps 20 --warmup 3 $C --no-ssd --frames-per-step 1 > gpurun_out/prof7.txt 2>&1
bash tools/profile.sh ${TAG}_1080p_ssd_f1 --steps 20 --warmup 3 $C --cost ssd --frames-per-step 1 > gpurun_out/prof8.txt 2>&1
bash tools/profile.sh ${TAG}_4k_ssd_f1 --steps 8 --warmup 2 $C --cost ssd --config 4k --frames-per-step 1 > gpurun_out/prof9.txt 2>&1
timeout -k 10 400 python bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err
cat gpurun_out/bench_${TAG}.json
fi
