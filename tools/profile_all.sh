set -e
bash tools/profile.sh r01i_1080p_sad --steps 20 --warmup 3 --no-cpu --no-stream > gpurun_out/prof1.txt 2>&1
bash tools/profile.sh r01i_1080p_ssd --steps 20 --warmup 3 --no-cpu --no-stream --cost ssd > gpurun_out/prof2.txt 2>&1
bash tools/profile.sh r01i_4k_sad --steps 10 --warmup 2 --no-cpu --no-stream --config 4k > gpurun_out/prof3.txt 2>&1
bash tools/profile.sh r01i_8k_sad --steps 3 --warmup 1 --no-cpu --no-stream --config 8k > gpurun_out/prof4.txt 2>&1
timeout -k 10 400 python bench.py > gpurun_out/bench_r1i.json 2> gpurun_out/bench_r1i.err
cat gpurun_out/bench_r1i.json
