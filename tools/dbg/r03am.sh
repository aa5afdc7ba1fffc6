set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03am_pytest_gpu.log 2>&1
tail -2 gpurun_out/r03am_pytest_gpu.log
O=gpurun_out/r03am_ab.jsonl
for rep in 1 2; do
ME_HIP_LIB=libme_hip_tune.so AB_FRAMES=16 timeout -k 10 120 python -u tools/dbg/flow_fair_ab.py >> $O
ME_HIP_LIB=libme_hip_tune.so ME_FAIR=0 ME_FLOW_ONE=0 AB_FRAMES=16 timeout -k 10 120 python -u tools/dbg/flow_fair_ab.py >> $O
ME_HIP_LIB=libme_hip_tune.so ME_FAIR=3 AB_FRAMES=16 timeout -k 10 120 python -u tools/dbg/flow_fair_ab.py >> $O
done
cat $O
bash tools/profile.sh r03am_1080p_sad --steps 20 --warmup 3 --no-cpu --no-stream --no-4k --no-ssd --frames-per-step 1 > gpurun_out/prof1.txt 2>&1
bash tools/profile.sh r03am_1080p_sad16 --steps 20 --warmup 3 --no-cpu --no-stream --no-4k --no-ssd > gpurun_out/prof2.txt 2>&1
timeout -k 10 400 python bench.py > gpurun_out/r03am_bench.json 2> gpurun_out/r03am_bench.err
python -c "import json;d=json.load(open('gpurun_out/r03am_bench.json'));print(d['value'],d['kernel_ms'],d['roofline']['valu'],d['single_frame']['kernel_ms'],d['stripe_4k']['value'])"
