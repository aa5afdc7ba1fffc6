set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
C="--no-cpu --no-stream --no-4k --no-single"
bash tools/profile.sh r03ap_1080p_ssd --steps 20 --warmup 3 $C --cost ssd > gpurun_out/prof2.txt 2>&1
bash tools/profile.sh r03ap_4k_ssd --steps 4 --warmup 1 $C --cost ssd --config 4k > gpurun_out/prof5.txt 2>&1
timeout -k 10 400 python bench.py > gpurun_out/r03ap_bench.json 2> gpurun_out/r03ap_bench.err
python -c "import json;d=json.load(open('gpurun_out/r03ap_bench.json'));print(d['value'],d['kernel_ms'],d['roofline']['valu']['frac'],d['ssd_mfma'])"
